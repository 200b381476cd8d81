#!/usr/bin/env bash
# 16-bit structure broadcast: kernel tests, tile/RCCL tests (the 2-rank rehearsal now has a
# B wider than 65536), then the default 2-rank gloo rehearsal of bench.py's N>1 line.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tiles.py tests/test_gpu_rccl.py > gpurun_out/r05_c19_tests.log 2>&1 || { tail -30 gpurun_out/r05_c19_tests.log; exit 1; }
tail -2 gpurun_out/r05_c19_tests.log
SPG_DIST_BACKEND=gloo timeout -k 10 700 python3 bench.py --gpus 2 --steps 3 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/r05_rehearse2_default.json 2> gpurun_out/r05_rehearse2_default.err || { tail -30 gpurun_out/r05_rehearse2_default.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r05_rehearse2_default.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d.get("b_values_pipeline")))
print(json.dumps(d.get("config5", {}).get("b_values_pipeline")), d.get("config5", {}).get("ms_per_step"))
P
