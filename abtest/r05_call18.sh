#!/usr/bin/env bash
# Values-before-symbolic check: the tile and RCCL tests, then the two-rank gloo rehearsal
# of bench.py's N>1 line (structure/values broadcast timings).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tiles.py tests/test_gpu_rccl.py > gpurun_out/r05_c18_tests.log 2>&1 || { tail -30 gpurun_out/r05_c18_tests.log; exit 1; }
tail -2 gpurun_out/r05_c18_tests.log
SPG_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 2 --warmup 1 --cpu-seconds 0 \
    --config5-n 131072 > gpurun_out/r05_rehearse2.json 2> gpurun_out/r05_rehearse2.err || { tail -30 gpurun_out/r05_rehearse2.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r05_rehearse2.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d.get("b_values_pipeline")))
print(json.dumps(d.get("config5", {}).get("b_values_pipeline")), d.get("config5", {}).get("ms_per_step"))
P
