#!/usr/bin/env bash
# values_first switch: RCCL world-1 test (3 modes) + tile tests, then the 2-rank gloo
# rehearsal of the N=2 line (symbolic_hidden_ms).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_rccl.py tests/test_gpu_tiles.py > gpurun_out/r05_c22_tests.log 2>&1 || { tail -30 gpurun_out/r05_c22_tests.log; exit 1; }
tail -2 gpurun_out/r05_c22_tests.log
SPG_DIST_BACKEND=gloo timeout -k 10 800 python3 bench.py --gpus 2 --steps 3 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/r05_rehearse2_default.json 2> gpurun_out/r05_rehearse2_default.err || { tail -30 gpurun_out/r05_rehearse2_default.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r05_rehearse2_default.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d.get("b_values_pipeline")))
print(json.dumps(d.get("config5", {}).get("b_values_pipeline")), d.get("config5", {}).get("ms_per_step"))
P
