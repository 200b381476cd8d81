#!/usr/bin/env bash
# fp32 entry runs (k_tile_dn<float>) parity + timing vs k_tile (SPG_F32_RUNS=0); config 5 record-group A/B
set -o pipefail
mkdir -p gpurun_out/ab gpurun_out/fp32
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fp32 or cooperative or random_bitexact or negative_zero or lds" > gpurun_out/r05_t3.log 2>&1 || { echo TESTS_FAILED; exit 1; }
A="--no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2 --n 8192 --density 0.1 --steps 10 --warmup 2"
timeout -k 10 300 python bench.py $A > gpurun_out/fp32/runs_d0.1.json 2>/dev/null || { echo F1; exit 1; }
SPG_F32_RUNS=0 timeout -k 10 300 python bench.py $A > gpurun_out/fp32/ktile_d0.1.json 2>/dev/null || { echo F2; exit 1; }
for f in runs_d0.1 ktile_d0.1; do python3 -c "import json; d=json.load(open('gpurun_out/fp32/$f.json')); print('$f', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"; done
bash abtest/r05_call2.sh || exit 1
echo ALL_OK
