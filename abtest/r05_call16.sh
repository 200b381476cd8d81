#!/usr/bin/env bash
# 6-byte fp32 records: fp32 parity, then fp32 timing (config 3 at 0.1 and 0.01, config-4-shaped)
set -o pipefail
mkdir -p gpurun_out/fp32
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tiles.py tests/test_gpu_lds_guard.py -k "f32 or fp32 or float32 or golden or random or guard or c64" > gpurun_out/r05_t16.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05_t16.log; exit 1; }
tail -1 gpurun_out/r05_t16.log
for sh in "8192 0.1" "8192 0.01" "65536 0.005"; do
  set -- $sh
  timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2 --n $1 --density $2 --steps 5 --warmup 2 > gpurun_out/fp32/r6_$1_$2.json 2>/dev/null || { echo B; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fp32/r6_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
done
echo ALL_OK
