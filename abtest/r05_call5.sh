#!/usr/bin/env bash
# symbolic early exit for full rows: parity + config-3 timing (fp32 and fp64 at density 0.1)
set -o pipefail
mkdir -p gpurun_out/fp32
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "random_bitexact or fp32 or dense or golden" > gpurun_out/r05_t5.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05_t5.log; exit 1; }
tail -1 gpurun_out/r05_t5.log
for dt in float32 float64; do
  timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype $dt --alg 2 --n 8192 --density 0.1 --steps 10 --warmup 2 > gpurun_out/fp32/exit_$dt.json 2>/dev/null || { echo B_$dt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/fp32/exit_$dt.json')); print('$dt', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
done
echo ALL_OK
