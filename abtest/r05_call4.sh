#!/usr/bin/env bash
# ring walk: full GPU suite, then config 4 / config 5 / fp32 timing
set -o pipefail
mkdir -p gpurun_out/fp32
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05_t4.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05_t4.log; exit 1; }
tail -2 gpurun_out/r05_t4.log
timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 > gpurun_out/r05_c4_ring.json 2>/dev/null || { echo B4; exit 1; }
timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/r05_c5_ring.json 2>/dev/null || { echo B5; exit 1; }
timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2 --n 8192 --density 0.1 --steps 10 --warmup 2 > gpurun_out/fp32/ring_d0.1.json 2>/dev/null || { echo BF; exit 1; }
for f in r05_c4_ring r05_c5_ring fp32/ring_d0.1; do python3 -c "import json; d=json.load(open('gpurun_out/$f.json')); ph=d.get('phases_ms_per_step') or d['config'].get('phases_ms_per_step'); print('$f', d['value'], d['ms_per_step'], ph)"; done
echo ALL_OK
