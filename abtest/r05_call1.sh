#!/usr/bin/env bash
# round 5, first GPU call: focused parity (RCCL world 1, tile groups, tile-path cases), config 5
# with cooperative record groups (default) vs the one-wave kernel, config-4 tile-width A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_tiles.py tests/test_gpu_parity.py -k "rccl or tile or cooperative" > gpurun_out/r05_t1.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/r05_c5_rg4.json 2> gpurun_out/r05_c5_rg4.err || { echo BENCH1_FAILED; exit 1; }
SPG_SP_RECORD_GROUP=1 timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/r05_c5_rg1.json 2> gpurun_out/r05_c5_rg1.err || { echo BENCH2_FAILED; exit 1; }
SPG_SYM_COOP=0 timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/r05_c5_sym1.json 2> gpurun_out/r05_c5_sym1.err || { echo BENCH3_FAILED; exit 1; }
VARIANTS="base t10 t10d2 t11d2" timeout -k 10 400 bash abtest/ab_c4.sh > gpurun_out/r05_ab_c4.log 2>&1 || { echo AB_FAILED; exit 1; }
timeout -k 10 900 bash abtest/r05_fp32.sh > gpurun_out/r05_fp32.log 2>&1 || { echo FP32_FAILED; exit 1; }
echo ALL_OK
