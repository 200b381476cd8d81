#!/usr/bin/env bash
# Round-6 profile collection (gpurun, repo root): configs 4 (the headline), 2 and 5 through
# profiles/collect.sh -- bench line, rocprofv3 kernel trace + stats, FETCH_SIZE and WRITE_SIZE
# passes -- each stamped with the library's build and source ids.  WHICH narrows the set;
# 3f = config 3's fp32 shape at N = 8192, density 0.1 (against the same-run sgemm).
set -uo pipefail
for c in ${WHICH:-4 2 5}; do
  case $c in
    4) TAG=r06_c4 BENCH_ARGS="--no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 3 --warmup 1" PMC_KEY=c4_n65536_d0.005_float64_alg3_w1 \
         PMC_KERNEL="k_tile_dn<double, int" bash profiles/collect.sh || exit 1 ;;
    2) TAG=r06_c2 BENCH_ARGS="--config 2 --cpu-seconds 0" PMC_KEY=c2_n16384_d0.001_float64_alg1_w1 \
         PMC_KERNEL="k_row<double, int, int, 2" bash profiles/collect.sh || exit 1 ;;
    5) TAG=r06_c5 BENCH_ARGS="--config 5 --cpu-seconds 0 --steps 3 --warmup 1" PMC_KEY=c5_n262144_d0.001_float64_alg2_w1 \
         PMC_KERNEL="k_tile_sp<double, int" bash profiles/collect.sh || exit 1 ;;
    3f) TAG=r06_c3f32 BENCH_ARGS="--config 4 --n 8192 --density 0.1 --dtype float32 --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 10 --warmup 2" \
         PMC_KEY=c4_n8192_d0.1_float32_alg3_w1 PMC_KERNEL="k_tile_dn<float, int" bash profiles/collect.sh || exit 1 ;;
  esac
done
