#!/usr/bin/env bash
# Round profile collection for the three bench workloads (profiles/collect.sh each):
# config 2 (the N=1 headline, k_row), config 4 (ALG3 chunked, dense tiles) and config 5 on
# one GPU (sparse tiles).  ROUND names the outputs.
set -euo pipefail
R=${ROUND:-r02}
TAG=${R}_c2 PMC_KEY=c2_n16384_d0.001_float64_alg1_w1 PMC_KERNEL='k_row<double, int, int, 2' \
    BENCH_ARGS="" bash profiles/collect.sh
TAG=${R}_c4 PMC_KEY=c4_n65536_d0.005_float64_alg3_w1 PMC_KERNEL='k_tile<double, int, true' \
    BENCH_ARGS="--config 4 --steps 3 --warmup 1" bash profiles/collect.sh
TAG=${R}_c5 PMC_KEY=c5_n262144_d0.001_float64_alg2_w1 PMC_KERNEL='k_tile<double, int, false' \
    BENCH_ARGS="--config 5 --steps 3 --warmup 1" bash profiles/collect.sh
echo "all collected ($R)"
