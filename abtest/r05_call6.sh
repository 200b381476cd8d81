#!/usr/bin/env bash
# k_tile_sym8 waves per task (shared bitmap): 1 / 2 / 4 on config 5
set -o pipefail
mkdir -p gpurun_out/ab
VARIANTS="cw1 cw2 cw4" STEPS=3 timeout -k 10 600 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
echo ALL_OK
