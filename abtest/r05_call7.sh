#!/usr/bin/env bash
# config 5: persistent cooperative record-group blocks, barrier every 1 / 4 / 16 items, vs RG 1
set -o pipefail
mkdir -p gpurun_out/ab
VARIANTS="cw2 rgn4 rgp1 rgp4 rgp16" STEPS=3 timeout -k 10 900 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
echo ALL_OK
