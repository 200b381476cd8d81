#!/usr/bin/env bash
# config 5: persistent RG 1 / 2 / 4 / 8 and the traffic of persistent RG 4; config 4: persistent
# grid and record groups of 2 dense tiles
set -o pipefail
mkdir -p gpurun_out/ab
VARIANTS="rg1p rgp2 rgp1 rgp8" STEPS=3 timeout -k 10 900 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
VARIANTS="dnb dnp dnrg2p" timeout -k 10 600 bash abtest/ab_c4.sh || { echo AB4_FAILED; exit 1; }
VARIANTS="rgp1" timeout -k 10 600 bash abtest/pmc_c5.sh || { echo PMC_FAILED; exit 1; }
echo ALL_OK
