#!/usr/bin/env bash
# config 5 symbolic: one row's 4 symbolic tiles per persistent block (sco4) vs shared-bitmap pairs (scw2)
set -o pipefail
mkdir -p gpurun_out/ab
VARIANTS="scw2 sco4" STEPS=3 timeout -k 10 600 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
VARIANTS="sco4" timeout -k 10 600 bash abtest/pmc_c5.sh || { echo PMC_FAILED; exit 1; }
echo ALL_OK
