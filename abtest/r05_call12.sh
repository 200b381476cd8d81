#!/usr/bin/env bash
# config 5 RG 4: 8 vs 16 chunks per step (is the cooperative kernel latency-bound?)
set -o pipefail
VARIANTS="rgm16 rgm8 rgm16" STEPS=3 timeout -k 10 600 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
echo ALL_OK
