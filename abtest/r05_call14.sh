#!/usr/bin/env bash
# saddr-form record loads (sad), + non-temporal policy (sadnt), vs the committed build (old)
set -o pipefail
VARIANTS="old sad sadnt" STEPS=3 timeout -k 10 600 bash abtest/ab_c5.sh || { echo AB5_FAILED; exit 1; }
VARIANTS="old sad sadnt" timeout -k 10 600 bash abtest/ab_c4.sh || { echo AB4_FAILED; exit 1; }
echo ALL_OK
