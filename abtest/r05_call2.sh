#!/usr/bin/env bash
# config 5 record-group width A/B (fp64 dev builds): RG 2 / 4 / 8 and the one-wave kernel
set -o pipefail
mkdir -p gpurun_out/ab
VARIANTS="rg2 rg4 rg8" STEPS=3 timeout -k 10 600 bash abtest/ab_c5.sh || { echo AB_FAILED; exit 1; }
SPG_SP_RECORD_GROUP=1 SPG_LIB=$PWD/spmm_amd/lib/libv_rg4.so timeout -k 10 240 python bench.py --config 5 --cpu-seconds 0 --steps 3 --warmup 1 > gpurun_out/ab/c5_rg1.json 2> gpurun_out/ab/c5_rg1.err || { echo RG1_FAILED; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab/c5_rg1.json')); print('c5 rg1', d['value'], d['ms_per_step'], d['config'].get('phases_ms_per_step'))"
