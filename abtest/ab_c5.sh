#!/usr/bin/env bash
# A/B of fp64 development builds on config 5 (one GPU): bench phases per variant.
# usage: VARIANTS="a b" abtest/ab_c5.sh
set -uo pipefail
mkdir -p gpurun_out/ab
for v in $VARIANTS; do
  SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 300 python bench.py --config 5 --cpu-seconds 0 --steps ${STEPS:-3} --warmup 1 > gpurun_out/ab/c5_$v.json 2> gpurun_out/ab/c5_$v.err || { echo "$v bench rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/c5_$v.json')); print('c5', '$v', d['value'], d['ms_per_step'], d['config'].get('phases_ms_per_step') or d.get('phases_ms_per_step'))"
done
