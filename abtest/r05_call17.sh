#!/usr/bin/env bash
# fp32 entry runs on every dense fp32 tile (SPG_F32_RUN_MIN=0) vs k_tile's owner rounds for short segments
set -o pipefail
mkdir -p gpurun_out/fp32
for sh in "65536 0.005" "8192 0.01" "16384 0.01"; do
  set -- $sh
  for v in main f32all; do
    L=$PWD/spmm_amd/lib/libmi355_spgemm.so; [ $v = f32all ] && L=$PWD/spmm_amd/lib/libv_f32all.so
    SPG_LIB=$L timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2 --n $1 --density $2 --steps 5 --warmup 2 > gpurun_out/fp32/a_${v}_$1_$2.json 2>/dev/null || { echo B; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/fp32/a_${v}_$1_$2.json')); print('$v $1 $2', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
  done
done
echo ALL_OK
