#!/usr/bin/env bash
# Spill-list grid (one wave per 16 rows of A up to 1024 waves, was one 4-wave block per 1024
# rows): the N = 1024 fp32 probe and the config-2 line with the old and the new library.
set -uo pipefail
for v in old new; do
  L=$PWD/spmm_amd/lib/libmi355_spgemm.so; [ $v = old ] && L=$PWD/spmm_amd/lib/libv_old.so
  echo "== $v"
  SPG_LIB=$L timeout -k 10 120 python abtest/small_probe.py || exit 1
  SPG_LIB=$L timeout -k 10 200 python bench.py --config 2 --cpu-seconds 0 > gpurun_out/c23_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/c23_$v.json').read().strip().splitlines()[-1]); print('config2', d['value'], d['ms_per_step'])"
done
