#!/usr/bin/env bash
# config 5: traffic and SQ waits of the persistent RG 8 kernel (vs the shipped RG 4 in profiles/r05_c5_*)
set -o pipefail
VARIANTS="rg8" timeout -k 10 600 bash abtest/pmc_c5.sh || { echo PMC_FAILED; exit 1; }
export TMPDIR=/tmp
P=gpurun_out/sq5; mkdir -p $P
for v in rg8 main; do
  L=$PWD/spmm_amd/lib/libv_$v.so; [ $v = main ] && L=$PWD/spmm_amd/lib/libmi355_spgemm.so
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $P/$v -o c -- python3 bench.py --config 5 --cpu-seconds 0 --steps 1 --warmup 0 > $P/$v.log 2>&1 || exit 1
  python3 profiles/summarize.py $P/$v | grep -E "k_tile_sp" ; find $P/$v -name "*.csv" -delete
done
echo ALL_OK
