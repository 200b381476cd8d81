#!/usr/bin/env bash
# A/B of fp64 development builds (abtest/build_variant.sh) on config 4: bench phases per
# variant, then (COUNTERS=1) TCC and SQ counter passes of each variant's kernels.
# usage: VARIANTS="dn1024 dn512" [COUNTERS=1] abtest/ab_c4.sh
set -uo pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
ARGS="--no-config2 --no-alg3-chunked --cpu-seconds 0 --steps ${STEPS:-3} --warmup 1 ${EXTRA:-}"
for v in $VARIANTS; do
  SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 240 python bench.py $ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { echo "$v bench rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.json')); print('$v', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
done
[ "${COUNTERS:-0}" = 1 ] || exit 0
for v in $VARIANTS; do
  P=gpurun_out/ab/prof_$v
  mkdir -p $P
  L=$PWD/spmm_amd/lib/libv_$v.so
  A="bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 1 --warmup 0"
  SPG_LIB=$L timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $P -o tcc1 -- python3 $A > $P/tcc1.log 2>&1 || exit 1
  SPG_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $P -o tcc2 -- python3 $A > $P/tcc2.log 2>&1 || exit 1
  SPG_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $P -o sq1 -- python3 $A > $P/sq1.log 2>&1 || exit 1
  SPG_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $P -o sq2 -- python3 $A > $P/sq2.log 2>&1 || exit 1
  python3 profiles/summarize.py $P | grep -E "==|k_tile" > $P/summary.txt
  echo "== $v"; cat $P/summary.txt
done
