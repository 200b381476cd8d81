#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per pass, its own time limit) of fp64 development builds on
# one config: L2 hits/misses, fabric bytes and SQ instruction/wait counters of the tile
# kernels.  usage: CFG=4|5 VARIANTS="new ..." profiles/r03b_counters.sh
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
A="bench.py --config ${CFG:-4} --no-config2 --cpu-seconds 0 --steps 1 --warmup 0"
for v in ${VARIANTS:-new}; do
  P=gpurun_out/ab/prof_c${CFG:-4}_$v
  mkdir -p $P
  L=$PWD/spmm_amd/lib/libv_$v.so
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $P -o tcc1 -- python3 $A > $P/tcc1.log 2>&1 || { echo "$v tcc1 failed"; exit 1; }
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $P -o tcc2 -- python3 $A > $P/tcc2.log 2>&1 || { echo "$v tcc2 failed"; exit 1; }
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $P -o sq1 -- python3 $A > $P/sq1.log 2>&1 || { echo "$v sq1 failed"; exit 1; }
  python3 profiles/summarize.py $P | grep -E "==|k_tile" > $P/summary.txt
  echo "== c${CFG:-4} $v"; cat $P/summary.txt
done
