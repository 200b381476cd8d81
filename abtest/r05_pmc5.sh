#!/usr/bin/env bash
# config 5's numeric kernel: TCC traffic + SQ waits, cooperative record groups (rg4) vs the
# one-wave kernel (rg1, SPG_SP_RECORD_GROUP=1); one rocprofv3 --pmc pass per counter set
set -uo pipefail
export TMPDIR=/tmp
for v in rg4 rg1; do
  P=gpurun_out/pmc5_$v; mkdir -p $P
  [ $v = rg1 ] && export SPG_SP_RECORD_GROUP=1 || unset SPG_SP_RECORD_GROUP
  A="bench.py --config 5 --cpu-seconds 0 --steps 1 --warmup 0"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $P -o a -- python3 $A > $P/a.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $P -o b -- python3 $A > $P/b.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $P -o c -- python3 $A > $P/c.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $P -o d -- python3 $A > $P/d.log 2>&1 || exit 1
  python3 profiles/summarize.py $P | grep -E "==|k_tile_sp|k_tile_sym" > $P/summary.txt
  find $P -name "*.csv" -delete
  echo "== $v"; cat $P/summary.txt
done
