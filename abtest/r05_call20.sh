#!/usr/bin/env bash
# LDS-side counters for the symbolic and numeric tile kernels (configs 4 and 5): is the
# symbolic pass bound by its LDS bit-set instructions?
set -uo pipefail
export TMPDIR=/tmp
P=gpurun_out/lds; mkdir -p $P
for c in 4 5; do
  A="bench.py --config $c --cpu-seconds 0 --steps 1 --warmup 0 --no-config2 --no-alg3-chunked"
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/c$c -o a -- python3 $A > $P/c${c}_a.log 2>&1 || { tail -5 $P/c${c}_a.log; exit 1; }
  echo "== config $c"; python3 profiles/summarize.py $P/c$c | grep -E "k_tile" | head -8
  find $P/c$c -name "*.csv" -delete
done
echo ALL_OK
