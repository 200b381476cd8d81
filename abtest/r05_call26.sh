#!/usr/bin/env bash
# Shipped build (record groups of 8): memory-pipeline stall counters of config 5's numeric
# kernel and config 4's, as abtest/r05_call13.sh measured for RG 1 / 4 / 8 builds.
set -uo pipefail
export TMPDIR=/tmp
P=gpurun_out/stall_final; mkdir -p $P
for c in 5 4; do
  A="bench.py --config $c --cpu-seconds 0 --steps 1 --warmup 0 --no-config2 --no-alg3-chunked"
  timeout -s KILL 240 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $P/c$c -o a -- python3 $A > $P/c${c}_a.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $P/c$c -o b -- python3 $A > $P/c${c}_b.log 2>&1 || exit 1
  echo "== config $c"; python3 profiles/summarize.py $P/c$c | grep -E "k_tile_sp|k_tile_dn"
  find $P/c$c -name "*.csv" -delete
done
echo ALL_OK
