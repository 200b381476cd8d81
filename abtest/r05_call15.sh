#!/usr/bin/env bash
# config 4: record groups of 2 dense tiles with one block per item (dnrg2n) vs independent items;
# fabric credit stalls of the shipped dense kernel
set -uo pipefail
export TMPDIR=/tmp
VARIANTS="dn1 dnrg2n" timeout -k 10 600 bash abtest/ab_c4.sh || { echo AB4_FAILED; exit 1; }
P=gpurun_out/stall4; mkdir -p $P
A="bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $P -o a -- python3 $A > $P/a.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum --output-format csv -d $P -o b -- python3 $A > $P/b.log 2>&1 || exit 1
python3 profiles/summarize.py $P | grep -E "k_tile_dn|k_tile_sym"; find $P -name "*.csv" -delete
echo ALL_OK
