#!/usr/bin/env bash
# config 5 numeric kernel: memory-pipeline stall counters, RG 1 / RG 4 (shipped) / RG 8
set -uo pipefail
export TMPDIR=/tmp
P=gpurun_out/stall5; mkdir -p $P
A="bench.py --config 5 --cpu-seconds 0 --steps 1 --warmup 0"
for v in rg1 rg4 rg8; do
  L=$PWD/spmm_amd/lib/libmi355_spgemm.so; [ $v = rg8 ] && L=$PWD/spmm_amd/lib/libv_rg8.so
  E=""; [ $v = rg1 ] && E="SPG_SP_RECORD_GROUP=1"
  env $E SPG_LIB=$L true
  if [ $v = rg1 ]; then export SPG_SP_RECORD_GROUP=1; else unset SPG_SP_RECORD_GROUP; fi
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $P/$v -o a -- python3 $A > $P/${v}_a.log 2>&1 || exit 1
  SPG_LIB=$L timeout -s KILL 240 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --output-format csv -d $P/$v -o b -- python3 $A > $P/${v}_b.log 2>&1 || exit 1
  echo "== $v"; python3 profiles/summarize.py $P/$v | grep -E "k_tile_sp"
  find $P/$v -name "*.csv" -delete
done
echo ALL_OK
