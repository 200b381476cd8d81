#!/usr/bin/env bash
# Counter passes for the tile path on one configuration (harness/configs.py, one product
# after a warmup): kernel trace, two SQ passes, one TCC pass.  TAG names the output dir.
set -euo pipefail
OUT=$PWD/gpurun_out/prof_${TAG:-tile}
mkdir -p "$OUT"
export TMPDIR=/tmp
A="harness/configs.py --configs ${CFG:-4} --alg ${ALG:-2} --steps 1 --check 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace -- python3 $A > "$OUT/trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT" -o sq1 -- python3 $A > "$OUT/sq1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT" -o sq2 -- python3 $A > "$OUT/sq2.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d "$OUT" -o tcc -- python3 $A > "$OUT/tcc.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d "$OUT" -o tcc2 -- python3 $A > "$OUT/tcc2.log" 2>&1
python3 profiles/summarize.py "$OUT" > "$OUT/summary.txt"
echo "counters done ($OUT)"
