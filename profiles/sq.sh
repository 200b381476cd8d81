#!/usr/bin/env bash
# kernel trace + SQ/TCC counter passes for one bench configuration (BENCH_ARGS)
set -euo pipefail
OUT=$PWD/gpurun_out/prof_${TAG:-sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
A="${BENCH_ARGS:-} --steps 10 --warmup 3 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace -- python3 bench.py $A > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT" -o sq1 -- python3 bench.py $A > "$OUT/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT" -o sq2 -- python3 bench.py $A > "$OUT/sq2.log" 2>&1
python3 profiles/summarize.py "$OUT" > "$OUT/summary.txt"
echo "sq done"
