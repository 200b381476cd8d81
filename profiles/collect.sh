#!/usr/bin/env bash
# Profile collection on the GPU box (run through gpurun from the repo root).
#   1. bench.py (default config) -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command -> gpurun_out/prof/trace_*
#   3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass)
# Every GPU step has its own time limit and the steps are chained with &&.
set -euo pipefail
ROUND=${ROUND:-r01}
ARGS=${BENCH_ARGS:-}
OUT=$PWD/gpurun_out
mkdir -p "$OUT/prof"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace \
    -- python3 bench.py $ARGS --cpu-seconds 0 > "$OUT/prof_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/prof" -o pmc_fetch \
    -- python3 bench.py $ARGS --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/prof_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/prof" -o pmc_write \
    -- python3 bench.py $ARGS --steps 5 --warmup 2 --cpu-seconds 0 > "$OUT/prof_write.log" 2>&1
python3 profiles/summarize.py "$OUT/prof" > "$OUT/summary_${ROUND}.txt"
KEY=${PMC_KEY:-n16384_d0.001_float64_alg1}
python3 profiles/pmc_to_json.py "$OUT/prof" "$KEY" "${PMC_KERNEL:-k_row<double, int, int, 1}" "$OUT/pmc_traffic.json"
echo "collect done ($ROUND)"
