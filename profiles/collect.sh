#!/usr/bin/env bash
# Profile collection on the GPU box (run through gpurun from the repo root).
#   1. bench.py (BENCH_ARGS) -> gpurun_out/bench_<tag>.json
#   2. rocprofv3 --kernel-trace --stats of the same command -> gpurun_out/prof_<tag>/trace_*
#   3. three separate PMC passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT + TCC_MISS: they do not fit
#      one TCC pass)
#   4. summary + pmc_traffic.json entry (stamped with the library's build id)
# Every GPU step has its own time limit and the steps are chained with &&.
set -euo pipefail
TAG=${TAG:-r02_c2}
ARGS=${BENCH_ARGS:-}
OUT=$PWD/gpurun_out
P=$OUT/prof_$TAG
mkdir -p "$P"
export TMPDIR=/tmp
# (the box starts without gpurun_out: take the committed file, keep every other entry)
[ -f "$OUT/pmc_traffic.json" ] || cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
timeout -k 10 400 python bench.py $ARGS > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P" -o trace \
    -- python3 bench.py $ARGS --cpu-seconds 0 > "$P/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P" -o pmc_fetch \
    -- python3 bench.py $ARGS --steps 3 --warmup 1 --cpu-seconds 0 > "$P/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P" -o pmc_write \
    -- python3 bench.py $ARGS --steps 3 --warmup 1 --cpu-seconds 0 > "$P/write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$P" -o pmc_hit \
    -- python3 bench.py $ARGS --steps 3 --warmup 1 --cpu-seconds 0 > "$P/hit.log" 2>&1
python3 profiles/summarize.py "$P" > "$OUT/summary_$TAG.txt"
python3 profiles/pmc_to_json.py "$P" "$PMC_KEY" "$PMC_KERNEL" "$OUT/pmc_traffic.json"
python3 profiles/kernel_traffic.py "$P" > "$OUT/traffic_$TAG.txt" 2>/dev/null || true
# (per-dispatch traces are large; the summaries above keep what is used)
find "$P" -name "*kernel_trace.csv" -delete
echo "collect done ($TAG)"
