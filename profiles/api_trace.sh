#!/usr/bin/env bash
# HIP runtime-API + kernel trace of a short bench run (no PMC counters in this pass), to
# see the host cost of each call: launches, memsets, copies and the stream sync.
set -uo pipefail
OUT=$PWD/gpurun_out/prof_api
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$OUT" -o api \
    -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$OUT/api.log" 2>&1
echo "api trace rc=$?"
