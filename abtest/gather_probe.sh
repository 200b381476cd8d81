#!/usr/bin/env bash
# Runs abtest/gather_probe over the slice sizes / segment lengths of the tile path (tile width TW
# at config 4: slice = TW x 3.94 KB, L = TW x 0.005) and collects, per run, the TCC request mix
# (32/64/128-B fabric read requests), FETCH_SIZE + TCC_HIT, and TCC_MISS + WRITE_SIZE, each pass
# its own rocprofv3 run.  Output: gpurun_out/probe/*; abtest/probe_report.py folds it.
set -euo pipefail
cd "$(dirname "$0")/.."
B=$PWD/abtest/gather_probe
OUT=$PWD/gpurun_out/probe
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 60 "$B" "$@" > "$OUT/$tag.json"
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
      --output-format csv -d "$OUT/p_$tag" -o req -- "$B" "$@" > "$OUT/p_$tag.req.log" 2>&1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d "$OUT/p_$tag" -o fh \
      -- "$B" "$@" > "$OUT/p_$tag.fh.log" 2>&1
  timeout -s KILL 60 rocprofv3 --pmc TCC_MISS_sum WRITE_SIZE --output-format csv -d "$OUT/p_$tag" -o mw \
      -- "$B" "$@" > "$OUT/p_$tag.mw.log" 2>&1
  echo "$tag $(cat "$OUT/$tag.json")"
}
run stream1g stream 1024
for s in ${SLICES:-1 2 4 8 16 64}; do run g_s${s}_l10 gather $s 10; done
run g_s2_l3 gather 2 3
run g_s8_l3 gather 8 3
run g_s8_l40 gather 8 40
run gs_s2_l3 gather 2 3 1
run gs_s4_l5 gather 4 5 1
run gs_s8_l10 gather 8 10 1
python3 abtest/probe_report.py "$OUT" > "$OUT/report.txt"
cat "$OUT/report.txt"
