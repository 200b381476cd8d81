#!/usr/bin/env bash
# Timing-only sweep of abtest/gather_probe: occupancy (waves per CU), loads in flight (U) and
# record size at the tile path's slice sizes / segment lengths.  One JSON line per run.
set -euo pipefail
cd "$(dirname "$0")/.."
B=$PWD/abtest/gather_probe
for cfg in ${CFGS:-"2 10" "2 3" "4 5" "8 10"}; do
  set -- $cfg
  for st in 0 1; do
    for w in 8 16 32; do
      for u in 8 16; do
        timeout -k 10 60 "$B" gather $1 $2 $st $w $u 12
      done
    done
  done
done
timeout -k 10 60 "$B" gather 2 10 1 16 8 16
timeout -k 10 60 "$B" gather 2 3 1 16 8 16
