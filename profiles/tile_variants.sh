#!/usr/bin/env bash
# Tile-path numeric kernel variants (SPG_TILE_RU / SPG_TILE_DENSE / SPG_TILE_TWS) on
# configs 3 (upper half) and 4, with sampled-row parity.  VARIANTS: one variant per line,
# "tag VAR=value ...".  Each variant is its own process and time limit; results:
# gpurun_out/tilevar_<tag>.jsonl.
set -uo pipefail
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"ru1 SPG_TILE_RU=1
ru8 SPG_TILE_RU=8"}
while IFS= read -r v; do
    [ -z "$v" ] && continue
    set -- $v
    tag=$1; shift
    env "$@" timeout -k 10 240 python harness/configs.py --configs ${CFGS:-3 4} --alg ${ALG:-2} --steps 3 --check 16 \
        > "gpurun_out/tilevar_$tag.jsonl" 2> "gpurun_out/tilevar_$tag.err"
    rc=$?
    echo "$tag rc=$rc"
    [ $rc -eq 0 ] || exit $rc
done <<< "$VARIANTS"
