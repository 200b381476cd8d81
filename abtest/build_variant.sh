#!/usr/bin/env bash
# Development A/B builds: abtest/build_variant.sh NAME [-DFLAG=V ...] builds an fp64-only
# library (SPG_ONLY_F64: ~3x faster to compile) with the extra flags as
# spmm_amd/lib/libv_NAME.so; load it with SPG_LIB=$PWD/spmm_amd/lib/libv_NAME.so.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
TYPES=-DSPG_ONLY_F64
[ -n "${ALLTYPES:-}" ] && TYPES=-USPG_ONLY_F64   # ALLTYPES=1: every value type (3x longer)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $TYPES "$@" \
    -DSPG_SOURCE_ID="\"variant-$name\"" -shared -Iinclude -Ispmm_amd/csrc spmm_amd/csrc/spgemm.hip \
    -o spmm_amd/lib/libv_$name.so
echo "built spmm_amd/lib/libv_$name.so ($*)"
