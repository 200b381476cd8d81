#!/usr/bin/env bash
# Builds an A/B pair for profiles/variants.sh: the committed HEAD engine as
# spmm_amd/lib/libva_head.so + libvc_head.so and the working tree as libvb_new.so +
# libvd_new.so (interleaved, so box drift shows up as head/head or new/new spread).
# Remove them with `rm spmm_amd/lib/libv*.so` afterwards.
set -euo pipefail
cd "$(dirname "$0")/.."
git stash push -q -- spmm_amd/csrc include
trap 'git stash pop -q' EXIT
make -s -j8 >/dev/null
cp spmm_amd/lib/libmi355_spgemm.so spmm_amd/lib/libva_head.so
cp spmm_amd/lib/libmi355_spgemm.so spmm_amd/lib/libvc_head.so
git stash pop -q
trap - EXIT
touch spmm_amd/csrc/spgemm.hip
make -s -j8 >/dev/null
cp spmm_amd/lib/libmi355_spgemm.so spmm_amd/lib/libvb_new.so
cp spmm_amd/lib/libmi355_spgemm.so spmm_amd/lib/libvd_new.so
