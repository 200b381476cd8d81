#!/usr/bin/env bash
# Where config 4's numeric time goes (timing-only builds, results wrong): no output (d8), no
# output + no segment-table reads (d72: synthetic 10-record segments), no output + no record
# loads (d10), neither (d74); and one wave walking a record group's 2 / 4 dense tiles in turn
# (seq2 / seq4, against base), with a bit-identity check.  Then the full GPU suite.
set -uo pipefail
for v in base seq2 seq4; do
  SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 120 python abtest/seqcheck.py || exit 1
done
STEPS=3 VARIANTS="base seq2 seq4 d8 d72 d10 d74" bash abtest/ab_c4.sh || exit 1
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05_gpu_final2.log 2>&1; e=$?
tail -3 gpurun_out/r05_gpu_final2.log; exit $e
