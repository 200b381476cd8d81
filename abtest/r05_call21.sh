#!/usr/bin/env bash
# Where config 4's numeric time goes (timing-only builds, results wrong): no output (d8), no
# output + no segment-table reads (d72: synthetic 10-record segments), no output + no record
# loads (d10), neither (d74).  Then the full GPU suite on the shipped library.
set -uo pipefail
STEPS=3 VARIANTS="d8 d72 d10 d74" bash abtest/ab_c4.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05_gpu_final2.log 2>&1; e=$?
tail -3 gpurun_out/r05_gpu_final2.log; exit $e
