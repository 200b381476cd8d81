#!/usr/bin/env bash
# Round-3 final run on one GPU: the GPU parity suite, then (only if green) the default bench
# line (the N=1 headline, with the scipy CPU baseline) and profiles/collect_r03.sh for
# configs 4, 2 and 5 (bench line, rocprofv3 kernel trace + stats, FETCH/WRITE passes).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
WHICH="${WHICH:-4 2 5}" bash profiles/collect_r03.sh
