#!/usr/bin/env bash
# GPU-box check used between kernel changes: the GPU parity tests, then the per-phase
# timings of profiles/phases.py (config 2).  Each GPU step has its own time limit; results
# land in gpurun_out/.  TESTS narrows the pytest selection (default: every gpu test).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
    --durations=15 > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests_rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python profiles/phases.py > gpurun_out/phases.json 2> gpurun_out/phases.err
echo "phases_rc=$?"
