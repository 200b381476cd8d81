#!/usr/bin/env bash
# Round-3 kernel check on one GPU: the GPU parity suite on the working-tree library, then an
# interleaved A/B of fp64 development builds (HEAD vs working tree, abtest/build_variant.sh)
# on configs 4 and 5 (bench phases).  Every GPU step has its own time limit; results land in
# gpurun_out/.  SKIP_TESTS=1 skips the suite; VARIANTS (default "head new") picks the builds.
set -uo pipefail
mkdir -p gpurun_out/ab
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
      --durations=10 > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CONFIGS:-4 5}; do
  for v in ${VARIANTS:-head new}; do
    SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 300 python bench.py --config $cfg --no-config2 --cpu-seconds 0 \
        --steps ${STEPS:-3} --warmup 1 > gpurun_out/ab/c${cfg}_$v.json 2> gpurun_out/ab/c${cfg}_$v.err || { echo "c$cfg $v bench rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/c${cfg}_$v.json')); print('c$cfg', '$v', d['value'], d['ms_per_step'], d.get('phases_ms_per_step') or d['config'].get('phases_ms_per_step'))"
  done
done
