#!/usr/bin/env bash
# Per-phase timings (profiles/phases.py) of alternative builds of the engine, for A/B
# experiments: every spmm_amd/lib/lib<name>.so other than the product library, through
# SPG_LIB.  Results: gpurun_out/phases_<name>.json.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 120 python profiles/phases.py --reps 30 > gpurun_out/phases_base.json 2> gpurun_out/variants.err
for so in spmm_amd/lib/lib*.so; do
    name=$(basename "$so" .so); name=${name#lib}
    [ "$name" = "mi355_spgemm" ] && continue
    SPG_LIB=$PWD/$so timeout -k 10 120 python profiles/phases.py --reps 30 > "gpurun_out/phases_$name.json" 2>> gpurun_out/variants.err || exit $?
done
echo variants done
