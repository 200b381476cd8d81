#!/usr/bin/env bash
# The reference's dense_vs_sparseGEMM grid in its own dtype (fp32) on the round-5 build, plus
# N = 8192 at densities 0.2 / 0.3 to bracket the break-even; compact table via dvs_table.py.
set -uo pipefail
mkdir -p gpurun_out
OUTFILE=gpurun_out/r05_dvs_fp32.txt RUNS=20 DTYPE=float32 timeout -k 10 700 bash harness/dense_vs_sparseGEMM/run.sh > /dev/null || exit 1
OUTFILE=gpurun_out/r05_dvs_fp32_hi.txt RUNS=10 DTYPE=float32 SIZES=8192 DENSITIES="0.2 0.3" timeout -k 10 300 bash harness/dense_vs_sparseGEMM/run.sh > /dev/null || exit 1
cat gpurun_out/r05_dvs_fp32.txt gpurun_out/r05_dvs_fp32_hi.txt > gpurun_out/r05_dvs_fp32_all.txt
python3 profiles/dvs_table.py gpurun_out/r05_dvs_fp32_all.txt profiles/r03_dense_vs_sparse_fp32.txt > gpurun_out/r05_dvs_fp32_table.txt
cat gpurun_out/r05_dvs_fp32_table.txt
