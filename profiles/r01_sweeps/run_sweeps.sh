set -euo pipefail
mkdir -p gpurun_out/sweeps
timeout -k 10 700 python harness/configs.py --configs 2 3 4 5 --steps 3 --check 8 > gpurun_out/sweeps/configs.jsonl 2> gpurun_out/sweeps/configs.err
timeout -k 10 600 python harness/dense_vs_sparseGEMM/main.py --size 8192 --density 1e-4 1e-3 1e-2 5e-2 1e-1 --dtype float64 --runs 3 > gpurun_out/sweeps/dense_vs_sparse_n8192_f64.txt 2>&1
timeout -k 10 600 python harness/SpGEMM_alg_comparison/profiler.py --size 1024 4096 --density 1e-2 1e-1 --dtype float32 --runs 3 > gpurun_out/sweeps/alg_comparison_f32.txt 2>&1
echo done
