#!/usr/bin/env bash
# Multi-rank rehearsal of the row-block paths on a ONE-GPU box: two ranks share the GPU and
# talk over gloo (RCCL needs one GPU per rank).  Runs bench.py's launcher-free --gpus 2 path
# (the command the driver's scaling run uses: config 4 weak + the config5 key strong, here at
# N5=131072 so both ranks' slabs fit one card) and the row-block harness with sampled-row
# parity.  Results in gpurun_out/ (committed as profiles/r03_rehearse_*.json).
set -euo pipefail
export SPG_DIST_BACKEND=gloo
timeout -k 10 500 python3 bench.py --gpus 2 --steps 2 --warmup 1 --cpu-seconds 0 --config5-n 131072 \
    > gpurun_out/rehearse_bench.json 2> gpurun_out/rehearse_bench.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29532 harness/multi_gpu/spgemm_rowblock.py --steps 1 --warmup 1 --check 32 \
    > gpurun_out/rehearse_rowblock.json 2> gpurun_out/rehearse_rowblock.err
echo "rehearsal done"
