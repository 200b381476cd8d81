#!/usr/bin/env bash
# Multi-rank rehearsal of the config-5 row-block path on a ONE-GPU box: two ranks share the
# GPU and talk over gloo (RCCL needs one GPU per rank).  Runs bench.py's own --gpus 2 path
# and the row-block harness with sampled-row parity.  Results in gpurun_out/.
set -euo pipefail
export SPG_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/rehearse_bench.json 2> gpurun_out/rehearse_bench.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29532 harness/multi_gpu/spgemm_rowblock.py --steps 1 --warmup 1 --check 32 \
    > gpurun_out/rehearse_rowblock.json 2> gpurun_out/rehearse_rowblock.err
echo "rehearsal done"
