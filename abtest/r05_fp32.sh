#!/usr/bin/env bash
# round 5: fp32 tile path profile: config 3 at rho 1e-2 / 1e-1 and a
# config-4-shaped fp32 product -- bench phases + rocprofv3 kernel stats per shape
set -o pipefail
mkdir -p gpurun_out/fp32
export TMPDIR=/tmp
A="--no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2"
for sh in "8192 0.01" "8192 0.1" "65536 0.005"; do
  set -- $sh
  tag=n$1_d$2
  timeout -k 10 300 python bench.py $A --n $1 --density $2 --steps 5 --warmup 2 > gpurun_out/fp32/$tag.json 2> gpurun_out/fp32/$tag.err || { echo "bench $tag failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp32/prof_$tag -o run -- python3 bench.py $A --n $1 --density $2 --steps 3 --warmup 1 > gpurun_out/fp32/prof_$tag.log 2>&1 || { echo "prof $tag failed"; exit 1; }
  find gpurun_out/fp32/prof_$tag -name "*kernel_trace.csv" -delete
done
echo FP32_OK
