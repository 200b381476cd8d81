#!/usr/bin/env bash
# The 2-rank gloo rehearsal of bench.py's N=2 line on the shipped build (record groups of 8).
set -uo pipefail
mkdir -p gpurun_out
SPG_DIST_BACKEND=gloo timeout -k 10 900 python3 bench.py --gpus 2 --steps 3 --warmup 2 --cpu-seconds 0 \
    > gpurun_out/r05_rehearse2_final.json 2> gpurun_out/r05_rehearse2_final.err || { tail -30 gpurun_out/r05_rehearse2_final.err; exit 1; }
python3 - <<'P'
import json
d = json.loads(open("gpurun_out/r05_rehearse2_final.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], json.dumps(d.get("b_values_pipeline")))
print(json.dumps(d.get("config5", {}).get("b_values_pipeline")), d.get("config5", {}).get("ms_per_step"))
P
