#!/usr/bin/env bash
# A/B of library builds on the same box: per-phase device time and wall per call (config 2)
set -uo pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-old new av0 old new av0}; do
  SPG_LIB=$PWD/abtest/lib$v.so timeout -k 10 120 python profiles/phases.py --reps 50 > gpurun_out/ph_$v.json 2>gpurun_out/ph_$v.err || exit 1
  python - "$v" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/ph_{sys.argv[1]}.json"))
print(sys.argv[1], " ".join(f"{a}: wall {d[a]['wall_ms']*1e3:.1f}us {json.dumps({k: round(v*1e3,1) for k,v in d[a]['phases_ms'].items()})}" for a in ("alg1","alg2")))
PY
done
