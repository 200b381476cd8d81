"""Prints the A/B phase timings written by profiles/variants.sh (gpurun_out/phases_v*.json)."""
import glob
import json

for f in sorted(glob.glob("gpurun_out/phases_base.json") + glob.glob("gpurun_out/phases_v*.json")):
    d = json.load(open(f))
    print(f.split("phases_")[1][:-5].ljust(8),
          "  ".join(f"{a}: {d[a]['wall_ms']*1e3:6.1f}us " +
                    "/".join(f"{k[:3]}={v*1e3:.1f}" for k, v in d[a]["phases_ms"].items())
                    for a in ("alg1", "alg2", "alg3")))
