# Dev tool: VGPR / occupancy / LDS / scratch per kernel from -Rpass-analysis=kernel-resource-usage.
# usage (from profiles/): python tools_resource.py [name filter]
import re, subprocess, sys
cmd = "hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I../include -I../spmm_amd/csrc -c ../spmm_amd/csrc/spgemm.hip -o /tmp/x.o -Rpass-analysis=kernel-resource-usage"
out = subprocess.run(cmd, shell=True, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()}
        rows.append(cur); continue
    for key in ("VGPRs", "SGPRs", "ScratchSize \[bytes/lane\]", "Occupancy \[waves/SIMD\]", "LDS Size \[bytes/block\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        n = re.sub(r"\(.*", "", r["name"]).replace("void spg::", "")
        print(f"{n[:95]:95s} vgpr={r.get('VGPRs')} occ={r.get('Occupancy')} lds={r.get('LDS')} scratch={r.get('ScratchSize')}")
