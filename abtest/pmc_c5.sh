#!/usr/bin/env bash
# TCC counters of config 5's numeric kernel for fp64 variants: FETCH_SIZE + TCC_HIT, WRITE_SIZE +
# TCC_MISS, one rocprofv3 pass each; prints per-launch bytes and the L2 hit rate, then deletes the CSVs.
set -uo pipefail
export TMPDIR=/tmp
for v in $VARIANTS; do
  P=gpurun_out/pmc5_$v; mkdir -p $P
  A="bench.py --config ${CFG:-5} --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 1 --warmup 0"
  SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $P -o a -- python3 $A > $P/a.log 2>&1 || exit 1
  SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --output-format csv -d $P -o b -- python3 $A > $P/b.log 2>&1 || exit 1
  python3 - "$P" "$v" <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if "k_tile" in kn:
            short = kn[kn.index("k_tile"):].split("(")[0][:40]
            acc[(short, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), c in sorted(acc.items(), key=lambda x: -x[0][1]):
    m = {n: sum(x) / len(x) for n, x in c.items()}
    h, mi = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
    print(v, k, g, "read_GB=%.1f" % (m.get("FETCH_SIZE", 0) * 2048 / 1e9), "write_GB=%.1f" % (m.get("WRITE_SIZE", 0) * 1024 / 1e9),
          "l2_hit=%.3f" % (h / (h + mi) if h + mi else 0), "req=%.3g" % (h + mi))
PY
  rm -rf $P/*/ $P/*.csv
done
