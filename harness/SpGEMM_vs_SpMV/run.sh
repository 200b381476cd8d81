#!/bin/bash
# Port of SpGEMM_vs_SpMV/run.sh: sizes {128,256,512,1024} x densities {0.01,0.05,0.1,0.5}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUTFILE="${OUTFILE:-benchmark_results.txt}"
RUNS="${RUNS:-100}"
echo "Benchmark results - $(date)" > "$OUTFILE"
echo -e "==========================================\n" >> "$OUTFILE"
for s in ${SIZES:-128 256 512 1024}; do
  for d in ${DENSITIES:-0.01 0.05 0.1 0.5}; do
    echo ">>> Running size = $s    Running density = $d" | tee -a "$OUTFILE"
    echo "--- computing ---" | tee -a "$OUTFILE"
    python3 "$HERE/profiler.py" --densityA $d --densityB $d --m $s --n $s --p $s --runs $RUNS >> "$OUTFILE" 2>&1
    echo "complete!"
    echo "" >> "$OUTFILE"
  done
done
echo -e "All runs completed. Results saved to $OUTFILE\n"
