#!/bin/bash
# Port of SpGEMM_alg_comparison/run.sh: n in {512,1024} x density in {0.1,0.5}, 100 runs
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUTFILE="${OUTFILE:-benchmark_results.txt}"
RUNS="${RUNS:-100}"
echo "Benchmark results - $(date)" > "$OUTFILE"
echo -e "==========================================\n" >> "$OUTFILE"
for s in ${SIZES:-512 1024}; do
  for d in ${DENSITIES:-0.1 0.5}; do
    echo -e "size = $s, density = $d" | tee -a "$OUTFILE"
    echo "--- computing ---" | tee -a "$OUTFILE"
    python3 "$HERE/profiler.py" --density $d --size $s --runs $RUNS >> "$OUTFILE" 2>&1
    echo "complete!"
    echo "" >> "$OUTFILE"
  done
done
echo -e "All runs completed. Results saved to $OUTFILE\n"
