#!/bin/bash
# Port of dense_vs_sparseGEMM/run.sh: N in {1024,2048,4096,8192} x density in
# {0.001,0.01,0.05,0.1}, 100 runs.  BASELINE config 3 is the N=8192 column with
# DENSITIES="0.0001 0.001 0.01 0.1" and DTYPE=float64.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUTFILE="${OUTFILE:-benchmark_results.txt}"
RUNS="${RUNS:-100}"
DTYPE="${DTYPE:-float32}"
echo "Benchmark results - $(date)" > "$OUTFILE"
echo -e "==========================================\n" >> "$OUTFILE"
for s in ${SIZES:-1024 2048 4096 8192}; do
  for d in ${DENSITIES:-0.001 0.01 0.05 0.1}; do
    echo -e "size = $s, density = $d" | tee -a "$OUTFILE"
    echo "--- computing ---" | tee -a "$OUTFILE"
    python3 "$HERE/main.py" --density $d --size $s --runs $RUNS --dtype $DTYPE >> "$OUTFILE" 2>&1
    echo "complete!"
    echo "" >> "$OUTFILE"
  done
done
echo -e "All runs completed. Results saved to $OUTFILE\n"
