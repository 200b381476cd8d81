#!/bin/bash
# Port of deterministic/test_deterministic.sh: for each algorithm and seed 1..10, run the
# dump twice in fresh processes and diff the outputs.
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
TMP="${TMPDIR:-/tmp}/spg_det.$$"
mkdir -p "$TMP"
status=0
for alg in 1 2 3; do
  echo "Testing alg$alg ..."
  deterministic=true
  for i in $(seq 1 ${SEEDS:-10}); do
    python3 "$HERE/spgemm_alg.py" --out "$TMP/file1.txt" --dtype float32 --seed $i --alg $alg
    python3 "$HERE/spgemm_alg.py" --out "$TMP/file2.txt" --dtype float32 --seed $i --alg $alg
    if ! diff -q "$TMP/file1.txt" "$TMP/file2.txt" >/dev/null 2>&1; then
      deterministic=false
      echo "alg$alg: mismatch at iteration $i"
      break
    fi
  done
  if [ "$deterministic" = true ]; then echo "alg$alg is deterministic"; else echo "alg$alg NOT deterministic"; status=1; fi
done
rm -rf "$TMP"
exit $status
