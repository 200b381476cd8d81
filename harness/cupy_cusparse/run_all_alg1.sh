#!/usr/bin/env bash
# Port of cupy_cusparse/run_all_alg1.sh: generate A/B/C_py with the Python shim (ALG1),
# run the native driver spgemm_from_txt_alg1 on A/B, compare C_py and C_cu bitwise.
# Same knobs: OUTDIR ($1), SIZES, DENSITIES, CHUNK_FRACTION, PYGEN_PY, PYGEN_SCRIPT, CUEXE,
# CMPPY_PY, CMPPY_SCRIPT, STRICT.  Report: $OUTDIR/report_alg1.txt.
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUTDIR="${1:-dump_alg1_txt}"
SIZES="${SIZES:-"32 64 128 256 512 1024"}"
DENSITIES="${DENSITIES:-"0.01 0.1 0.3 0.5"}"
CHUNK_FRACTION="${CHUNK_FRACTION:-0.2}"
PYGEN_PY="${PYGEN_PY:-python3}"
PYGEN_SCRIPT="${PYGEN_SCRIPT:-$HERE/gen_and_save_alg1_txt.py}"
CUEXE="${CUEXE:-$HERE/../../drivers/bin/spgemm_from_txt_alg1}"
CMPPY_PY="${CMPPY_PY:-python3}"
CMPPY_SCRIPT="${CMPPY_SCRIPT:-$HERE/compare_csrs_txt.py}"
STRICT="${STRICT:-}"

echo "==[1/3] generate A/B/C(py, ALG1) to $OUTDIR =="
"$PYGEN_PY" "$PYGEN_SCRIPT" --sizes $SIZES --densities $DENSITIES --outdir "$OUTDIR" \
  --chunk-fraction "$CHUNK_FRACTION"

echo "==[2/3] native ALG1 (libmi355_spgemm) for C(cu) =="
shopt -s nullglob
cases=("$OUTDIR"/A_n*_dens*_alg1_indptr.txt)
if [ ${#cases[@]} -eq 0 ]; then
  echo "no A_* files (_alg1_) in $OUTDIR" >&2
  exit 2
fi
pass=0; fail=0; total=0
report="$OUTDIR/report_alg1.txt"
: > "$report"
for a_indptr in "${cases[@]}"; do
  prefix="${a_indptr%_indptr.txt}"
  tag="$(basename "$prefix")"
  base="${tag#A_}"
  Apre="$OUTDIR/A_${base}"; Bpre="$OUTDIR/B_${base}"
  Cpy="$OUTDIR/C_py_${base}"; Ccu="$OUTDIR/C_cu_${base}"
  for need in "${Bpre}_indptr.txt" "${Cpy}_indptr.txt"; do
    if [ ! -f "$need" ]; then echo "[SKIP] missing:$need" | tee -a "$report"; continue 2; fi
  done
  echo "-> [$base] native computing..."
  CHUNK_FRACTION="$CHUNK_FRACTION" "$CUEXE" "$Apre" "$Bpre" "$Ccu" >/dev/null
  echo "   comparing..."
  if "$CMPPY_PY" "$CMPPY_SCRIPT" "$Cpy" "$Ccu" $STRICT >/dev/null; then
    echo "[PASS] $base" | tee -a "$report"; pass=$((pass+1))
  else
    echo "[FAIL] $base" | tee -a "$report"; fail=$((fail+1))
  fi
  total=$((total+1))
done
echo "==[3/3] finish:$pass PASS / $fail FAIL / $total TOTAL =="
echo "Report:$report"
[ "$fail" -eq 0 ]
