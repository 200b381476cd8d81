#!/usr/bin/env bash
# shipped build: full GPU suite, the default bench line, config 5
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r05_t9.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05_t9.log; exit 1; }
tail -1 gpurun_out/r05_t9.log
timeout -k 10 400 python bench.py > gpurun_out/r05_default.json 2> gpurun_out/r05_default.err || { echo BENCH_FAILED; exit 1; }
timeout -k 10 300 python bench.py --config 5 > gpurun_out/r05_c5.json 2> gpurun_out/r05_c5.err || { echo B5_FAILED; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05_default.json"))
print("c4", d["value"], d["ms_per_step"], d["phases_ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel"])
print("c2", d["config2"]["gflops"], d["config2"]["ms_per_step"])
print("alg3", {k: d["alg3_chunked"][k] for k in ("alg3_over_alg2_time", "alg3_over_alg2_peak", "alg3_over_alg2_workspace")}, d["alg3_chunked"]["alg2"]["ms_per_step"], d["alg3_chunked"]["alg3"]["ms_per_step"])
print("fp32", d["config3_fp32"]["ms_per_step"], d["config3_fp32"]["phases_ms_per_step"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["omp"])
e = json.load(open("gpurun_out/r05_c5.json"))
print("c5", e["value"], e["ms_per_step"], e["config"]["phases_ms_per_step"], e["roofline"]["frac"])
PY
echo ALL_OK
