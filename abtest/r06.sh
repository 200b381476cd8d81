#!/usr/bin/env bash
# One parameterised gpurun driver for the A/B and counter steps (replaces the one-off
# r05_call*.sh scripts).  Every argument is a step, run in order; the first failing step ends
# the call (nothing more runs on the GPU after a failure).
#   ab4:V1,V2,..     config-4 bench phases of fp64 variant builds (abtest/ab_c4.sh)
#   ab5:V1,V2,..     the same on config 5 (abtest/ab_c5.sh)
#   seq:V1,V2,..     bit-identity digest of each variant against the others (abtest/seqcheck.py)
#   dram5 / dram4    fabric reads split into DRAM and Infinity-Cache hits for the numeric kernel
#                    of config 5 / 4 on the shipped library (TCC_EA0_RDREQ vs _RDREQ_DRAM)
#   pmc4:V1,..       per-variant counter passes on config 4 (PMC4_SETS: space-separated
#                    comma lists, one rocprofv3 --pmc pass each; a pass that rocprofv3 rejects
#                    is reported and skipped)
#   f32:V1,..        fp32 products (F32_SHAPES "N:density ..."): bench phases per variant
#   ptest:V:EXPR     pytest -m gpu -k EXPR against variant V's library (SPG_LIB; EXPR all: no -k)
#   gputests         the whole -m gpu suite on the shipped library
#   bench            the default bench line on the shipped library
# usage: gpurun -- 'bash abtest/r06.sh ab4:base,d8 dram5'
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}; arg=${arg//,/ }
  echo "== step $step"
  case $kind in
    ab4) STEPS=${STEPS:-3} VARIANTS="$arg" bash abtest/ab_c4.sh || exit 1 ;;
    ab5) STEPS=${STEPS:-2} VARIANTS="$arg" bash abtest/ab_c5.sh || exit 1 ;;
    seq)
      for v in $arg; do
        SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 120 python abtest/seqcheck.py > gpurun_out/r06/seq_$v.txt 2>&1 || { cat gpurun_out/r06/seq_$v.txt; exit 1; }
        echo "$v $(tr '\n' ' ' < gpurun_out/r06/seq_$v.txt)"
      done ;;
    dram5|dram4)
      c=${kind#dram}; P=gpurun_out/r06/dram$c; mkdir -p $P
      A="bench.py --config $c --cpu-seconds 0 --steps 1 --warmup 0 --no-config2 --no-alg3-chunked"
      timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum GRBM_GUI_ACTIVE --output-format csv -d $P -o a -- python3 $A > $P/a.log 2>&1 || { tail -5 $P/a.log; exit 1; }
      python3 profiles/summarize.py $P | grep -E "k_tile" | tee $P/summary.txt
      find $P -name "*.csv" -delete ;;
    pmc4)
      for v in $arg; do
        P=gpurun_out/r06/pmc4_$v; mkdir -p $P; i=0
        for set in ${PMC4_SETS:-SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_INSTS_VMEM_WR,SQ_INSTS_VMEM_RD,SQ_INST_CYCLES_VMEM_WR,SQ_INST_CYCLES_VMEM_RD TCP_TCC_WRITE_REQ_sum,TCP_TCC_READ_REQ_sum,TCP_PENDING_STALL_CYCLES_sum,TA_DATA_STALLED_BY_TC_CYCLES_sum,TA_ADDR_STALLED_BY_TC_CYCLES_sum,GRBM_GUI_ACTIVE}; do
          i=$((i+1))
          SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d $P -o p$i -- python3 bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 1 --warmup 0 > $P/p$i.log 2>&1 || { echo "pass $i ($set) failed rc=$?"; tail -3 $P/p$i.log; }
        done
        echo "== $v"; python3 profiles/summarize.py $P | grep -E "k_tile_dn" | tee $P/summary.txt
        find $P -name "*.csv" -delete
      done ;;
    kt4)
      for v in $arg; do
        P=gpurun_out/r06/kt4_$v; mkdir -p $P
        SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $P -o kt -- python3 bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --steps 2 --warmup 1 > $P/kt.log 2>&1 || { echo "kt4 $v failed"; tail -3 $P/kt.log; exit 1; }
        echo "== $v"; python3 profiles/summarize.py $P | head -12 | tee $P/summary.txt
        find $P -name "*.csv" -delete
      done ;;
    f32)
      for sh in ${F32_SHAPES:-65536:0.005 16384:0.01 8192:0.01 8192:0.1}; do
        n=${sh%%:*}; d=${sh#*:}
        for v in $arg; do
          SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 300 python bench.py --no-config2 --no-alg3-chunked --cpu-seconds 0 --dtype float32 --alg 2 --n $n --density $d --steps 5 --warmup 2 > gpurun_out/r06/f32_${v}_${n}_${d}.json 2> gpurun_out/r06/f32_${v}_${n}_${d}.err || { echo "f32 $v $n $d failed"; tail -3 gpurun_out/r06/f32_${v}_${n}_${d}.err; exit 1; }
          python3 -c "import json; d=json.load(open('gpurun_out/r06/f32_${v}_${n}_${d}.json')); print('$v $n $d', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
        done
      done ;;
    ptest)
      v=${arg%%:*}; k=${arg#*:}; K=(-k "$k"); [ "$k" = all ] && K=(-m gpu)
      SPG_LIB=$PWD/spmm_amd/lib/libv_$v.so timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu "${K[@]}" --timeout 300 --timeout-method thread > gpurun_out/r06/ptest_$v.log 2>&1; e=$?
      tail -3 gpurun_out/r06/ptest_$v.log; [ $e = 0 ] || exit 1 ;;
    gputests)
      timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06/gpu_tests.log 2>&1; e=$?
      tail -3 gpurun_out/r06/gpu_tests.log; [ $e = 0 ] || exit 1 ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err || { tail -5 gpurun_out/r06/bench.err; exit 1; }
      cat gpurun_out/r06/bench.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_OK
