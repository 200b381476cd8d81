VARIANTS="ph1 ph2 ph4 ph8" bash abtest/ab_c4.sh > gpurun_out/ab_ph.log 2>&1; echo rc=$?; cat gpurun_out/ab_ph.log
VARIANTS="ph1 sp4 sp8 sp16" bash abtest/ab_c5.sh > gpurun_out/ab_sp.log 2>&1; echo rc=$?; cat gpurun_out/ab_sp.log
SPG_LIB=$PWD/spmm_amd/lib/libv_ph4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "65536 or config3" -x -q --timeout 250 --timeout-method thread > gpurun_out/ph4_tests.log 2>&1; echo t_rc=$?; tail -3 gpurun_out/ph4_tests.log
SPG_LIB=$PWD/spmm_amd/lib/libv_sp8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "262144-0.001-2" -x -q --timeout 250 --timeout-method thread > gpurun_out/sp8_tests.log 2>&1; echo t_rc=$?; tail -3 gpurun_out/sp8_tests.log
