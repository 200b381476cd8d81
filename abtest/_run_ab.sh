VARIANTS="rec10 r10ntr ph1 rec10" bash abtest/ab_c5.sh > gpurun_out/ab_ntr.log 2>&1; echo rc=$?; cat gpurun_out/ab_ntr.log
VARIANTS="ph1 rec10 r10ntr" bash abtest/pmc_c5.sh > gpurun_out/pmc5.log 2>&1; echo rc=$?; cat gpurun_out/pmc5.log
VARIANTS="rec10nta r10ntr" CFG=4 bash abtest/pmc_c5.sh > gpurun_out/pmc4.log 2>&1; echo rc=$?; cat gpurun_out/pmc4.log
