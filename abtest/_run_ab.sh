VARIANTS="noaln aln alnm0 noaln aln alnm0" bash abtest/ab_c5.sh > gpurun_out/ab_aln.log 2>&1; echo rc=$?; cat gpurun_out/ab_aln.log
VARIANTS="alnm0" bash abtest/pmc_c5.sh > gpurun_out/pmc5a.log 2>&1; cat gpurun_out/pmc5a.log
