VARIANTS="base5 noseg base5 noseg" bash abtest/ab_c4.sh > gpurun_out/ab_ns.log 2>&1; echo rc=$?; cat gpurun_out/ab_ns.log
