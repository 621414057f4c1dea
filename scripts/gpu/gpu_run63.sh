source scripts/gpu/guard.sh
mkdir -p gpurun_out/r63
step lb timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r63/lb_split.log 2>&1
cat gpurun_out/r63/lb_split.log
SV_DOMAIN_SPLIT=0 step lb0 timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r63/lb_nosplit.log 2>&1
cat gpurun_out/r63/lb_nosplit.log
