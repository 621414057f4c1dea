source scripts/gpu/guard.sh
mkdir -p gpurun_out/r65
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r65/tests.log 2>&1
tail -2 gpurun_out/r65/tests.log
SV_DOMAIN_SPLIT=0 step lb0 timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r65/lb_nosplit.log 2>&1
grep loopback gpurun_out/r65/lb_nosplit.log
step lb timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r65/lb_split.log 2>&1
grep loopback gpurun_out/r65/lb_split.log
