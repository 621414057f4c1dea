source scripts/gpu/guard.sh
mkdir -p gpurun_out/r66
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r66/tests.log 2>&1
tail -2 gpurun_out/r66/tests.log
for r in 8 16 0; do
SV_DOMAIN_RESERVE=$r step lb$r timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r66/lb_$r.log 2>&1
echo reserve $r; grep loopback gpurun_out/r66/lb_$r.log
done
SV_DOMAIN_RESERVE=8 step rej timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r66/rej.log 2>&1
cat gpurun_out/r66/rej.log
