source scripts/gpu/guard.sh
mkdir -p gpurun_out/r97
step rej timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r97/rej.log 2>&1
cat gpurun_out/r97/rej.log
step lb timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r97/lb.log 2>&1
grep loopback gpurun_out/r97/lb.log
step batch timeout -k 10 900 python scripts/perf/domain_batch.py > gpurun_out/r97/batch.log 2>&1
grep batch gpurun_out/r97/batch.log
