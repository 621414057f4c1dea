source scripts/gpu/guard.sh
mkdir -p gpurun_out/r58
step rej timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r58/rej.log 2>&1
cat gpurun_out/r58/rej.log
