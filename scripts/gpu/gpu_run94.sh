source scripts/gpu/guard.sh
mkdir -p gpurun_out/r94
step ph timeout -k 10 300 python scripts/perf/replica_phases.py > gpurun_out/r94/ph.log 2>&1
grep -v "^\[sv replicas\]" gpurun_out/r94/ph.log
grep "^\[sv replicas\]" gpurun_out/r94/ph.log | tail -8
