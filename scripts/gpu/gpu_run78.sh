source scripts/gpu/guard.sh
mkdir -p gpurun_out/r78
SV_DEBUG_TIMING=1 step dbg timeout -k 10 200 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r78/dbg.log 2>&1
grep "sv replicas" gpurun_out/r78/dbg.log | head -20
