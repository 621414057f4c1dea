source scripts/gpu/guard.sh
mkdir -p gpurun_out/r83
SV_DEBUG_TIMING=1 step dbg timeout -k 10 300 python bench.py --steps 2000 --warmup 5 --no-cpu-baseline > gpurun_out/r83/dbg.log 2>&1
grep -c abort gpurun_out/r83/dbg.log
