source scripts/gpu/guard.sh
mkdir -p gpurun_out/r59
SV_DEBUG_TIMING=1 step dbg timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/r59/dbg.log 2>&1
grep -c . gpurun_out/r59/dbg.log
