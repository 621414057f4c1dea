source scripts/gpu/guard.sh
mkdir -p gpurun_out/r108
export SV_DEBUG_TIMING=1
step d timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r108/bench.log 2> gpurun_out/r108/dbg.log
step d2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 640 > gpurun_out/r108/bench640.log 2> gpurun_out/r108/dbg640.log
