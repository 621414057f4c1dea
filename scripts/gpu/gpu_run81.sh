source scripts/gpu/guard.sh
mkdir -p gpurun_out/r81
for it in 1 2 4; do
SV_GS_ITERS=$it step w$it timeout -k 10 200 python bench.py --workload worldline --no-cpu-baseline > gpurun_out/r81/w$it.log 2>&1
echo WL iters $it $(grep -o '"value": [0-9.]*' gpurun_out/r81/w$it.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r81/w$it.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r81/w$it.log)
done
