source scripts/gpu/guard.sh
mkdir -p gpurun_out/r101
for rep in 1 2; do
for sp in 0 1; do
SV_SPIN=$sp step h$sp timeout -k 10 300 python bench.py --workload hammer --no-cpu-baseline --steps 100 > gpurun_out/r101/h$sp.log 2>&1
echo HAMMER spin $sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r101/h$sp.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r101/h$sp.log)
SV_SPIN=$sp step b$sp timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r101/b$sp.log 2>&1
echo HEAD spin $sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r101/b$sp.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r101/b$sp.log)
SV_SPIN=$sp step l$sp timeout -k 10 300 python scripts/perf/loopback_cost.py > gpurun_out/r101/l$sp.log 2>&1
echo LOOP spin $sp $(grep "loopback=True" gpurun_out/r101/l$sp.log)
done
done
