source scripts/gpu/guard.sh
mkdir -p gpurun_out/r80
for rep in 1 2; do
for b in 16 32 64 128; do
SV_BATCH=$b step b$b timeout -k 10 200 python bench.py --no-cpu-baseline --steps 600 > gpurun_out/r80/b$b.log 2>&1
echo BATCH $b $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r80/b$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r80/b$b.log)
done
done
