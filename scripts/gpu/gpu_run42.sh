source scripts/gpu/guard.sh
mkdir -p gpurun_out/r42
export TMPDIR=/tmp
for m in batch launch batch launch; do
step b$m bash -c "timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --event-timing $m > gpurun_out/r42/b$m.log 2>&1"
echo "$m: $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r42/b$m.log | tr '\n' ' ')"
done
