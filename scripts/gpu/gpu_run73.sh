source scripts/gpu/guard.sh
mkdir -p gpurun_out/r73
for rep in 1 2; do
for th in 40 44 48 52 56 64; do
SV_FUSED_TH=$th step th$th timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/r73/th$th.log 2>&1
echo TH $th $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r73/th$th.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r73/th$th.log)
done
done
