source scripts/gpu/guard.sh
mkdir -p gpurun_out/r72
for th in 32 48 64 80 96 128; do
SV_FUSED_TH=$th step th$th timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r72/th$th.log 2>&1
echo TH $th $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r72/th$th.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r72/th$th.log)
done
