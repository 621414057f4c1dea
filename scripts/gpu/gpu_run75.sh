source scripts/gpu/guard.sh
mkdir -p gpurun_out/r75
for cfg in "6 48" "6 60" "6 36" "4 52"; do
set -- $cfg
SV_FUSED_NW=$1 SV_FUSED_TH=$2 step nw$1_$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/r75/nw$1_$2.log 2>&1
echo NW $1 TH $2 $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r75/nw$1_$2.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r75/nw$1_$2.log)
done
for th in 24 32 48 64; do
SV_FUSED_TH=$th step rth$th timeout -k 10 200 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r75/rth$th.log 2>&1
echo REPL TH $th $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r75/rth$th.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r75/rth$th.log)
done
step rdef timeout -k 10 200 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r75/rdef.log 2>&1
echo REPL default $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r75/rdef.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r75/rdef.log)
