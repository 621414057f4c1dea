source scripts/gpu/guard.sh
mkdir -p gpurun_out/r86
for rep in 1 2; do
for v in base ilp lat o2 wprio bias; do
if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so; fi
step $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r86/$v.log 2>&1
echo VAR $v $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r86/$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r86/$v.log)
done
done
