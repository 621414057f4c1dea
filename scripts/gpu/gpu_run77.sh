source scripts/gpu/guard.sh
mkdir -p gpurun_out/r77
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_worms.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r77/tests.log 2>&1
tail -2 gpurun_out/r77/tests.log
for rep in 1 2; do
step new timeout -k 10 200 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r77/new.log 2>&1
echo NEW $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r77/new.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r77/new.log)
SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_nofr.so step old timeout -k 10 200 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r77/old.log 2>&1
echo OLD $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r77/old.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r77/old.log)
done
