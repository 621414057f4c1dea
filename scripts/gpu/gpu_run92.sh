source scripts/gpu/guard.sh
mkdir -p gpurun_out/r92
for rep in 1 2; do
for v in base nok3; do
if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so; fi
step $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r92/$v.log 2>&1
echo VAR $v $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r92/$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r92/$v.log)
done
done
unset SV_LIB_OVERRIDE
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_domain.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r92/tests.log 2>&1
tail -1 gpurun_out/r92/tests.log
