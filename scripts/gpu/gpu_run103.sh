source scripts/gpu/guard.sh
mkdir -p gpurun_out/r103
for rep in 1 2; do
for v in base old; do
if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so; fi
step w$v timeout -k 10 300 python bench.py --workload wlhammer --no-cpu-baseline --steps 100 > gpurun_out/r103/w$v.log 2>&1
echo WLHAMMER $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r103/w$v.log)
done
done
unset SV_LIB_OVERRIDE
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline_local.py tests/test_gpu_worldline.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r103/tests.log 2>&1
tail -1 gpurun_out/r103/tests.log
