source scripts/gpu/guard.sh
mkdir -p gpurun_out/r109
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r109/tests.log 2>&1
tail -1 gpurun_out/r109/tests.log
for rep in 1 2; do
for v in base old; do
if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so; fi
step h$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 640 > gpurun_out/r109/h$v$rep.log 2>&1
echo HEAD $v $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/r109/h$v$rep.log)
done
done
