source scripts/gpu/guard.sh
mkdir -p gpurun_out/r111
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_villain_local.py tests/test_gpu_worldline_local.py tests/test_gpu_worldline.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r111/tests.log 2>&1
tail -1 gpurun_out/r111/tests.log
step h timeout -k 10 300 python bench.py --workload hammer --no-cpu-baseline --steps 100 > gpurun_out/r111/h.log 2>&1
echo HAMMER $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r111/h.log)
step w timeout -k 10 300 python bench.py --workload wlhammer --no-cpu-baseline --steps 100 > gpurun_out/r111/w.log 2>&1
echo WLHAMMER $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r111/w.log)
