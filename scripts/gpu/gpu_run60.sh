source scripts/gpu/guard.sh
mkdir -p gpurun_out/r60
step build_check true
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worms.py tests/test_gpu_pipeline.py tests/test_gpu_villain_local.py tests/test_gpu_worldline_local.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r60/tests.log 2>&1
tail -5 gpurun_out/r60/tests.log
step wbench timeout -k 10 300 python bench.py --workload worms --steps 20 --warmup 2 > gpurun_out/r60/worms.log 2>&1
tail -2 gpurun_out/r60/worms.log
