source scripts/gpu/guard.sh
mkdir -p gpurun_out/r82
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worms.py tests/test_gpu_villain_local.py tests/test_gpu_worldline_local.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r82/tests.log 2>&1
tail -2 gpurun_out/r82/tests.log
step wb timeout -k 10 300 python bench.py --workload worms --steps 200 --warmup 5 --kappa 1.0 > gpurun_out/r82/worms.log 2>&1
echo WORMS $(grep -o '"value": [0-9.]*' gpurun_out/r82/worms.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r82/worms.log)
