source scripts/gpu/guard.sh
mkdir -p gpurun_out/r61
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r61/tests.log 2>&1
tail -3 gpurun_out/r61/tests.log
step pipe3 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -q --timeout 120 --timeout-method thread -k keepevery > gpurun_out/r61/pipe.log 2>&1
tail -1 gpurun_out/r61/pipe.log
step wbench timeout -k 10 300 python bench.py --workload worms --steps 200 --warmup 5 --kappa 1.0 > gpurun_out/r61/worms.log 2>&1
tail -1 gpurun_out/r61/worms.log | cut -c1-600
