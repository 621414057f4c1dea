source scripts/gpu/guard.sh
mkdir -p gpurun_out/r89
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r89/tests.log 2>&1
tail -3 gpurun_out/r89/tests.log
