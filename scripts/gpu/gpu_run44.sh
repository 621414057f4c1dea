source scripts/gpu/guard.sh
mkdir -p gpurun_out/r44
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline_local.py tests/test_gpu_villain_local.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r44/tests.log 2>&1
tail -25 gpurun_out/r44/tests.log
