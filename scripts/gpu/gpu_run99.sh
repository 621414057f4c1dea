source scripts/gpu/guard.sh
mkdir -p gpurun_out/r99
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r99/tests.log 2>&1
tail -2 gpurun_out/r99/tests.log
