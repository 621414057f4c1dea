source scripts/gpu/guard.sh
mkdir -p gpurun_out/r43
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r43/tests.log 2>&1
tail -3 gpurun_out/r43/tests.log
step bench timeout -k 10 300 python bench.py > gpurun_out/r43/bench.log 2>&1
tail -1 gpurun_out/r43/bench.log
