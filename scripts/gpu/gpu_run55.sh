source scripts/gpu/guard.sh
mkdir -p gpurun_out/r55
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r55/tests.log 2>&1
tail -15 gpurun_out/r55/tests.log
