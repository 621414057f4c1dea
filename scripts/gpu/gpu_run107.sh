source scripts/gpu/guard.sh
mkdir -p gpurun_out/r107
export TMPDIR=/tmp
step bench timeout -k 10 400 python bench.py > gpurun_out/r107/bench.log 2>&1
tail -1 gpurun_out/r107/bench.log > profiles/r01_bench.json
step prof timeout -k 10 1000 bash scripts/profile.sh r01 > gpurun_out/r107/profile.log 2>&1
step t timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r107/tests.log 2>&1
tail -1 gpurun_out/r107/tests.log
