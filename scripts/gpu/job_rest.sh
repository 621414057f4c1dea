# GPU tests in two passes: everything but the statistical comparisons, then those alone.
source scripts/gpu/guard.sh
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
step rest timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_statparity.py > $O/rest.log 2>&1
grep -E "FAILED|ERROR|passed|failed" $O/rest.log | tail -20
step stat timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_statparity.py > $O/stat.log 2>&1
grep -E "N=|FAILED|passed|failed" $O/stat.log | tail -30
