source scripts/gpu/guard.sh
T=${1:-r217}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step wd timeout -k 10 400 python -u -m pytest tests/test_gpu_wdomain.py -x -v --timeout 200 --timeout-method thread > $O/tests_wd.log 2>&1
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests_wd.log | tail -20
step dom timeout -k 10 400 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 200 --timeout-method thread > $O/tests_dom.log 2>&1
tail -2 $O/tests_dom.log
