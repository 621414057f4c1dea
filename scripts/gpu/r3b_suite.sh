# The full -m gpu suite on the current tree.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_suite
mkdir -p $O
step tests timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
