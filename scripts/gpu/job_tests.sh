# Selected GPU tests.  Usage: bash scripts/gpu/job_tests.sh TAG pytest-args...
source scripts/gpu/guard.sh
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/tests.log 2>&1
tail -25 $O/tests.log
