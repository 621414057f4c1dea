source scripts/gpu/guard.sh
T=${1:-r350}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
