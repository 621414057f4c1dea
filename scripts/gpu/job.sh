source scripts/gpu/guard.sh
T=${1:-r363}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -q -k "other_choice or predicted" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -15 $O/tests.log
