# split_order as a slot permutation: the split suites (incl. the N=2048 head-slot regression), domain tiles, Villain
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_splitfix}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_domain.py tests/test_gpu_villain.py tests/test_gpu_overflow.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
