source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_t1
mkdir -p $O
step dbg env SV_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/perf/split_two_dbg.py > $O/split_two.log 2>&1
grep -v "^\[sv\] plan\|^\[sv\] launch" $O/split_two.log
step t timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_domain.py tests/test_gpu_block.py tests/test_gpu_band.py tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_worldline.py tests/test_gpu_wdomain.py tests/test_gpu_wf_layout.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
tail -5 $O/tests.log
