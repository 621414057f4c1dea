source scripts/gpu/guard.sh
mkdir -p gpurun_out/r62
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r62/tests.log 2>&1
tail -3 gpurun_out/r62/tests.log
step rej timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r62/rej_split.log 2>&1
cat gpurun_out/r62/rej_split.log
SV_DOMAIN_SPLIT=0 step rej0 timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r62/rej_nosplit.log 2>&1
cat gpurun_out/r62/rej_nosplit.log
step b11 timeout -k 10 300 python bench.py --tiles 1x1 --no-cpu-baseline > gpurun_out/r62/b11.log 2>&1
tail -1 gpurun_out/r62/b11.log | cut -c1-400
