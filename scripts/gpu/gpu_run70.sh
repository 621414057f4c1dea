source scripts/gpu/guard.sh
mkdir -p gpurun_out/r70
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r70/tests.log 2>&1
tail -2 gpurun_out/r70/tests.log
step batch timeout -k 10 900 python scripts/perf/domain_batch.py > gpurun_out/r70/batch.log 2>&1
grep batch gpurun_out/r70/batch.log
