set -u
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== pytest"; timeout -k 10 1200 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench"; timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
