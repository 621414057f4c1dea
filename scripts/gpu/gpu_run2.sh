set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 1200 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== trace"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -3 gpurun_out/bench_trace.log
if [ $rc -ne 0 ]; then exit $rc; fi
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
echo done
