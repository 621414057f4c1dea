set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== debug plaq"; timeout -k 10 120 python scripts/debug_plaquette.py 32 1 > gpurun_out/debug_plaq.log 2>&1; echo "rc=$?"; cat gpurun_out/debug_plaq.log | tail -20
echo "== pytest villain"; timeout -k 10 900 python -m pytest tests/test_gpu_villain.py -m gpu -q -x --timeout 600 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== trace"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace3 -o run --output-format csv -- python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; grep metric gpurun_out/bench_trace.log | cut -c1-600
