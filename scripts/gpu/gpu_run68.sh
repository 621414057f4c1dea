source scripts/gpu/guard.sh
mkdir -p gpurun_out/r68 profiles
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worms.py tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r68/tests.log 2>&1
tail -3 gpurun_out/r68/tests.log
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r68/prof -o run --output-format csv -- python bench.py --workload worms --steps 200 --warmup 5 --kappa 1.0 --no-cpu-baseline > gpurun_out/r68/prof.log 2>&1
cp gpurun_out/r68/prof/run_kernel_stats.csv profiles/r01_kernel_stats_worms.csv
tail -1 gpurun_out/r68/prof.log > profiles/r01_bench_worms.json
