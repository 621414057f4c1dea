source scripts/gpu/guard.sh
mkdir -p gpurun_out/r84
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r84/tests.log 2>&1
tail -2 gpurun_out/r84/tests.log
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r84/prof -o run --output-format csv -- python bench.py --workload worms --steps 200 --warmup 5 --kappa 1.0 --no-cpu-baseline > gpurun_out/r84/prof.log 2>&1
step wb timeout -k 10 300 python bench.py --workload worms --steps 200 --warmup 5 --kappa 1.0 > gpurun_out/r84/worms.log 2>&1
step repl timeout -k 10 300 python bench.py --workload replicas > gpurun_out/r84/repl.log 2>&1
step wl timeout -k 10 300 python bench.py --workload worldline > gpurun_out/r84/wl.log 2>&1
