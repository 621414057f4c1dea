source scripts/gpu/guard.sh
mkdir -p gpurun_out/r30
export TMPDIR=/tmp
step tests bash -c 'timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r30/tests.log 2>&1'
tail -2 gpurun_out/r30/tests.log
step bench bash -c 'timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r30/bench.log 2>&1'
grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r30/bench.log
step reps bash -c 'timeout -k 10 300 python scripts/replica_timing.py > gpurun_out/r30/reps.log 2>&1'
cat gpurun_out/r30/reps.log
