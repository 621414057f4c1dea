source scripts/gpu/guard.sh
mkdir -p gpurun_out/r23
export TMPDIR=/tmp
step tests bash -c 'timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r23/tests.log 2>&1'
tail -15 gpurun_out/r23/tests.log
step bench1 bash -c 'timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r23/bench1.log 2>&1'
tail -1 gpurun_out/r23/bench1.log | cut -c1-300
grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r23/bench1.log
step reps bash -c 'timeout -k 10 300 python scripts/replica_timing.py > gpurun_out/r23/reps.log 2>&1'
cat gpurun_out/r23/reps.log
