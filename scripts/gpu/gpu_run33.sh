source scripts/gpu/guard.sh
mkdir -p gpurun_out/r33
export TMPDIR=/tmp
step tests bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_replicas.py -x -q > gpurun_out/r33/tests.log 2>&1'
tail -2 gpurun_out/r33/tests.log
step reps bash -c 'timeout -k 10 300 python scripts/replica_timing.py > gpurun_out/r33/reps.log 2>&1'
cat gpurun_out/r33/reps.log
