source scripts/gpu/guard.sh
mkdir -p gpurun_out/r35
export TMPDIR=/tmp
step wl bash -c 'timeout -k 10 300 python bench.py --workload worldline --steps 20 --warmup 2 > gpurun_out/r35/wl.log 2>&1'
tail -1 gpurun_out/r35/wl.log
step reps bash -c 'timeout -k 10 300 python bench.py --workload replicas --steps 100 --warmup 5 > gpurun_out/r35/reps.log 2>&1'
tail -1 gpurun_out/r35/reps.log
step wltests bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_worldline.py -x -q > gpurun_out/r35/wltests.log 2>&1'
tail -2 gpurun_out/r35/wltests.log
