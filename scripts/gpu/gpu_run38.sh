source scripts/gpu/guard.sh
mkdir -p gpurun_out/r38
export TMPDIR=/tmp
step wltests bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_worldline.py -x -q > gpurun_out/r38/wltests.log 2>&1'
tail -5 gpurun_out/r38/wltests.log
step wl bash -c 'timeout -k 10 300 python bench.py --workload worldline --steps 100 --warmup 5 > gpurun_out/r38/wl.log 2>&1'
grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r38/wl.log
