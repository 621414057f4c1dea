source scripts/gpu/guard.sh
T=${1:-r206}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step villain timeout -k 10 400 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_boundary.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests_villain.log 2>&1
tail -3 $O/tests_villain.log
step all timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_all.log 2>&1
tail -3 $O/tests_all.log
step bench timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.log 2>&1
grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"lemire_rejections_in_timed_steps": [0-9]*' $O/bench.log
step bench256 timeout -k 10 300 python bench.py --L 256 --steps 2000 --warmup 100 --no-cpu-baseline --no-copy-ceiling > $O/bench256.log 2>&1
grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*' $O/bench256.log
