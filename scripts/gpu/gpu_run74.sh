source scripts/gpu/guard.sh
mkdir -p gpurun_out/r74
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r74/tests.log 2>&1
tail -2 gpurun_out/r74/tests.log
step bench timeout -k 10 300 python bench.py > gpurun_out/r74/bench.log 2>&1
grep -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r74/bench.log | head -3
step prof timeout -k 10 1000 bash scripts/profile.sh r01 > gpurun_out/r74/profile.log 2>&1
tail -3 gpurun_out/r74/profile.log
