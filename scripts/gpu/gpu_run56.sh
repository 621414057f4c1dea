source scripts/gpu/guard.sh
mkdir -p gpurun_out/r56
export TMPDIR=/tmp
step prof timeout -k 10 1200 bash scripts/profile.sh r01 > gpurun_out/r56/profile.log 2>&1
tail -5 gpurun_out/r56/profile.log
step bench timeout -k 10 300 python bench.py > gpurun_out/r56/bench.log 2>&1
tail -1 gpurun_out/r56/bench.log
