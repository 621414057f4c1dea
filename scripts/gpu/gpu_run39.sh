source scripts/gpu/guard.sh
mkdir -p gpurun_out/r39
export TMPDIR=/tmp
step profile bash -c 'bash scripts/profile.sh r01 > gpurun_out/r39/profile.log 2>&1'
tail -30 gpurun_out/r39/profile.log
step bench bash -c 'timeout -k 10 400 python bench.py > gpurun_out/r39/bench.log 2>&1'
tail -1 gpurun_out/r39/bench.log
