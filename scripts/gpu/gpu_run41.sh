source scripts/gpu/guard.sh
export TMPDIR=/tmp
step profile bash -c 'bash scripts/profile.sh r01 > gpurun_out/profile_r01.log 2>&1'
step bench bash -c 'timeout -k 10 400 python bench.py > gpurun_out/prof_r01/bench.log 2>&1'
tail -1 gpurun_out/prof_r01/bench.log | cut -c1-200
