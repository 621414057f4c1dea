source scripts/gpu/guard.sh
mkdir -p gpurun_out/r95
export TMPDIR=/tmp
step prof timeout -k 10 1000 bash scripts/profile.sh r01 > gpurun_out/r95/profile.log 2>&1
