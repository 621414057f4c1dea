source scripts/gpu/guard.sh
mkdir -p gpurun_out/r32
export TMPDIR=/tmp
step prof bash -c 'cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r32/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/replica_timing.py 1024 128 0 128 128 0 > $GRAFT_REPO_ROOT/gpurun_out/r32/prof.log 2>&1'
cat gpurun_out/r32/prof.log | grep TH
