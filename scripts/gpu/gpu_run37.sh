source scripts/gpu/guard.sh
mkdir -p gpurun_out/r37
export TMPDIR=/tmp
step prof bash -c 'cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r37/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload worldline --steps 20 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r37/prof.log 2>&1'
