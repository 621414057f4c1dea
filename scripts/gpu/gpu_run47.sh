source scripts/gpu/guard.sh
mkdir -p gpurun_out/r47
export TMPDIR=/tmp
for w in vortex wrapping wlhammer; do
step b$w timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r47/$w.log 2>&1
done
cd /tmp && step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r47/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload wlhammer --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r47/prof.log 2>&1
cd /tmp && step prof2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r47/prof2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload hammer --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r47/prof2.log 2>&1
