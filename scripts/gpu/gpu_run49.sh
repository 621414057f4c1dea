source scripts/gpu/guard.sh
mkdir -p gpurun_out/r49
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r49/tests.log 2>&1
tail -3 gpurun_out/r49/tests.log
for w in worldline wlhammer vortex; do
step b$w timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r49/$w.log 2>&1
done
cd /tmp && step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r49/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload wlhammer --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r49/prof.log 2>&1
cd /tmp && step prof2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r49/prof2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload worldline --steps 50 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r49/prof2.log 2>&1
