source scripts/gpu/guard.sh
mkdir -p gpurun_out/r48
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline_local.py tests/test_gpu_villain_local.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r48/tests.log 2>&1
tail -3 gpurun_out/r48/tests.log
for w in site link exact cohomology hammer vortex wrapping wlhammer; do
step b$w timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r48/$w.log 2>&1
done
cd /tmp && step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r48/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload wlhammer --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r48/prof.log 2>&1
cd /tmp && step prof2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r48/prof2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload hammer --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r48/prof2.log 2>&1
