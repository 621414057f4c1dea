source scripts/gpu/guard.sh
mkdir -p gpurun_out/r22
export TMPDIR=/tmp
step domain bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_domain.py -x -q > gpurun_out/r22/domain.log 2>&1'
tail -15 gpurun_out/r22/domain.log
step torchfirst bash -c 'NCCL_DEBUG=WARN timeout -k 10 200 python scripts/check_torch_first.py > gpurun_out/r22/torchfirst.log 2>&1'
tail -15 gpurun_out/r22/torchfirst.log
step prof bash -c 'cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r22/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --tiles 1x2 --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r22/prof.log 2>&1'
tail -3 gpurun_out/r22/prof.log
find gpurun_out/r22/prof -name "*stats*"
