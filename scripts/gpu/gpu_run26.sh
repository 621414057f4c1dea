source scripts/gpu/guard.sh
mkdir -p gpurun_out/r26
export TMPDIR=/tmp
step pcs bash -c 'cd /tmp && timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --kernel-include-regex villain_sweep_fused -d $GRAFT_REPO_ROOT/gpurun_out/r26/pcs -o pcs --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r26/pcs.log 2>&1'
tail -5 gpurun_out/r26/pcs.log
find gpurun_out/r26/pcs -type f | head; du -sh gpurun_out/r26/pcs
