# Config 5 timeline: a kernel trace of the replicas bench (idle gaps around NumPy Lemire aborts) + host debug timing.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_reptrace
mkdir -p $O
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/trace.log 2>&1
python scripts/perf/idle_gaps.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) villain_sweep_hot_fr 15
SV_DEBUG_TIMING=1 step dbg timeout -k 10 200 python -u bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/dbg.json 2> $O/dbg.err
tail -12 $O/dbg.err
