# Round 4: where the driver form's wall-to-kernel gap goes -- host-side batch timing (SV_DEBUG_TIMING) and a kernel +
# memory-copy trace of `bench.py --gpus 1 --steps 20 --warmup 5`, summarised by scripts/perf/gap_summary.py.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_gap}
mkdir -p $O
SV_DEBUG_TIMING=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_dbg.json 2> $O/drv_dbg.err || { echo "[drv dbg] failed"; tail -20 $O/drv_dbg.err; exit 3; }
grep "\[sv\]" $O/drv_dbg.err | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o t --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "[trace] failed"; tail -20 $O/trace.log; exit 3; }
python scripts/perf/gap_summary.py $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace_rep -o t --output-format csv -- python bench.py --workload replicas --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_rep.log 2>&1 || { echo "[trace rep] failed"; tail -20 $O/trace_rep.log; exit 3; }
python scripts/perf/gap_summary.py $O/trace_rep villain_sweep 10
