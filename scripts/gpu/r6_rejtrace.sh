# Round 6: kernel trace of forced rejections at L=256 (config 2), for the timeline around each replay
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_rejtrace
mkdir -p $O
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python scripts/perf/reject_cost_small.py 256 200 3 100 > $O/tr.log 2>&1
tail -2 $O/tr.log
f=$(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1)
python scripts/perf/reject_trace_small.py $f 12 4 > $O/timeline.txt
head -60 $O/timeline.txt
