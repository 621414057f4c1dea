# Kernel trace of the rejection window (where a rejection's cost goes)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_rtrace}
mkdir -p $O
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python -u scripts/perf/reject_window.py 4096 20 60 > $O/trace.log 2>&1
tail -2 $O/trace.log
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python scripts/perf/reject_trace.py $f > $O/reject_trace.txt 2>&1
cat $O/reject_trace.txt
rm -f $f
