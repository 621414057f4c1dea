source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_split5}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split.py tests/test_gpu_villain.py tests/test_gpu_overflow.py > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
step stl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 200 python -u scripts/perf/split_timeline.py 0.37 > $O/stl.log 2>&1
cat $O/stl.log
step rw timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window.log 2>&1
cat $O/reject_window.log
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python -u scripts/perf/reject_window.py 4096 20 60 > $O/trace.log 2>&1
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python scripts/perf/reject_trace.py $f > $O/reject_trace.txt 2>&1
tail -4 $O/reject_trace.txt
rm -f $f
