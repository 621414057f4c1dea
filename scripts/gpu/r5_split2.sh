source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_split2}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split.py tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_boundary.py tests/test_gpu_pipeline.py tests/test_gpu_table_purge.py > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
step rw timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window.log 2>&1
cat $O/reject_window.log
step head timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver.json 2> $O/driver.err
python -c "import json; d=json.loads(open('$O/driver.json').readline()); print('driver', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python -u scripts/perf/reject_window.py 4096 20 60 > $O/trace.log 2>&1
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python scripts/perf/reject_trace.py $f > $O/reject_trace.txt 2>&1
tail -4 $O/reject_trace.txt
rm -f $f
