# Round-5 baseline on a fresh box: the -m gpu suite, the driver-form line, the rejection-window cost
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_base}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
unset AMD_LOG_LEVEL
step head timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err
python -c "import json; d=json.loads(open('$O/driver.json').readline()); print('driver', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
step rw timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window.log 2>&1
cat $O/reject_window.log
