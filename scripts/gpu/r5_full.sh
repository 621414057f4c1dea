# Full -m gpu suite (runtime error log on), smoke, the driver-form headline, the rejection window
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_full4}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for r in 1 2; do
step head timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err
python -c "import json; d=json.loads(open('$O/driver_$r.json').readline()); print('driver', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
done
step rw timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window.log 2>&1
cut -c1-250 $O/reject_window.log
