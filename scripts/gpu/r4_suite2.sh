# Full -m gpu suite after the temporal-blocking changes (runtime error log on), smoke, L=256 and headline lines
source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r4_suite2}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -4 $O/tests.log
unset AMD_LOG_LEVEL
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for rep in 1 2; do
  step l256 timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_$rep.json 2> $O/l256_$rep.err
  python -c "import json; d=json.loads(open('$O/l256_$rep.json').readline()); print('l256', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
step head timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err
python -c "import json; d=json.loads(open('$O/driver.json').readline()); print('driver', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
for rep in 1 2; do
  for x in 0 1; do
    step xcd$x env SV_BLOCK_XCD=$x timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_xcd${x}_$rep.json 2> $O/l256_xcd${x}_$rep.err
    python -c "import json; d=json.loads(open('$O/l256_xcd${x}_$rep.json').readline()); print('xcd$x', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  done
done
