# Pinned plan uploads + one-launch snapshots: suites and the worldline / villain bench lines.
source scripts/gpu/guard.sh
O=gpurun_out/r3_up; mkdir -p $O
step t timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_statparity.py > $O/t.log 2>&1
tail -1 $O/t.log
for r in 1 2; do
  step w$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/w$r.json 2> $O/w$r.err
  python -c "import json; d=json.loads(open('$O/w$r.json').readline()); print('wl', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"
  step d$r timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d$r.json 2> $O/d$r.err
  python -c "import json; d=json.loads(open('$O/d$r.json').readline()); print('driver', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
done
