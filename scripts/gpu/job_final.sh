# End-of-session check: full GPU suite, smoke, driver-form bench lines (3x), the 200-sweep default and the config lines.
# Usage: bash scripts/gpu/job_final.sh TAG
source scripts/gpu/guard.sh
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for r in 1 2 3; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err
  python -c "import json; d=json.loads(open('$O/driver_$r.json').readline()); print('driver', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
done
step def timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err
python -c "import json; d=json.loads(open('$O/default.json').readline()); print('default', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
