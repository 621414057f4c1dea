# End-of-session evidence: full -m gpu suite, smoke, headline trace + PMC (scripts/profile.sh r03b), bench lines.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_final
mkdir -p $O/bench
step tests timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -2 $O/tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2 3; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench/driver_$r.json 2> $O/bench/driver_$r.err
done
step def timeout -k 10 300 python -u bench.py > $O/bench/default.json 2> $O/bench/default.err
step wl timeout -k 10 300 python -u bench.py --workload worldline > $O/bench/worldline.json 2> $O/bench/worldline.err
step l256 timeout -k 10 300 python -u bench.py --L 256 > $O/bench/l256.json 2> $O/bench/l256.err
step rep timeout -k 10 300 python -u bench.py --workload replicas > $O/bench/replicas.json 2> $O/bench/replicas.err
step t8 timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles2x4.json 2> $O/bench/tiles2x4.err
step prof timeout -k 10 900 bash scripts/profile.sh r03b
for f in $O/bench/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3), d['config'].get('lemire_rejections_in_timed_steps'))"; done
