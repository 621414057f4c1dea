# final tree confirmation: full -m gpu suite, smoke, the default bench line and config 3
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_confirm}
mkdir -p $O
step tests timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step def timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err
step wl timeout -k 10 300 python -u bench.py --workload worldline > $O/worldline.json 2> $O/worldline.err
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['roofline']['frac'])"; done
