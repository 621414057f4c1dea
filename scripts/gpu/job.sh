source scripts/gpu/guard.sh
T=${1:-r378}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for w in hammer wlhammer site link exact vortex wrapping worldline; do
step b$w timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-copy-ceiling > $O/b_$w.log 2>&1
grep '^{' $O/b_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', round(d['value']/1e9,3), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2))"
done
