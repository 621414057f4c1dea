source scripts/gpu/guard.sh
T=${1:-r307}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for w in hammer wlhammer; do
step b$w timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/b_$w.log 2>&1
grep '^{' $O/b_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
