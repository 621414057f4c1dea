source scripts/gpu/guard.sh
T=${1:-r218}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step wd timeout -k 10 400 python -u -m pytest tests/test_gpu_wdomain.py -x -q --timeout 200 --timeout-method thread > $O/tests_wd.log 2>&1
tail -2 $O/tests_wd.log
for t in 1x2 2x4; do
step bt$t timeout -k 10 300 python bench.py --workload worldline --tiles $t --steps 100 --warmup 10 --no-cpu-baseline --no-copy-ceiling > $O/bwl_$t.log 2>&1
grep '^{' $O/bwl_$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value']/1e9, d['roofline']['avg_launch_us'], d['config']['weak_scaling'])"
done
