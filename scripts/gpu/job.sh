source scripts/gpu/guard.sh
T=${1:-r321}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_worms.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for rep in 1 2; do
step brep timeout -k 10 300 python bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/brep_$rep.log 2>&1
grep '^{' $O/brep_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('replicas', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
SV_DEBUG_TIMING=1 step dbg timeout -k 10 300 python bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/dbg.log 2>&1
grep 'sv replicas' $O/dbg.log | tail -8
