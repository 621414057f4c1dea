source scripts/gpu/guard.sh
T=${1:-r356}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step brep timeout -k 10 300 python bench.py --workload replicas > $O/b_replicas.log 2>&1
grep '^{' $O/b_replicas.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3))"
step brep2 timeout -k 10 300 python bench.py --workload replicas --steps 1000 --no-cpu-baseline > $O/b_replicas1000.log 2>&1
grep "^{" $O/b_replicas1000.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep1000', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2))"
step prep timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rep -o rep --output-format csv -- python bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/prof_rep.log 2>&1
head -3 $O/prof_rep/rep_kernel_stats.csv
