source scripts/gpu/guard.sh
T=${1:-r331}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step brep timeout -k 10 300 python bench.py --workload replicas > $O/b_replicas.log 2>&1
grep '^{' $O/b_replicas.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rep', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3))"
step prep timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rep -o rep -- python bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/prof_rep.log 2>&1
step pph timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ph -o ph -- python bench.py --rng philox --no-cpu-baseline --no-copy-ceiling > $O/prof_ph.log 2>&1
find $O -name '*kernel_stats.csv'
