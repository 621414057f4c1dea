# Replicas trace (wall vs kernel gaps) and the weak-scaling layouts emulated on one GPU
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_rep_weak}
mkdir -p $O
step reptr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rtrace -o run --output-format csv -- python -u bench.py --workload replicas --no-cpu-baseline > $O/rtrace.log 2>&1
f=$(find $O/rtrace -name "run_kernel_trace.csv" | head -1)
python scripts/perf/idle_gaps.py $f villain_sweep_hot_fr 16 > $O/rep_idle.txt 2>&1
cat $O/rep_idle.txt
rm -f $f
step w11 timeout -k 10 300 python -u bench.py --tiles 1x1 --weak --steps 20 --warmup 5 --no-cpu-baseline > $O/w11.json 2> $O/w11.err
python -c "import json; d=json.loads(open('$O/w11.json').readline()); print('weak 1x1', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling'])"
step s24 timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 20 --warmup 5 --no-cpu-baseline > $O/s24.json 2> $O/s24.err
python -c "import json; d=json.loads(open('$O/s24.json').readline()); print('strong 2x4', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling'])"
step w24 timeout -k 10 600 python -u bench.py --tiles 2x4 --weak --steps 10 --warmup 3 --warmup-s 0 --no-cpu-baseline > $O/w24.json 2> $O/w24.err
python -c "import json; d=json.loads(open('$O/w24.json').readline()); print('weak 2x4', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling'])"
