source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_rep2}
mkdir -p $O
step rep env AMD_LOG_LEVEL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_replicas.py tests/test_gpu_observables.py > $O/rep.log 2>&1
tail -2 $O/rep.log
grep -E "[0-9]+ passed" $O/rep.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/rep.log > /dev/null || { echo "[rep] not green"; exit 1; }
for r in 1 2; do
step repb timeout -k 10 300 python -u bench.py --workload replicas --no-cpu-baseline > $O/replicas_$r.json 2> $O/replicas_$r.err
python -c "import json; d=json.loads(open('$O/replicas_$r.json').readline()); print('replicas', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
step reptr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rtrace -o run --output-format csv -- python -u bench.py --workload replicas --no-cpu-baseline > $O/rtrace.log 2>&1
f=$(find $O/rtrace -name "run_kernel_trace.csv" | head -1)
python scripts/perf/idle_gaps.py $f villain_sweep_hot_fr 10 > $O/rep_idle.txt 2>&1
cat $O/rep_idle.txt
rm -f $f
step w24p env SV_DOMAIN_PREDICT=1 timeout -k 10 600 python -u bench.py --tiles 2x4 --weak --steps 10 --warmup 3 --warmup-s 0 --no-cpu-baseline > $O/w24p.json 2> $O/w24p.err
python -c "import json; d=json.loads(open('$O/w24p.json').readline()); print('weak 2x4 predicted', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling']['E_N'])"
