# bench.py after the roofline fallback: replicas twice, the headline driver form once, L=256 once
source scripts/gpu/guard.sh
O=gpurun_out/r4_benchcheck
mkdir -p $O
for w in "rep1:--workload replicas" "rep2:--workload replicas" "drv:--gpus 1 --steps 20 --warmup 5" "l256:--L 256"; do
  n=${w%%:*}; a=${w#*:}
  step $n timeout -k 10 300 python -u bench.py $a > $O/$n.json 2> $O/$n.err
  python -c "import json; d=json.loads(open('$O/$n.json').readline()); print('$n', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us', d['roofline'].get('launch_time_source'), d['cpu_baseline'] is not None)"
done
