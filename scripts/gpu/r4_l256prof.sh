# Config 2 kernel-trace summary (rocprofv3 --kernel-trace --stats) of the L=256 bench, and three more driver-form lines
source scripts/gpu/guard.sh
O=gpurun_out/r4_l256prof
mkdir -p $O
export TMPDIR=/tmp
step trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --L 256 --no-cpu-baseline > $O/trace.log 2>&1
for r in 1 2 3; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_$r.json 2> $O/driver_$r.err
  python -c "import json; d=json.loads(open('$O/driver_$r.json').readline()); print('driver', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
done
