source scripts/gpu/guard.sh
T=${1:-r312}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SV_DEBUG_TIMING=1 step dbg timeout -k 10 200 python bench.py --steps 640 --warmup 5 --no-cpu-baseline --no-copy-ceiling --warmup-s 1 > $O/dbg.log 2>&1
grep '^{' $O/dbg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('d640', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['avg_launch_us'],1), d['config'].get('lemire_rejections_in_timed_steps'))"
grep '\[sv\]' $O/dbg.log | tail -40
