# Host phases of the L=256 bench call (SV_DEBUG_TIMING: plan, launch, wait per batch), two runs
source scripts/gpu/guard.sh
O=gpurun_out/r4_l256dbg
mkdir -p $O
for rep in 1 2; do
  step dbg env SV_DEBUG_TIMING=1 timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_$rep.json 2> $O/l256_$rep.err
  python -c "import json; d=json.loads(open('$O/l256_$rep.json').readline()); print('l256', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  grep "\[sv\]" $O/l256_$rep.err | tail -8
done
