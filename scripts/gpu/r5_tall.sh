# one round of tall strips (SV_STRIPS=uniform SV_FUSED_TH=h) vs the default band_strips schedule, L=4096 headline
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tall}
mkdir -p $O
for r in 1 2; do
  step base$r timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/base_$r.json 2> $O/base_$r.err
  for h in 137 121 105 69; do
    step t$h$r env SV_STRIPS=uniform SV_FUSED_TH=$h timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/th${h}_$r.json 2> $O/th${h}_$r.err
  done
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"; done
