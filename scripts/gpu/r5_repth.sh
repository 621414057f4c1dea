# config 5 strip height A/B: 64-row tiles (default, 2048 workgroups) vs whole-replica strips (SV_FUSED_TH=128)
source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r5_repth}
mkdir -p $O
for r in 1 2; do
  step d$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/th64_$r.json 2> $O/th64_$r.err
  step t$r env SV_FUSED_TH=128 timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/th128_$r.json 2> $O/th128_$r.err
  step u$r env SV_FUSED_TH=96 timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/th96_$r.json 2> $O/th96_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
