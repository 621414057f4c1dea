# A/B: the whole-lattice hot launch's last SV_HOT_WT workgroups store write-through (0 = none)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_hotwt}
mkdir -p $O
step t env SV_HOT_WT=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overflow.py -k headline > $O/tests.log 2>&1
for r in 1 2; do
  for wt in 0 256 512 1024; do
    step h${wt}_$r env SV_HOT_WT=$wt timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_wt${wt}_$r.json 2> $O/head_wt${wt}_$r.err
  done
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"; done
for r in 1 2; do
  for wt in 0 512 1024; do
    step r${wt}_$r env SV_REP_WT=$wt timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_wt${wt}_$r.json 2> $O/rep_wt${wt}_$r.err
  done
done
for f in $O/rep_*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
