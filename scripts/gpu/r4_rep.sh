# Round 4: config 5 (1024 x L=128 replicas, W=2, inline observables) with host-paced chunks of 8 sweeps (SV_REP_CHUNK=8,
# the default) vs the whole batch enqueued at once (SV_REP_CHUNK=0): wall and kernel time per sweep, two repetitions.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_rep}
mkdir -p $O
for rep in 1 2; do
  for c in 8 0; do
    SV_REP_CHUNK=$c timeout -k 10 300 python bench.py --workload replicas --no-cpu-baseline > $O/rep_c${c}_$rep.json 2> $O/rep_c${c}_$rep.err || { echo "[rep c=$c] failed"; tail -20 $O/rep_c${c}_$rep.err; exit 3; }
    echo "replicas chunk=$c $rep $(python -c "import json; d=json.load(open('$O/rep_c${c}_$rep.json')); print(round(d['value']/1e9,3), 'G wall', round(d['ms_per_step']*1e3,1), 'kernel', round(d['roofline']['avg_launch_us'],1))")"
  done
done
