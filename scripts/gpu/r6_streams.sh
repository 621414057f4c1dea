# Round 6: config 5 (1024 x L=128 replicas, inline observables) by the number of part-batches on their own streams
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_streams
mkdir -p $O
for r in 1 2; do
  for s in 2 3 4 1; do
    step s$s$r timeout -k 10 120 python -u bench.py --workload replicas --streams $s --no-cpu-baseline --no-copy-ceiling > $O/rep_s${s}_$r.json 2> $O/rep_s${s}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
