# Round 6: the headline's per-XCD strip schedule (SV_STRIPS, heights per 512-row XCD band) -- the default
# "57x5,41x5,22" against three other descending lists, interleaved, 200 sweeps each
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_strips
mkdir -p $O
for r in 1 2 3; do
  i=0
  for s in "57x5,41x5,22" "61x4,45x4,25x3,13" "57x6,37x4,22" "49x6,41x4,21,17,16"; do
    i=$((i+1))
    step s$i$r env SV_STRIPS=$s timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/s${i}_$r.json 2> $O/s${i}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
