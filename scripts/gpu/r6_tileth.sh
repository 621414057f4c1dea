# Round 6: where the decomposed tiles lose against the single lattice -- the whole L=4096 lattice as one tile (1x1,
# the tile path) against the single-lattice path, and the N = 2 tile (4096 x 2048) by strip height (SV_FUSED_TH;
# default 37 rows = 1.84 rounds of the slots), 100 sweeps each, prediction on (no aborts in the windows)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
export SV_DOMAIN_PREDICT=1
O=gpurun_out/r6_tileth
mkdir -p $O
for r in 1 2; do
  step s$r timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-copy-ceiling > $O/single_$r.json 2> $O/single_$r.err
  step t11$r timeout -k 10 150 python -u bench.py --tiles 1x1 --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t1x1_$r.json 2> $O/t1x1_$r.err
  step t12$r timeout -k 10 150 python -u bench.py --tiles 1x2 --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t1x2_$r.json 2> $O/t1x2_$r.err
  for th in 53 45 29 21; do
    step t12_$th$r env SV_FUSED_TH=$th timeout -k 10 150 python -u bench.py --tiles 1x2 --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t1x2_th${th}_$r.json 2> $O/t1x2_th${th}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
