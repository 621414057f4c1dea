# Round 6: R1 and the single-lattice reference timed over max(--steps, 100) sweeps -- the tile emulations again
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_r1
mkdir -p $O
for r in 1 2; do
  for t in 1x2 2x2 2x4; do
    step t$t$r timeout -k 10 150 python -u bench.py --tiles $t --steps 40 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t${t}_$r.json 2> $O/t${t}_$r.err
  done
done
step w timeout -k 10 200 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 3 --no-cpu-baseline --no-copy-ceiling > $O/t2x4w.json 2> $O/t2x4w.err
step wl timeout -k 10 150 python -u bench.py --workload worldline --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/wl2x4.json 2> $O/wl2x4.err
for f in $O/*.json; do python scripts/summ_line.py $f; done
