# Round 6: config 4's tile layouts in one-GPU emulation -- for N = 8 the 2x4 default (2048 x 1024 tiles, 9 strip
# columns of which 2 at the tile's edges) against 8x1 (512 x 4096: 34 strip columns, 2 at the edges), 4x2, 1x8; for
# N = 4 2x2 against 4x1; for N = 2 1x2 against 2x1.  Per-tile kernel time = the launch average.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_layout
mkdir -p $O
for r in 1 2; do
  for t in 2x4 8x1 4x2 1x8 2x2 4x1 1x2 2x1; do
    step t$t$r timeout -k 10 150 python -u bench.py --tiles $t --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t${t}_$r.json 2> $O/t${t}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
