# Round 6: nontemporal row loads (variants/libsvhip_ntl.so) and row stores (libsvhip_nts.so) in villain_sweep_hot on
# the whole L=4096 lattice, against the tree, interleaved
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_nt
mkdir -p $O
V=supervillain_amd/variants
for r in 1 2 3; do
  step b$r timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  for v in ntl nts; do
    step $v$r env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/${v}_$r.json 2> $O/${v}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
