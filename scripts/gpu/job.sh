source scripts/gpu/guard.sh
T=${1:-r367}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
for nw in 4 8; do
SV_SIZES=2048x1024 SV_HOT_NW=$nw step d$nw timeout -k 10 300 python scripts/perf/deep_halo.py 4 > $O/d${nw}_$rep.log 2>&1
grep us/sweep $O/d${nw}_$rep.log | sed "s/^/nw$nw /"
done
done
