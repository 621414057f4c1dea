# Round 6: the two-rejection split replay failure (scripts/perf/split_two_dbg.py), config 3 with the per-workgroup
# stats flush (default now) vs the exact words in registers (wfwg1) and no words (wfwg2, timing only), and the host
# phases of a rejection at L=256
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_dbg
mkdir -p $O
V=supervillain_amd/variants
step dbg timeout -k 10 300 python -u scripts/perf/split_two_dbg.py > $O/split_two.log 2>&1
cat $O/split_two.log
for r in 1 2; do
  for v in r5base wfwg1 wfwg2; do
    step $v$r env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_${v}_$r.json 2> $O/wl_${v}_$r.err
  done
  step new$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
done
step rej env SV_DEBUG_TIMING=1 timeout -k 10 200 python -u scripts/perf/reject_cost_small.py 256 200 3 100 > $O/rej_dbg.log 2>&1
tail -60 $O/rej_dbg.log
for f in $O/*.json; do python scripts/summ_line.py $f; done
