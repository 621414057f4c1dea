# Round 6: one-level exact acceptance sums on the device (common.h): the full -m gpu suite; then the headline and
# worldline (config 3) lines of the tree, of round 5's kernels (variants/libsvhip_r5base.so) and of mad128 as 64-bit
# column accumulators (variants/libsvhip_mad1.so, -DSV_MAD128=1: 356 -> 322 VALU in the headline loop), interleaved;
# config 5; the 2x4 tile emulation with rejection prediction on (as 8 ranks run it) against the one-process default
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_one
mkdir -p $O
V=supervillain_amd/variants
step suite timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
for r in 1 2; do
  step hn$r timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/head_new_$r.json 2> $O/head_new_$r.err
  for v in r5base mad1; do
    step h$v$r env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/head_${v}_$r.json 2> $O/head_${v}_$r.err
  done
  step wn$r timeout -k 10 120 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
  for v in r5base mad1; do
    step w$v$r env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 120 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_${v}_$r.json 2> $O/wl_${v}_$r.err
  done
done
step rn timeout -k 10 120 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_new.json 2> $O/rep_new.err
step t0 env SV_DEBUG_TIMING=1 timeout -k 10 150 python -u bench.py --tiles 2x4 --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/tiles_def.json 2> $O/tiles_def.err
step t1 env SV_DEBUG_TIMING=1 SV_DOMAIN_PREDICT=1 timeout -k 10 150 python -u bench.py --tiles 2x4 --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/tiles_pred.json 2> $O/tiles_pred.err
grep -h "sv domain" $O/tiles_*.err | grep -v " [15] sweeps" || true
for f in $O/*.json; do python scripts/summ_line.py $f; done
