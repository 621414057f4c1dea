# Round 6: config 3's regression -- LDS size (SV_WFFX 1 / 2 now without the LDS words) vs the stats atomics per wave
# (SV_WFLUSH_WG=1: one per workgroup), against round 5's kernels
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_wfab2
mkdir -p $O
V=supervillain_amd/variants
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_domain.py tests/test_gpu_block.py tests/test_gpu_band.py tests/test_gpu_villain.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for r in 1 2; do
  for v in r5base wffx1 wffx2 wfwg wfwg2; do
    step $v$r env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_${v}_$r.json 2> $O/wl_${v}_$r.err
  done
  step new$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
done
for r in 1 2; do
  step rc$r timeout -k 10 200 python -u scripts/perf/reject_cost_small.py 256 200 30 100 > $O/rej_new_$r.log 2>&1
  step rb$r env SV_LIB_OVERRIDE=$V/libsvhip_r5base.so timeout -k 10 200 python -u scripts/perf/reject_cost_small.py 256 200 30 100 > $O/rej_base_$r.log 2>&1
done
cat $O/rej_*.log
for f in $O/*.json; do python scripts/summ_line.py $f; done
step dt timeout -k 10 300 env SV_DEBUG_TIMING=1 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/tiles_dbg.json 2> $O/tiles_dbg.err
tail -40 $O/tiles_dbg.err
python scripts/summ_line.py $O/tiles_dbg.json
