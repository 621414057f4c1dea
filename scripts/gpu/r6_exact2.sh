# Round 6: worldline acceptance words in LDS (config 3 regression fix) and config 5 as two part-batches on two streams:
# the affected suites, then A/B lines against the round-5 kernels.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_exact2
mkdir -p $O
B=supervillain_amd/variants/libsvhip_r5base.so
step t timeout -k 10 900 python -u -m pytest tests/test_gpu_observables.py tests/test_gpu_replicas.py tests/test_gpu_tuning.py tests/test_gpu_worms.py tests/test_gpu_worldline.py tests/test_gpu_wf_layout.py tests/test_gpu_wdomain.py tests/test_gpu_persistence.py tests/test_gpu_overflow.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for r in 1 2 3; do
  step wn$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
  step wb$r env SV_LIB_OVERRIDE=$B timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step r2$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_s2_$r.json 2> $O/rep_s2_$r.err
  step r1$r timeout -k 10 200 python -u bench.py --workload replicas --streams 1 --no-cpu-baseline --no-copy-ceiling > $O/rep_s1_$r.json 2> $O/rep_s1_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
