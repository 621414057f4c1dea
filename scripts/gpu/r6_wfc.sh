# Round 6: config 3's coexact passes on interior strips with per-wave precomputed draw offsets (as the plaquette
# passes), positions for reports computed only on a report (variants/libsvhip_wfc.so) against the tree, interleaved;
# then the worldline suites on the variant
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_wfc
mkdir -p $O
W=supervillain_amd/variants/libsvhip_wfc.so
for r in 1 2 3; do
  step b$r timeout -k 10 120 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step w$r env SV_LIB_OVERRIDE=$W timeout -k 10 120 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_wfc_$r.json 2> $O/wl_wfc_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
step t env SV_LIB_OVERRIDE=$W timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wf_layout.py tests/test_gpu_wdomain.py tests/test_gpu_statparity.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_wfc.log 2>&1
tail -2 $O/tests_wfc.log
