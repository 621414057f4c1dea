# worldline write-through stores as default: worldline tests; then A/B on the headline: villain_sweep_hot with
# write-through row stores (variants/libsvhip_hotsc1.so, -DSV_HOT_SC1=1) vs plain stores
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_hotsc1}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_hotsc1.so
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wf_layout.py tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/tests.log 2>&1
step tv env SV_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overflow.py -k headline > $O/tests_hot.log 2>&1
for r in 1 2 3; do
  step hb$r timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_base_$r.json 2> $O/head_base_$r.err
  step hs$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_sc1_$r.json 2> $O/head_sc1_$r.err
done
step wl timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_new.json 2> $O/wl_new.err
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
