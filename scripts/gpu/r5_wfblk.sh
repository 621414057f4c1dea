# worldline_step_fused with the block descriptors by value (kernarg): worldline tests, then A/B vs variants/libsvhip_wfbase.so
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wfblk}
mkdir -p $O
step tests timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/tests.log 2>&1
V=supervillain_amd/variants/libsvhip_wfbase.so
for r in 1 2 3; do
  step wb$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step wn$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_new_$r.json 2> $O/wl_new_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
