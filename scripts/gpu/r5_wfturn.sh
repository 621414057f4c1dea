# worldline_step_fused: block descriptors by value, row-seam advance maps, the turned strip layout.  Tests, then
# A/B: HEAD-of-round build (variants/libsvhip_wfbase.so) vs this build with SV_WF_TURN=0 vs this build
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wfturn}
mkdir -p $O
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wf_layout.py tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/tests.log 2>&1
V=supervillain_amd/variants/libsvhip_wfbase.so
for r in 1 2 3; do
  step wb$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step wp$r env SV_WF_TURN=0 timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_plain_$r.json 2> $O/wl_plain_$r.err
  step wt$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_turn_$r.json 2> $O/wl_turn_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
