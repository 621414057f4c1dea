# worldline_step_fused turned layout, second version: tests, per-WG timelines (turned / plain), A/B base / plain / turned
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wfturn2}
mkdir -p $O
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wf_layout.py tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/tests.log 2>&1
step tl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wftime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline_turned.log 2>&1
step tl0 env SV_WF_TURN=0 SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wftime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline_plain.log 2>&1
V=supervillain_amd/variants/libsvhip_wfbase.so
for r in 1 2; do
  step wb$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step wp$r env SV_WF_TURN=0 timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_plain_$r.json 2> $O/wl_plain_$r.err
  step wt$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_turn_$r.json 2> $O/wl_turn_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
