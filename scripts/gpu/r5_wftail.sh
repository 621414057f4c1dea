# config 3: the turned layout's last row strip cut in two: tests, timeline, A/B (SV_WF_TAIL=0 vs default)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wftail}
mkdir -p $O
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wf_layout.py tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/tests.log 2>&1
step tl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wftime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline_tail.log 2>&1
for r in 1 2 3; do
  step wn$r env SV_WF_TAIL=0 timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_notail_$r.json 2> $O/wl_notail_$r.err
  step wt$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_tail_$r.json 2> $O/wl_tail_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
