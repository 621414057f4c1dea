# Worldline prologue: first row prefetch before the row-base jumps (SV_WF_PF0).  Worldline suites, A/B of the
# config-3 bench against the session-start library, WG timeline.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_wfpf
mkdir -p $O
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wdomain.py tests/test_gpu_statparity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2 3; do
  SV_LIB_OVERRIDE=$PWD/variants/libsvhip_base.so step b$r timeout -k 10 200 python -u bench.py --workload worldline --steps 400 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  step n$r timeout -k 10 200 python -u bench.py --workload worldline --steps 400 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/new_$r.json 2> $O/new_$r.err
done
SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wftime.so step tl timeout -k 10 120 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline.log 2>&1
tail -5 $O/timeline.log
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2))"; done
