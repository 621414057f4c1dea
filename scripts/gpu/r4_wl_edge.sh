# Round 4: worldline_step_fused with narrower edge strips (SV_WF_EDGE percent of the uniform width; 0 = uniform):
# parity, the config-3 bench at 0 / 80 / 88 / 94 and without the chained row bases (SV_WF_CHAIN=0), and the
# per-workgroup timeline at the default.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_wl_edge}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/test.log 2>&1 || { echo "[wl tests] failed"; tail -30 $O/test.log; exit 3; }
tail -1 $O/test.log
for rep in 1 2; do
  for e in 0 80 88 94 nochain nopf2; do
    unset SV_LIB_OVERRIDE SV_WF_CHAIN
    if [ $e = nochain ]; then export SV_WF_CHAIN=0 SV_WF_EDGE=88;
    elif [ $e = nopf2 ]; then export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wfpf2off.so SV_WF_EDGE=88;
    else export SV_WF_EDGE=$e; fi
    timeout -k 10 120 python bench.py --workload worldline --steps 300 --warmup 30 --no-cpu-baseline > $O/wl_e${e}_$rep.json 2> $O/wl_e${e}_$rep.err || { echo "[wl e=$e] failed"; tail -20 $O/wl_e${e}_$rep.err; exit 3; }
    echo "wl edge=$e $rep $(python -c "import json; d=json.load(open('$O/wl_e${e}_$rep.json')); print(round(d['value']/1e9,3), round(d['roofline']['avg_launch_us'],2))")"
  done
done
unset SV_WF_CHAIN SV_WF_EDGE SV_LIB_OVERRIDE
SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wftime.so timeout -k 10 120 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline.log 2>&1 || { echo "[timeline] failed"; tail -20 $O/timeline.log; exit 3; }
head -8 $O/timeline.log
