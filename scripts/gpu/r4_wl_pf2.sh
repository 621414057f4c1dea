# Round 4: worldline_step_fused with / without the prologue's two row-load rounds overlapped (SV_WF_PF2), three
# interleaved repetitions; worldline + worldline-domain parity and the jump-table purge regression test first.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_wl_pf2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_worldline.py tests/test_gpu_wdomain.py tests/test_gpu_table_purge.py > $O/test.log 2>&1 || { echo "[tests] failed"; tail -30 $O/test.log; exit 3; }
tail -1 $O/test.log
for rep in 1 2 3; do
  for v in base pf2off; do
    if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wfpf2off.so; fi
    timeout -k 10 120 python bench.py --workload worldline --steps 300 --warmup 30 --no-cpu-baseline > $O/wl_${v}_$rep.json 2> $O/wl_${v}_$rep.err || { echo "[wl $v] failed"; tail -20 $O/wl_${v}_$rep.err; exit 3; }
    echo "wl $v $rep $(python -c "import json; d=json.load(open('$O/wl_${v}_$rep.json')); print(round(d['value']/1e9,3), round(d['roofline']['avg_launch_us'],2))")"
  done
done
