# Round 4: band barrier polled with agent-scope loads -- parity tests, config 2 at K = 3, 5, 7, timeline K = 5
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_band3}
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_band.py > $O/test.log 2>&1 || { echo "[band tests] failed"; tail -30 $O/test.log; exit 3; }
grep -c PASSED $O/test.log
for k in 3 5 7; do
  SV_BAND_K=$k timeout -k 10 120 python bench.py --L 256 --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo "[bench k=$k] failed"; tail -20 $O/bench_k$k.err; exit 3; }
  echo "k=$k $(python -c "import json,sys; d=json.load(open('$O/bench_k$k.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")"
done
SV_BAND_K=5 SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 120 python -u scripts/perf/band_timeline.py 256 60 > $O/band_k5.log 2>&1 || { echo "[bandtime] failed"; tail -20 $O/band_k5.log; exit 3; }
head -7 $O/band_k5.log
# worldline_step_fused: 32-bit row offsets, 2-op range check, uniform row-base advance -- parity, then A/B vs HEAD
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_worldline.py tests/test_gpu_overflow.py > $O/wl_test.log 2>&1 || { echo "[wl tests] failed"; tail -30 $O/wl_test.log; exit 3; }
tail -1 $O/wl_test.log
for rep in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_head.so; else unset SV_LIB_OVERRIDE; fi
    timeout -k 10 120 python bench.py --workload worldline --steps 300 --warmup 30 --no-cpu-baseline > $O/wl_${v}_$rep.json 2> $O/wl_${v}_$rep.err || { echo "[wl bench $v] failed"; tail -20 $O/wl_${v}_$rep.err; exit 3; }
    echo "wl $v $rep $(python -c "import json; d=json.load(open('$O/wl_${v}_$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")"
  done
done
for rep in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_head.so; else unset SV_LIB_OVERRIDE; fi
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/vh_${v}_$rep.json 2> $O/vh_${v}_$rep.err || { echo "[vh bench $v] failed"; tail -20 $O/vh_${v}_$rep.err; exit 3; }
    echo "vh $v $rep $(python -c "import json; d=json.load(open('$O/vh_${v}_$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")"
  done
done
unset SV_LIB_OVERRIDE
