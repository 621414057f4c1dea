# Round 4: band launches with deferred statistics and overlapped row-base jumps -- parity tests, config 2 at K = 0, 3,
# 5, 7, 9, the per-sweep timeline (K = 7, 5), then the VALU ablation passes (r4_ablate.sh).
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_band2}
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_band.py > $O/test.log 2>&1 || { echo "[band tests] failed"; tail -30 $O/test.log; exit 3; }
grep -c PASSED $O/test.log
for k in 0 3 5 7 9; do
  SV_BAND_K=$k timeout -k 10 120 python bench.py --L 256 --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo "[bench k=$k] failed"; tail -20 $O/bench_k$k.err; exit 3; }
  echo "k=$k $(python -c "import json,sys; d=json.load(open('$O/bench_k$k.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])")"
done
for k in 7 5; do
  SV_BAND_K=$k SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 120 python -u scripts/perf/band_timeline.py 256 63 > $O/band_k$k.log 2>&1 || { echo "[bandtime k$k] failed"; tail -20 $O/band_k$k.log; exit 3; }
  head -9 $O/band_k$k.log
done
OUT=r4_ablate bash scripts/gpu/r4_ablate.sh
