# Round 4: multi-sweep band launches (villain_sweep_hot_band) -- parity tests, then config 2 (L=256) at K = 7 (default),
# 5, 3, 9 and without bands (SV_BAND_K=0), each a bench line with the kernel-event time per sweep.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_band}
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread tests/test_gpu_band.py > $O/test.log 2>&1 || { echo "[band tests] failed"; tail -30 $O/test.log; exit 3; }
grep -c PASSED $O/test.log
for k in 7 0 5 3 9; do
  SV_BAND_K=$k timeout -k 10 120 python bench.py --L 256 --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo "[bench k=$k] failed"; tail -20 $O/bench_k$k.err; exit 3; }
  echo "k=$k $(python -c "import json,sys; d=json.load(open('$O/bench_k$k.json')); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))")"
done
