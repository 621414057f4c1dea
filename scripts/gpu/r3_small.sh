# L=256 strip heights for the 8-wave small-lattice form (SV_SMALL_TH): one row iteration at TH <= 5, two at <= 13.
source scripts/gpu/guard.sh
O=gpurun_out/r3_small; mkdir -p $O
for th in 8 5 13 4 3; do
  step th$th env SV_SMALL_TH=$th timeout -k 10 120 python -u scripts/perf/sweep_time.py 2000 256 > $O/th$th.log 2>&1
  echo "TH=$th $(cat $O/th$th.log)"
done
step t env SV_SMALL_TH=5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_villain.py > $O/t.log 2>&1
tail -2 $O/t.log
