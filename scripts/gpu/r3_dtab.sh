# Domain strip tables: the N=2 tile with and without them, and the domain suite (incl. the table test).
source scripts/gpu/guard.sh
O=gpurun_out/r3_dtab; mkdir -p $O
for r in 1 2; do
  step u$r env SV_STRIPS=uniform SV_SIZES=4096x2048 timeout -k 10 200 python -u scripts/perf/tile_th.py "" > $O/u$r.log 2>&1
  step t$r env SV_SIZES=4096x2048 timeout -k 10 200 python -u scripts/perf/tile_th.py "" > $O/t$r.log 2>&1
  echo "uniform: $(cat $O/u$r.log)  tables: $(cat $O/t$r.log)"
done
step t timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_domain.py tests/test_gpu_villain.py > $O/t.log 2>&1
tail -2 $O/t.log
