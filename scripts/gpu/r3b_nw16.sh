# 16-wave villain_sweep_hot: correctness with the 16-wave form forced, then tile / single-lattice timings.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_nw16
mkdir -p $O
SV_DOMAIN_NW=16 SV_HOT_NW=16 step t16 timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py tests/test_gpu_villain.py tests/test_gpu_overflow.py -x -q --timeout 200 --timeout-method thread > $O/tests16.log 2>&1
tail -3 $O/tests16.log
for r in 1 2; do
  step b$r timeout -k 10 120 python -u scripts/perf/tile_nw.py base > $O/tile_base_$r.log 2>&1; cat $O/tile_base_$r.log
  for th in 45 61 77 93; do
    SV_DOMAIN_NW=16 SV_DOMAIN_TH16=$th step n$th timeout -k 10 120 python -u scripts/perf/tile_nw.py nw16_th$th > $O/tile_16_${th}_$r.log 2>&1; cat $O/tile_16_${th}_$r.log
  done
done
step L0 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/L4096_base.json 2>&1
for th in 61 77 109; do
  SV_HOT_NW=16 SV_FUSED_TH=$th step L$th timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/L4096_16_$th.json 2>&1
done
for f in $O/L4096*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['roofline']['avg_launch_us'],2))"; done
