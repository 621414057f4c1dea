# Round 4, item 5: the config-4 tile (2048 x 1024, depth 4) with two waves of strips (tall for the workgroups
# dispatched first, SV_TILE_SCHED=1, default) vs uniform 37-row strips (SV_TILE_SCHED=0): domain parity first, then
# the tile alone and through RCCL loopback (scripts/perf/deep_halo.py), and the 2 x 4 emulation bench line.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_tile}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_domain.py > $O/test.log 2>&1 || { echo "[domain tests] failed"; tail -30 $O/test.log; exit 3; }
tail -1 $O/test.log
for rep in 1 2; do
  for s in 1 0; do
    SV_TILE_SCHED=$s SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_s${s}_$rep.log 2>&1 || { echo "[tile s=$s] failed"; tail -20 $O/tile_s${s}_$rep.log; exit 3; }
    echo "sched=$s rep $rep: $(tr '\n' ' ' < $O/tile_s${s}_$rep.log)"
  done
done
for s in 1 0; do
  SV_TILE_SCHED=$s timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/t8_s$s.json 2> $O/t8_s$s.err || { echo "[t8 s=$s] failed"; tail -20 $O/t8_s$s.err; exit 3; }
  echo "tiles2x4 sched=$s $(python -c "import json; d=json.load(open('$O/t8_s$s.json')); print(round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,1), 'us/sweep')")"
done
# replays of a rejected sweep: the hot kernel's skip form (default) vs the general int32 kernel (SV_HOT_SKIP=0)
for s in 1 0; do
  SV_HOT_SKIP=$s timeout -k 10 300 python -u scripts/perf/reject_window.py 4096 20 150 > $O/rejwin_s$s.log 2>&1 || { echo "[rejwin s=$s] failed"; tail -20 $O/rejwin_s$s.log; exit 3; }
  echo "skip=$s: $(tail -3 $O/rejwin_s$s.log | tr '\n' ' ')"
done
