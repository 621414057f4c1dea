# Strip heights 4k+1 / 8k-3: single lattices at 1024/2048/4096 (old heights as SV_FUSED_TH / SV_STRIPS), the
# 2048x1024 tile, and the suites that cover the strip geometry.
source scripts/gpu/guard.sh
O=gpurun_out/r3_th; mkdir -p $O
step ab4096 timeout -k 10 400 python -u scripts/perf/strips_ab.py 4096 300 4 56x5,40x5,32 57x5,41x5,22 > $O/ab4096.log 2>&1
cat $O/ab4096.log
step s_new timeout -k 10 200 python -u scripts/perf/sweep_time.py 200 2048 1024 > $O/s_new.log 2>&1
step s_old16 env SV_FUSED_TH=16 timeout -k 10 200 python -u scripts/perf/sweep_time.py 200 1024 > $O/s_old16.log 2>&1
step s_old52 env SV_FUSED_TH=52 timeout -k 10 200 python -u scripts/perf/sweep_time.py 200 2048 > $O/s_old52.log 2>&1
cat $O/s_new.log $O/s_old16.log $O/s_old52.log
step tile env SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/tile_th.py "" > $O/tile.log 2>&1
cat $O/tile.log
step t timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_domain.py tests/test_gpu_wdomain.py tests/test_gpu_boundary.py > $O/t.log 2>&1
tail -2 $O/t.log
