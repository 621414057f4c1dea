# Reference-order Plaquette (device level plan): its tests and bench line; the 2048x1024 tile vs strip height.
source scripts/gpu/guard.sh
O=gpurun_out/r3_m2; mkdir -p $O
export TMPDIR=/tmp
step t timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_worldline.py tests/test_gpu_boundary.py > $O/tests.log 2>&1
tail -3 $O/tests.log
step wlref timeout -k 10 300 python -u bench.py --workload worldline --L 1024 --plaquette reference --steps 20 --warmup 2 > $O/wlref.json 2> $O/wlref.err
cat $O/wlref.json
export SV_SIZES=2048x1024
step th timeout -k 10 300 python -u scripts/perf/tile_th.py 8 12 16 20 24 28 32 40 "" > $O/th.log 2>&1
cat $O/th.log
