source scripts/gpu/guard.sh
T=${1:-r306}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_villain.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step emit timeout -k 10 300 python scripts/perf/emit_overlap.py > $O/emit.log 2>&1
tail -2 $O/emit.log
step emit2 timeout -k 10 300 python scripts/perf/emit_overlap.py --keep 8 > $O/emit8.log 2>&1
tail -2 $O/emit8.log
