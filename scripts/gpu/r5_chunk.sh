source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_chunk}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_split.py tests/test_gpu_villain.py > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
for rep in 1 2; do
for ch in 0 2 4; do
  step rw$ch env SV_CHUNK=$ch timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/rw_${ch}_$rep.log 2>&1
  echo "chunk $ch: $(cut -c1-220 $O/rw_${ch}_$rep.log)"
done
done
