# The runtime-switch suite and the suites whose launch choices the switch cleanup touched, then the end-of-round evidence
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tune}
mkdir -p $O
step tune timeout -k 10 600 python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_block.py tests/test_gpu_band.py tests/test_gpu_villain.py tests/test_gpu_worldline.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
TESTS=0 bash scripts/gpu/r5_final.sh
