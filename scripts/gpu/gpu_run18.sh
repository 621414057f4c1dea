set -u
mkdir -p gpurun_out/r18
timeout -k 10 300 python -m pytest tests/test_gpu_worldline.py -m gpu -q -p no:cacheprovider -k "reference_order" > gpurun_out/r18/b.log 2>&1; echo "golden+oracle rc=$?"; tail -2 gpurun_out/r18/b.log; ls gpurun_out/
