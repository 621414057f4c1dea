set -u
mkdir -p gpurun_out/r15
timeout -k 10 300 python -m pytest tests/test_gpu_worldline.py -m gpu -q -p no:cacheprovider -k "reference_order_oracle" > gpurun_out/r15/a.log 2>&1; echo "only-oracle rc=$?"; tail -2 gpurun_out/r15/a.log
timeout -k 10 300 python -m pytest tests/test_gpu_worldline.py -m gpu -q -p no:cacheprovider -k "reference_order" > gpurun_out/r15/b.log 2>&1; echo "golden+oracle rc=$?"; tail -2 gpurun_out/r15/b.log
timeout -k 10 300 python -m pytest tests/test_gpu_worldline.py -m gpu -q -p no:cacheprovider -k "coexact or reference_order_oracle" > gpurun_out/r15/c.log 2>&1; echo "coexact+oracle rc=$?"; tail -2 gpurun_out/r15/c.log
