set -u
mkdir -p gpurun_out/r14
timeout -k 10 600 python scripts/stress_plaquette.py 60 > gpurun_out/r14/stress.log 2>&1; echo "stress rc=$?"; tail -5 gpurun_out/r14/stress.log
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/r14/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r14/pytest.log
