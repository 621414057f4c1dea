set -u
mkdir -p gpurun_out/r19
for i in 1 2 3; do
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > gpurun_out/r19/pytest$i.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r19/pytest$i.log
if [ $rc -gt 1 ]; then exit $rc; fi
done
timeout -k 10 600 python scripts/stress_plaquette.py 60 > gpurun_out/r19/stress.log 2>&1; echo "stress rc=$?"; tail -2 gpurun_out/r19/stress.log
