source scripts/gpu/guard.sh
mkdir -p gpurun_out/r112
step t timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r112/tests.log 2>&1
tail -1 gpurun_out/r112/tests.log
step s timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r112/smoke.log 2>&1
tail -1 gpurun_out/r112/smoke.log
