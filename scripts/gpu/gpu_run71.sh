source scripts/gpu/guard.sh
mkdir -p gpurun_out/r71
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r71/tests.log 2>&1
tail -2 gpurun_out/r71/tests.log
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r71/smoke.log 2>&1
tail -1 gpurun_out/r71/smoke.log
step bench timeout -k 10 300 python bench.py > gpurun_out/r71/bench.log 2>&1
tail -1 gpurun_out/r71/bench.log | cut -c1-200
step b24 timeout -k 10 300 python bench.py --tiles 2x4 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r71/b24.log 2>&1
tail -1 gpurun_out/r71/b24.log | cut -c1-200
