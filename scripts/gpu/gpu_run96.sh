source scripts/gpu/guard.sh
mkdir -p gpurun_out/r96
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r96/tests.log 2>&1
tail -2 gpurun_out/r96/tests.log
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r96/smoke.log 2>&1
step bench timeout -k 10 400 python bench.py > gpurun_out/r96/bench.log 2>&1
step repl timeout -k 10 300 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r96/repl.log 2>&1
