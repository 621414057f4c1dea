source scripts/gpu/guard.sh
mkdir -p gpurun_out/r79
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r79/tests.log 2>&1
tail -2 gpurun_out/r79/tests.log
step repl timeout -k 10 200 python bench.py --workload replicas > gpurun_out/r79/repl.log 2>&1
echo REPL $(grep -o '"value": [0-9.]*' gpurun_out/r79/repl.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r79/repl.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r79/repl.log)
