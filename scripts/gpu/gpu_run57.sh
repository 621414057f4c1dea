source scripts/gpu/guard.sh
mkdir -p gpurun_out/r57
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r57/tests.log 2>&1
tail -3 gpurun_out/r57/tests.log
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r57/smoke.log 2>&1
tail -2 gpurun_out/r57/smoke.log
step bench timeout -k 10 300 python bench.py > gpurun_out/r57/bench.log 2>&1
tail -1 gpurun_out/r57/bench.log
