source scripts/gpu/guard.sh
mkdir -p gpurun_out/r93
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r93/tests.log 2>&1
tail -2 gpurun_out/r93/tests.log
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r93/smoke.log 2>&1
step bench timeout -k 10 400 python bench.py > gpurun_out/r93/bench.log 2>&1
step prof timeout -k 10 1000 bash scripts/profile.sh r01 > gpurun_out/r93/profile.log 2>&1
