source scripts/gpu/guard.sh
mkdir -p gpurun_out/r87
step bench timeout -k 10 400 python bench.py > gpurun_out/r87/bench.log 2>&1
grep '^{' gpurun_out/r87/bench.log | tail -1 > gpurun_out/r87/bench.json
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r87/smoke.log 2>&1
