source scripts/gpu/guard.sh
mkdir -p gpurun_out/r110
step s timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r110/smoke.log 2>&1
tail -1 gpurun_out/r110/smoke.log
step b timeout -k 10 400 python bench.py > gpurun_out/r110/bench.log 2>&1
grep '"metric"' gpurun_out/r110/bench.log | cut -c1-400
