# Round 4: the native reference-order permutation (worldline suites, reference bench line), the whole-batch enqueue
# (Villain suites) and the skip-form replays (forced-rejection tests).
source scripts/gpu/guard.sh
export TMPDIR=/tmp AMD_LOG_LEVEL=1
O=gpurun_out/${OUT:-r4_ref}
mkdir -p $O
step tworank timeout -k 10 600 python -u -m pytest tests/test_gpu_00_two_ranks.py -v -rxs --timeout 300 --timeout-method thread -m gpu > $O/two_ranks.log 2>&1
grep -E "^=+ .*(passed|failed|xfail)|XFAIL|refused" $O/two_ranks.log | head -5
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_villain.py tests/test_gpu_boundary.py tests/test_gpu_overflow.py -x -v -s --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
grep -E "^=+ .*(passed|failed)" $O/tests.log
grep -q -E "^=+ .*[0-9]+ passed" $O/tests.log && ! grep -q -E "^=+ .*failed" $O/tests.log || exit 1
step wlref timeout -k 10 300 python -u bench.py --workload worldline --plaquette reference --steps 20 --warmup 3 > $O/bench_wl_reference.json 2> $O/bench_wl_reference.err
step drv timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
for f in $O/bench_*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', d['value'], round(d['ms_per_step']*1e3,2), d['roofline'].get('avg_launch_us'))"; done
