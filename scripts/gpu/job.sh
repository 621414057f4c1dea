source scripts/gpu/guard.sh
T=${1:-r216}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step wl timeout -k 10 400 python -u -m pytest tests/test_gpu_worldline.py -x -q --timeout 200 --timeout-method thread > $O/tests_wl.log 2>&1
tail -2 $O/tests_wl.log
step dbg timeout -k 10 120 python scripts/debug_wf.py > $O/dbg.log 2>&1
cat $O/dbg.log
step bwl timeout -k 10 300 python bench.py --workload worldline --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/bwl.log 2>&1
grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' $O/bwl.log | tr '\n' ' '; echo
