# Worldline suites at the default kernel choice, the config-3 bench line and a rocprofv3 kernel trace of it, then the
# headline timeline.  Usage: bash scripts/gpu/job_wl_timeline.sh TAG
source scripts/gpu/guard.sh
T=${1:-wlt}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wdomain.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
step wl timeout -k 10 200 python -u bench.py --workload worldline --steps 400 --warmup 20 > $O/wl.json 2> $O/wl.err
cat $O/wl.json
step wlprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wlprof -o run -- python3 -u bench.py --workload worldline --steps 400 --warmup 20 --no-copy-ceiling --no-cpu-baseline > $O/wlprof.json 2> $O/wlprof.err
bash scripts/gpu/job_timeline.sh $T/tl
