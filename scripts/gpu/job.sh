# The current gpurun job (overwritten per call; the tags under gpurun_out/ keep the results).
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu/job.sh r201
source scripts/gpu/guard.sh
T=${1:-r201}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step bench timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.log 2>&1
tail -1 $O/bench20.log
step bench200 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench200.log 2>&1
tail -1 $O/bench200.log
step l256 timeout -k 10 300 python bench.py --L 256 --steps 2000 --warmup 100 > $O/bench_l256.log 2>&1
tail -1 $O/bench_l256.log
step copy timeout -k 10 120 python scripts/perf/copy_calibrate.py > $O/copy.log 2>&1
cat $O/copy.log
step fetch timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal_fetch -o p --output-format csv -- python scripts/perf/copy_calibrate.py 2 > $O/cal_fetch.log 2>&1
step write timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/cal_write -o p --output-format csv -- python scripts/perf/copy_calibrate.py 2 > $O/cal_write.log 2>&1
step trace timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1
echo done
