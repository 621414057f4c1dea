# Villain suites (incl. the L=4096 oracle pin) and driver-form bench lines after a hot-path change.
source scripts/gpu/guard.sh
O=gpurun_out/${1:-r3_check}; mkdir -p $O
export TMPDIR=/tmp
step t timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_boundary.py tests/test_gpu_pipeline.py tests/test_gpu_domain.py > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$r.json 2> $O/driver_$r.err
  python -c "import json; d=json.loads(open('$O/driver_$r.json').readline()); print('driver', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
done
step def timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/default.json 2> $O/default.err
python -c "import json; d=json.loads(open('$O/default.json').readline()); print('default', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
step ovh env SV_DEBUG_TIMING=1 timeout -k 10 200 python -u scripts/perf/call_overhead.py 4096 20 8 > $O/ovh.log 2>&1
grep "^call" $O/ovh.log
step tr timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/tr.json 2> $O/tr.err
python -c "import json; d=json.loads(open('$O/tr.json').readline()); print('traced', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config']['lemire_rejections_in_timed_steps'])"
