source scripts/gpu/guard.sh
T=${1:-r377}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_villain_local.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o h --output-format csv -- python bench.py --workload hammer --steps 50 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/prof.log 2>&1
grep -i cohomology $O/prof/h_kernel_stats.csv | cut -c1-200
step bh timeout -k 10 300 python bench.py --workload hammer --no-cpu-baseline --no-copy-ceiling > $O/b_hammer.log 2>&1
grep '^{' $O/b_hammer.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hammer', round(d['value']/1e9,3), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2))"
