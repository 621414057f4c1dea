# Config 5 chunked enqueue: replica suites, then an A/B of the config-5 bench (baseline library vs new) + trace.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_rep2
mkdir -p $O
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_overflow.py tests/test_gpu_pipeline.py tests/test_gpu_worms.py tests/test_gpu_villain.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3; do
  SV_LIB_OVERRIDE=$PWD/variants/libsvhip_base.so step b$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  step n$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/new_$r.json 2> $O/new_$r.err
done
step tr timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/trace.log 2>&1
python scripts/perf/idle_gaps.py $O/trace/run_kernel_trace.csv villain_sweep_hot_fr 6
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"; done
