# Two-part plan of a call's first batch on small lattices (SV_PLAN2): Villain suites, then L=256 lines A/B
source scripts/gpu/guard.sh
O=gpurun_out/r4_plan2
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 700 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_band.py tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_table_purge.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
unset AMD_LOG_LEVEL
for rep in 1 2 3; do
  for v in 1 0; do
    step p$v env SV_PLAN2=$v SV_DEBUG_TIMING=1 timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_p${v}_$rep.json 2> $O/l256_p${v}_$rep.err
    python -c "import json; d=json.loads(open('$O/l256_p${v}_$rep.json').readline()); print('plan2=$v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  done
done
grep "\[sv\]" $O/l256_p1_1.err | tail -4
