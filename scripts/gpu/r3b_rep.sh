# Speculative replica batches: replica suites, then an A/B of the config-5 bench (baseline library vs new).
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_rep
mkdir -p $O
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_overflow.py tests/test_gpu_pipeline.py tests/test_gpu_worms.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2; do
  SV_LIB_OVERRIDE=$PWD/variants/libsvhip_base.so step b$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  step n$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/new_$r.json 2> $O/new_$r.err
done
SV_DEBUG_TIMING=1 step dbg timeout -k 10 200 python -u bench.py --workload replicas --steps 200 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/dbg.json 2> $O/dbg.err
tail -8 $O/dbg.err
for f in $O/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,1), round(d['roofline']['avg_launch_us'],1))"; done
