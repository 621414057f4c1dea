# villain_sweep_block after the prologue split, descriptor prefetch and dense lanes: block + band suites, L=256 lines
# per K, the workgroup timeline
source scripts/gpu/guard.sh
O=gpurun_out/r4_block3
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_band.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
unset AMD_LOG_LEVEL
for rep in 1 2; do
for v in "K3:SV_BLOCK_K=3" "K5:SV_BLOCK_K=5" "K7:SV_BLOCK_K=7"; do
  n=${v%%:*}; e=${v#*:}
  step $n env $e timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_${n}_$rep.json 2> $O/l256_${n}_$rep.err
  python -c "import json; d=json.loads(open('$O/l256_${n}_$rep.json').readline()); print('$n', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
done
for K in 3 5; do
  step tl$K env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_blktime_flat.so timeout -k 10 120 python -u scripts/perf/block_timeline.py 256 63 $K > $O/timeline_K$K.log 2>&1
  echo "== K=$K"; cat $O/timeline_K$K.log
done
