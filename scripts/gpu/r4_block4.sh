# villain_sweep_block after the prologue reorder: block suite, timeline, L=256 lines (base / without the scratch stores,
# timing only / 256-sweep batches), and the device timeline of an L=256 call (kernel trace: durations and gaps)
source scripts/gpu/guard.sh
O=gpurun_out/r4_block4
mkdir -p $O
export TMPDIR=/tmp
export AMD_LOG_LEVEL=1
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_block.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -2 $O/tests.log
unset AMD_LOG_LEVEL
step tl3 env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_blktime_flat.so timeout -k 10 120 python -u scripts/perf/block_timeline.py 256 63 3 > $O/timeline_K3.log 2>&1
cat $O/timeline_K3.log
for rep in 1 2; do
for v in base nodraw1 noscratch batch256; do
  E="SV_BLOCK_K=3"
  [ $v = noscratch ] && E="$E SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_noscratch.so"
  [ $v = nodraw1 ] && E="$E SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_nodraw1.so"
  [ $v = batch256 ] && E="$E SV_BATCH=256"
  step $v env $E timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_${v}_$rep.json 2> $O/l256_${v}_$rep.err
  python -c "import json; d=json.loads(open('$O/l256_${v}_$rep.json').readline()); print('$v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
done
step trace timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python bench.py --L 256 --steps 60 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1
python scripts/perf/gap_summary.py $O/trace villain_sweep_block 10 > $O/gaps.txt 2>&1; tail -25 $O/gaps.txt
step rephost timeout -k 10 200 python -u scripts/perf/replica_host.py > $O/replica_host.log 2>&1; cat $O/replica_host.log
# flat prologue jumps (SV_FLAT_JUMP) A/B: suites on the base library, then headline / worldline / tile lines per variant
export AMD_LOG_LEVEL=1
step suites timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_band.py tests/test_gpu_overflow.py tests/test_gpu_worldline.py tests/test_gpu_domain.py tests/test_gpu_wdomain.py tests/test_gpu_replicas.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/suites.log 2>&1
tail -2 $O/suites.log
unset AMD_LOG_LEVEL
for rep in 1 2; do
for v in base noflatjump; do
  E=""
  [ $v = noflatjump ] && E="SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_noflatjump.so"
  step h$v env $E timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/head_${v}_$rep.json 2> $O/head_${v}_$rep.err
  python -c "import json; d=json.loads(open('$O/head_${v}_$rep.json').readline()); print('head $v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"
  step w$v env $E timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_${v}_$rep.json 2> $O/wl_${v}_$rep.err
  python -c "import json; d=json.loads(open('$O/wl_${v}_$rep.json').readline()); print('wl $v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  step t$v env $E SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_${v}_$rep.log 2>&1
  echo "tile $v: $(tr "\n" " " < $O/tile_${v}_$rep.log)"
done
done
