# villain_sweep_block: frame rows split by column parity in LDS (SV_BLK_SPLIT), suites then L=256 A/B
source scripts/gpu/guard.sh
O=gpurun_out/r4_split
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 700 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_band.py tests/test_gpu_villain.py tests/test_gpu_overflow.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
unset AMD_LOG_LEVEL
for rep in 1 2 3; do
  for v in base nosplit; do
    E=""
    [ $v = nosplit ] && E="SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_nosplit.so"
    step $v env $E timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_${v}_$rep.json 2> $O/l256_${v}_$rep.err
    python -c "import json; d=json.loads(open('$O/l256_${v}_$rep.json').readline()); print('$v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  done
done
