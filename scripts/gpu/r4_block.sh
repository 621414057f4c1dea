# Temporal-blocking launches (villain_sweep_block): parity suites, then L=256 bench lines per K against bands and
# one sweep per launch.
source scripts/gpu/guard.sh
O=gpurun_out/r4_block
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_band.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
unset AMD_LOG_LEVEL
for rep in 1 2; do
for v in "K3:SV_BLOCK_K=3" "K5:SV_BLOCK_K=5" "K7:SV_BLOCK_K=7" "band:SV_MULTISWEEP=2" "single:SV_MULTISWEEP=3"; do
  n=${v%%:*}; e=${v#*:}
  step $n env $e timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_${n}_$rep.json 2> $O/l256_${n}_$rep.err
  python -c "import json; d=json.loads(open('$O/l256_${n}_$rep.json').readline()); print('$n', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
done
