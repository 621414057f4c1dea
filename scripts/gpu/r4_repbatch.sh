# config 5: replica batch size 64 (default) / 128 / 256 sweeps (SV_REP_BATCH variants), replica suite on the 128 one
source scripts/gpu/guard.sh
O=gpurun_out/r4_repbatch
mkdir -p $O
step tests env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_repb128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_replicas.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in base repb128 repb256; do
    E=""
    [ $v != base ] && E="SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so"
    step $v env $E timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_${v}_$rep.json 2> $O/rep_${v}_$rep.err
    python -c "import json; d=json.loads(open('$O/rep_${v}_$rep.json').readline()); print('$v', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  done
done
