# Plaquette acceptance table in worldline_step_fused: the worldline suites, then an interleaved A/B against the
# previous kernel (variants/libsvhip_wfold.so) on config 3
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wltab}
mkdir -p $O
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wdomain.py tests/test_gpu_tuning.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
for r in 1 2 3; do
  step new$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/new_$r.json 2> $O/new_$r.err
  step old$r env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wfold.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/old_$r.json 2> $O/old_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
