# replica observables measured in the library's copy-out (sv_replicas_run_measured): replica suites, then config 5
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_repmeas}
mkdir -p $O
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_observables.py tests/test_gpu_tuning.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
for r in 1 2 3; do
  step rep$r timeout -k 10 300 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_$r.json 2> $O/rep_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', round(d['ms_per_step']*1e3/d['roofline']['avg_launch_us'],3))"; done
