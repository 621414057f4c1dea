# (1) the worms/Hammer fault of r5_full: the failing file alone, serialized, error log on; (2) replicas suites + bench
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_fault2}
mkdir -p $O
step worms env AMD_LOG_LEVEL=1 AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3 SV_ALLOC_LOG=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_worms.py > $O/worms.log 2>&1
tail -3 $O/worms.log
grep -E "[0-9]+ passed" $O/worms.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/worms.log > /dev/null || { echo "[worms] not green"; exit 1; }
step rep env AMD_LOG_LEVEL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_replicas.py tests/test_gpu_observables.py tests/test_gpu_pipeline.py > $O/rep.log 2>&1
tail -2 $O/rep.log
grep -E "[0-9]+ passed" $O/rep.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/rep.log > /dev/null || { echo "[rep] not green"; exit 1; }
for r in 1 2; do
step repb timeout -k 10 300 python -u bench.py --workload replicas --no-cpu-baseline > $O/replicas_$r.json 2> $O/replicas_$r.err
python -c "import json; d=json.loads(open('$O/replicas_$r.json').readline()); print('replicas', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
