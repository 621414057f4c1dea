set -u
mkdir -p gpurun_out/r13
timeout -k 10 900 python -m pytest tests/test_gpu_villain.py -m gpu -q -x --timeout 600 -p no:cacheprovider > gpurun_out/r13/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r13/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r13/b$i.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/r13/b$i.log').read().strip().splitlines()[-1]);print('base', round(d['value']/1e9,2),'G/s', round(d['roofline']['avg_launch_us'],1),'us', round(d['ms_per_step'],3), 'ms/step')"
done
