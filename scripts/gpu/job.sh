source scripts/gpu/guard.sh
T=${1:-r330}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_philox.py tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
for rng in pcg64 philox; do
step b$rng timeout -k 10 300 python bench.py --rng $rng --no-cpu-baseline --no-copy-ceiling > $O/b_$rng.log 2>&1
grep '^{' $O/b_$rng.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$rng', round(d['value']/1e9,2), d['ms_per_step'], round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3), d['config']['acceptance_rate'])"
done
