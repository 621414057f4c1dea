source scripts/gpu/guard.sh
T=${1:-r344}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_domain.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
step deep timeout -k 10 600 python scripts/perf/deep_halo.py 1 4 8 > $O/deep.log 2>&1
grep us/sweep $O/deep.log
step b24 timeout -k 10 300 python bench.py --tiles 2x4 --no-cpu-baseline --no-copy-ceiling > $O/b_tiles24.log 2>&1
grep '^{' $O/b_tiles24.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('2x4 emu', round(d['value']/1e9,2), d['ms_per_step'], d['config']['weak_scaling'], d['config']['sweeps_per_halo_exchange'])"
