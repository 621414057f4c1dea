# Round 6, first box: the new persistence tests, SV_SYNC_CHECK on two suites, then the domain lines' E_N twice each
# (strong 2x4 and weak 2x4 emulated on one GPU) and the default headline line.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_first
mkdir -p $O
#step pers timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_persistence.py > $O/pers.log 2>&1
#step sync env SV_SYNC_CHECK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_villain.py tests/test_gpu_split.py > $O/sync.log 2>&1
for r in 1 2; do
  step ts$r timeout -k 10 200 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/tiles_strong_$r.json 2> $O/tiles_strong_$r.err
  step tw$r timeout -k 10 300 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 5 --no-cpu-baseline > $O/tiles_weak_$r.json 2> $O/tiles_weak_$r.err
done
step head timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/head.json 2> $O/head.err
for f in $O/*.json; do python -c "
import json; d=json.loads(open('$f').readline()); s=d['config'].get('scaling_reference', {})
print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', 'E_N', s.get('E_N'), 'E_single', s.get('E_N_vs_single_lattice'), 'R1', s.get('R1'), 'single', s.get('single_lattice_rate'), 'rej', d['config'].get('lemire_rejections_in_timed_steps'), d['metric'])"; done
