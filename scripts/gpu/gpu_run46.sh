source scripts/gpu/guard.sh
mkdir -p gpurun_out/r46
export TMPDIR=/tmp
for w in site link exact cohomology hammer; do
step b$w timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r46/$w.log 2>&1
python -c "
import json,sys; d=json.loads(open('gpurun_out/r46/$w.log').read().strip().splitlines()[-1])
print('$w', '%.3g'%d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], '%.3f'%d['roofline']['frac'])"
done
cd /tmp && step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r46/prof -o hammer -- python $GRAFT_REPO_ROOT/bench.py --workload hammer --steps 20 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r46/prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/r46/prof -name "*stats*"
