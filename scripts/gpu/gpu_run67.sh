source scripts/gpu/guard.sh
mkdir -p gpurun_out/r67
step tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r67/tests.log 2>&1
tail -2 gpurun_out/r67/tests.log
step bench timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/r67/bench.log 2>&1
python -c "import json;d=json.loads(open('gpurun_out/r67/bench.log').read().strip().splitlines()[-1]);print('persistent', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'])"
SV_PERSISTENT=0 step bench0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/r67/bench0.log 2>&1
python -c "import json;d=json.loads(open('gpurun_out/r67/bench0.log').read().strip().splitlines()[-1]);print('nonpersistent', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'])"
step rej timeout -k 10 300 python scripts/perf/reject_cost.py > gpurun_out/r67/rej.log 2>&1
cat gpurun_out/r67/rej.log
step repl timeout -k 10 300 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r67/repl.log 2>&1
python -c "import json;d=json.loads(open('gpurun_out/r67/repl.log').read().strip().splitlines()[-1]);print('replicas', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'])"
