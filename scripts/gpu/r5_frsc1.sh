# A/B config 5: replica batches with write-through row stores (variants/libsvhip_frsc1.so), 64-row tiles (default) and
# whole-replica 128-row strips (SV_FUSED_TH=128: one round of 1024 workgroups)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_frsc1}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_frsc1.so
step t env SV_LIB_OVERRIDE=$V SV_FUSED_TH=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_replicas.py > $O/tests.log 2>&1
for r in 1 2; do
  step b$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_base_$r.json 2> $O/rep_base_$r.err
  step s$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_sc1_$r.json 2> $O/rep_sc1_$r.err
  step bt$r env SV_FUSED_TH=128 timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_th128_$r.json 2> $O/rep_th128_$r.err
  step st$r env SV_LIB_OVERRIDE=$V SV_FUSED_TH=128 timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep_th128sc1_$r.json 2> $O/rep_th128sc1_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
