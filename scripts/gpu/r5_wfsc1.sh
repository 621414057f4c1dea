# A/B: worldline_step_fused's row stores write-through (variants/libsvhip_wfsc1.so, -DSV_WF_SC1=1) vs plain stores
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wfsc1}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_wfsc1.so
step t env SV_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wf_layout.py -k equals > $O/tests.log 2>&1
for r in 1 2 3; do
  step wb$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step ws$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_sc1_$r.json 2> $O/wl_sc1_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
