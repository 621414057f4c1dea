# A/B: worldline_step_fused's row loads non-temporal (variants/libsvhip_wfnt.so) vs default
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wfnt}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_wfnt.so
for r in 1 2 3; do
  step wb$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step wn$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_nt_$r.json 2> $O/wl_nt_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
