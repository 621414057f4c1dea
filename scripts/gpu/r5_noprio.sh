# A/B: the kernels built without -mllvm --amdgpu-set-wave-priority (variants/libsvhip_noprio.so) vs the default build
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_noprio}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_noprio.so
for r in 1 2; do
  step hb$r timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_base_$r.json 2> $O/head_base_$r.err
  step hp$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_noprio_$r.json 2> $O/head_noprio_$r.err
  step wb$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step wp$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline > $O/wl_noprio_$r.json 2> $O/wl_noprio_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
