# Round-5 end: A/B of the Worldline domain tiles' write-through stores (variants/libsvhip_wltplain.so = plain stores),
# then the end-of-round evidence (scripts/gpu/r5_final.sh: full -m gpu suite, smoke, bench lines, profiles)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r5_wlt
mkdir -p $O
V=supervillain_amd/variants/libsvhip_wltplain.so
for r in 1 2; do
  step wb$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --workload worldline --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/wlt_base_$r.json 2> $O/wlt_base_$r.err
  step ws$r timeout -k 10 200 python -u bench.py --workload worldline --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/wlt_sc1_$r.json 2> $O/wlt_sc1_$r.err
done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
bash scripts/gpu/r5_final.sh
