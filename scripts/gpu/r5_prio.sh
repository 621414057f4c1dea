# A/B: issue priority by the row steps left (variants/libsvhip_prio.so, -DSV_HOT_PRIO=1) vs the default build:
# the 2048 x 1024 tile alone (deep_halo.py, depth 4), the L=4096 headline (200 sweeps), the weak 2 x 4 emulation
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_prio}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_prio.so
for r in 1 2; do
  step tb$r env SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_base_$r.log 2>&1
  step tp$r env SV_LIB_OVERRIDE=$V SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_prio_$r.log 2>&1
  step hb$r timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_base_$r.json 2> $O/head_base_$r.err
  step hp$r env SV_LIB_OVERRIDE=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/head_prio_$r.json 2> $O/head_prio_$r.err
done
step wb env SV_DOMAIN_PREDICT=1 timeout -k 10 300 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 3 --no-cpu-baseline > $O/weak_base.json 2> $O/weak_base.err
step wp env SV_LIB_OVERRIDE=$V SV_DOMAIN_PREDICT=1 timeout -k 10 300 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 3 --no-cpu-baseline > $O/weak_prio.json 2> $O/weak_prio.err
grep -h "rccl=0" $O/tile_*.log /dev/null | cat
for f in $O/tile_*.log; do echo "$f $(grep rccl=0 $f)"; done
for f in $O/*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config'].get('lemire_rejections_in_timed_steps'))"; done
