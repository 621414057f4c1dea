# villain_sweep_block workgroup timeline (variants -DSV_BLKTIME=1, prologue row bases by flat / dependent table jumps),
# L=256 at K = 3 and 5, then block sides 8 / 32 timed
source scripts/gpu/guard.sh
O=gpurun_out/r4_blktime
mkdir -p $O
for v in flat noflat; do
for K in 3 5; do
  step tl$v$K env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_blktime_$v.so timeout -k 10 120 python -u scripts/perf/block_timeline.py 256 63 $K > $O/timeline_${v}_K$K.log 2>&1
  echo "== $v K=$K"; cat $O/timeline_${v}_K$K.log
done
done
for bs in 16 8 32; do
  step bs$bs env SV_BLOCK_BS=$bs timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_bs$bs.json 2> $O/l256_bs$bs.err
  python -c "import json; d=json.loads(open('$O/l256_bs$bs.json').readline()); print('bs $bs', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
