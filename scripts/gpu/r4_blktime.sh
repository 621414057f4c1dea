# villain_sweep_block workgroup timeline (variant -DSV_BLKTIME=1), L=256 at K = 3 and 5, and block sides 8 / 32 timed
source scripts/gpu/guard.sh
O=gpurun_out/r4_blktime
mkdir -p $O
for K in 3 5; do
  step tl$K env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_blktime.so timeout -k 10 120 python -u scripts/perf/block_timeline.py 256 63 $K > $O/timeline_K$K.log 2>&1
  cat $O/timeline_K$K.log
done
for bs in 8 32; do
  step bs$bs env SV_BLOCK_BS=$bs timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_bs$bs.json 2> $O/l256_bs$bs.err
  python -c "import json; d=json.loads(open('$O/l256_bs$bs.json').readline()); print('bs $bs', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
done
