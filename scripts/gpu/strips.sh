source scripts/gpu/guard.sh
O=gpurun_out/r3_strips; mkdir -p $O
step ab timeout -k 10 300 python -u scripts/perf/strips_ab.py 4096 200 3 uniform 56x5,40x5,32 48x9,44,36 56x7,32x3,24 64x7,20x3,4 52x7,40x3,28 40x12,32 60x4,40x6,32 > $O/ab.log 2>&1
cat $O/ab.log
export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so
step single timeout -k 10 120 python -u scripts/perf/wg_timeline.py single 4096 > $O/single.log 2>&1
step tile timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/tile.log 2>&1
cut -c1-400 $O/single.log $O/tile.log | grep -v resident
