source scripts/gpu/guard.sh
# needs the timestamped build first: bash scripts/build_variant.sh wgtime -DSV_WGTIME=1
O=gpurun_out/r3_wgt; mkdir -p $O
export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so
step single timeout -k 10 120 python -u scripts/perf/wg_timeline.py single 4096 > $O/single.log 2>&1
step tile timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/tile.log 2>&1
step l256 timeout -k 10 120 python -u scripts/perf/wg_timeline.py single 256 > $O/l256.log 2>&1
cut -c1-600 $O/*.log
