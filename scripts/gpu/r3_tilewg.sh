# WG timelines of the 2048x1024 tile at the automatic strip height and at TH=20 (needs the SV_WGTIME build).
source scripts/gpu/guard.sh
O=gpurun_out/r3_tilewg; mkdir -p $O
export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so
step auto timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/auto.log 2>&1
step th20 env SV_FUSED_TH=20 timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/th20.log 2>&1
step th12 env SV_FUSED_TH=12 timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/th12.log 2>&1
grep -h "group 2" $O/*.log | cut -c1-700
