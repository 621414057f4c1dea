# Prologue split (entry -> row bases -> loop) of the hot kernel: tile 2048x1024, L=256, L=4096 (SV_WGTIME build).
source scripts/gpu/guard.sh
O=gpurun_out/r3_prolog; mkdir -p $O
export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so
step tile timeout -k 10 120 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/tile.log 2>&1
step l256 timeout -k 10 120 python -u scripts/perf/wg_timeline.py single 256 > $O/l256.log 2>&1
step l4096 timeout -k 10 120 python -u scripts/perf/wg_timeline.py single 4096 > $O/l4096.log 2>&1
grep -h "prologue" $O/*.log | cut -c1-400
