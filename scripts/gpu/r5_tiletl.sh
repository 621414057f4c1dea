# where the 2048 x 1024 tile's extra time goes -- per-workgroup timelines (-DSV_WGTIME=1 variant) of
# the tile's exact-tile launch and of the single L=4096 lattice, and the per-launch kernel times of a 4-sweep group
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tiletl}
mkdir -p $O
step tl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py tile 2048 1024 > $O/tile_tl.log 2>&1
step sl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py single 4096 > $O/single_tl.log 2>&1
step kt env SV_SIZES=2048x1024 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python scripts/perf/deep_halo.py 4 > $O/kt.log 2>&1
cat $O/kt.log | tail -3
tail -12 $O/tile_tl.log
