source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_stl}
mkdir -p $O
step stl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 200 python -u scripts/perf/split_timeline.py 0.37 > $O/stl.log 2>&1
cat $O/stl.log
step rw timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window.log 2>&1
cat $O/reject_window.log
