# per-workgroup timeline of config 3's worldline_step_fused (variant built with -DSV_WFTIME=1)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_wftl}
mkdir -p $O
step tl env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_wftime.so timeout -k 10 200 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline.log 2>&1
