# Re-run of the full -m gpu suite (one illegal-address failure at the first Worldline domain test in r3b_wft), then
# the worldline WG timeline.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_wft2
mkdir -p $O
step tests timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wftime.so step tl timeout -k 10 120 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline.log 2>&1
tail -16 $O/timeline.log
