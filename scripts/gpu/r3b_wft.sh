# Worldline WG timeline (variant with SV_WFTIME) + the full -m gpu suite on the current tree.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_wft
mkdir -p $O
SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wftime.so step tl timeout -k 10 120 python -u scripts/perf/wg_timeline.py worldline 1024 > $O/timeline.log 2>&1
tail -16 $O/timeline.log
step tests timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
