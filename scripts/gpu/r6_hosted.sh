# Round 6: two real ranks on one GPU through the hosted transport (sv_domain_create_hosted over gloo) -- Villain and
# Worldline 1 x 2, forced rejections, with and without rejection prediction; then the domain suites (unchanged paths)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_hosted
mkdir -p $O
step two timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_00_two_ranks.py -m gpu > $O/two.log 2>&1
grep -E "PASS|FAIL|XFAIL|ERROR|passed|failed" $O/two.log | tail -12
step dom timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_domain.py tests/test_gpu_wdomain.py -m gpu > $O/dom.log 2>&1
tail -2 $O/dom.log
