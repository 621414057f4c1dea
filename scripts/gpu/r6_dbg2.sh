source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_dbg2
mkdir -p $O
step dbg env SV_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/perf/split_two_dbg.py 'different rows' 'same row' > $O/split_two.log 2>&1
cat $O/split_two.log
