source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r5_splitdbg}
mkdir -p $O
step dbg timeout -k 10 400 python -u scripts/perf/split_dbg.py > $O/dbg.log 2> $O/dbg.err
cat $O/dbg.log; tail -5 $O/dbg.err
