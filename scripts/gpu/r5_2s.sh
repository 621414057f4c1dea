# tail-recovery potential: two independent L=4096 chains on two streams vs one (scripts/perf/two_streams.py)
source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r5_2s}
mkdir -p $O
step ts timeout -k 10 300 python -u scripts/perf/two_streams.py 4096 200 > $O/ts.log 2>&1
cat $O/ts.log | grep "L="
