# config 5 tail-recovery potential: one 1024-replica batch vs two 512-replica batches on two streams
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tworep}
mkdir -p $O
step two timeout -k 10 300 python -u scripts/perf/two_streams_replicas.py 200 > $O/two.log 2>&1
cat $O/two.log
