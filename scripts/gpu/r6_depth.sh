# Round 6: the config-4 N = 8 tile through RCCL loopback by halo depth (sweeps per exchange), prediction on
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_depth
mkdir -p $O
step depth timeout -k 10 300 python -u scripts/perf/domain_depth_cost.py 3 2,4,6,8 > $O/depth.log 2>&1
cat $O/depth.log
