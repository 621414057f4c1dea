source scripts/gpu/guard.sh
mkdir -p gpurun_out/r88
for proto in default LL LL128 Simple; do
if [ $proto = default ]; then unset NCCL_PROTO; else export NCCL_PROTO=$proto; fi
step lb_$proto timeout -k 10 200 python scripts/perf/loopback_cost.py > gpurun_out/r88/lb_$proto.log 2>&1
echo PROTO $proto $(grep "loopback=True" gpurun_out/r88/lb_$proto.log)
done
