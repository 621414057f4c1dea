# config 5 host timeline per batch (SV_DEBUG_TIMING)
source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r5_repdbg}
mkdir -p $O
step dbg env SV_DEBUG_TIMING=1 timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline > $O/rep.json 2> $O/rep.err
grep -c "sv replicas" $O/rep.err
tail -30 $O/rep.err
