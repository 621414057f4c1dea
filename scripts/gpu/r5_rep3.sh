source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_rep3}
mkdir -p $O
step repdbg env SV_DEBUG_TIMING=1 timeout -k 10 300 python -u bench.py --workload replicas --no-cpu-baseline --steps 200 --warmup 2 --warmup-s 0 > $O/repdbg.json 2> $O/repdbg.err
grep "sv replicas" $O/repdbg.err | tail -12
