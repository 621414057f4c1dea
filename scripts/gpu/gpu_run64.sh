source scripts/gpu/guard.sh
mkdir -p gpurun_out/r64
export TMPDIR=/tmp
SV_DOMAIN_SPLIT=0 step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r64/prof -o run --output-format csv -- python scripts/perf/loopback_only.py > gpurun_out/r64/prof.log 2>&1
grep "per sweep" gpurun_out/r64/prof.log
find gpurun_out/r64/prof -name "*kernel_stats.csv" | head -2
