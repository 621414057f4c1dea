# Timeline of the driver-form headline bench: kernels, copies and HIP API calls (no counters).
# Usage: bash scripts/gpu/job_timeline.sh TAG
source scripts/gpu/guard.sh
T=${1:-timeline}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step trace timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-copy-ceiling --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cat $O/bench.json
find $O/prof -name "*.csv" | head
