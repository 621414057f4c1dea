# Host-side phase timings of the driver-form bench (SV_DEBUG_TIMING).  Usage: bash scripts/gpu/job_hosttime.sh TAG
source scripts/gpu/guard.sh
T=${1:-hosttime}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SV_DEBUG_TIMING=1 step bench1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-copy-ceiling > $O/bench1.json 2> $O/bench1.err
cat $O/bench1.json
tail -12 $O/bench1.err
step bench2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-copy-ceiling > $O/bench2.json 2> $O/bench2.err
cat $O/bench2.json
