# worldline_step_fused 4 vs 8 waves: bit-exact suites with 8 waves forced, then A/B bench lines; host phase timings of
# the headline bench.  Usage: bash scripts/gpu/job_wfnw.sh TAG
source scripts/gpu/guard.sh
T=${1:-wfnw}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SV_WF_NW=8 step tests8 timeout -k 10 400 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wdomain.py -x -q --timeout 120 --timeout-method thread > $O/tests8.log 2>&1
tail -2 $O/tests8.log
for r in 1 2; do
  for nw in 4 8; do
    SV_WF_NW=$nw step wl$nw timeout -k 10 200 python -u bench.py --workload worldline --steps 400 --warmup 20 --no-copy-ceiling > $O/wl${nw}_$r.json 2> $O/wl${nw}_$r.err
    python -c "import json,sys; d=json.load(open('$O/wl${nw}_$r.json')); print('nw=$nw', d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
  done
done
SV_DEBUG_TIMING=1 step bench1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-copy-ceiling > $O/bench1.json 2> $O/bench1.err
cat $O/bench1.json
tail -12 $O/bench1.err
