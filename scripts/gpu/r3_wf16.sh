# 16-wave worldline_step_fused: bit-exactness (the Worldline suites with SV_WF_NW=16) and step time vs strip height.
source scripts/gpu/guard.sh
O=gpurun_out/r3_wf16; mkdir -p $O
step t env SV_WF_NW=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_worldline.py tests/test_gpu_wdomain.py > $O/t.log 2>&1
tail -2 $O/t.log
B="--workload worldline --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling"
for cfg in "8 40" "16 41" "16 25" "16 57" "16 33" "8 40"; do
  set -- $cfg
  step w$1_$2 env SV_WF_NW=$1 SV_WF_TH=$2 timeout -k 10 200 python -u bench.py $B > $O/w$1_$2.json 2> $O/w$1_$2.err
  python -c "import json; d=json.loads(open('$O/w$1_$2.json').readline()); print('NW=$1 TH=$2', round(d['value']/1e9,2), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3))"
done
