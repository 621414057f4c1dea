# worldline_step_fused, 8 waves: strip heights and occupancy.  Usage: bash scripts/gpu/job_wfth.sh TAG
source scripts/gpu/guard.sh
T=${1:-wfth}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
one() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env "$@" SV_LIB_OVERRIDE=$lib timeout -k 10 200 python -u bench.py --workload worldline --steps 400 --warmup 20 --no-copy-ceiling --no-cpu-baseline > $O/$name.json 2> $O/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc"; exit $rc; fi
  python -c "import json; d=json.loads(open('$O/$name.json').readline()); print('$name', round(d['value']/1e9,2), round(d['roofline']['avg_launch_us'],2))"
}
D=supervillain_amd/libsvhip.so
V=supervillain_amd/variants/libsvhip_wf8o4.so
SV_LIB_OVERRIDE=$V SV_WF_NW=8 step tests8o4 timeout -k 10 400 python -u -m pytest tests/test_gpu_worldline.py tests/test_gpu_wdomain.py -x -q --timeout 120 --timeout-method thread > $O/tests8o4.log 2>&1
tail -1 $O/tests8o4.log
for r in 1 2; do
  one nw4_$r $D SV_WF_NW=4
  one nw8_th32_$r $D SV_WF_NW=8 SV_WF_TH=32
  one nw8_th40_$r $D SV_WF_NW=8
  one nw8_th48_$r $D SV_WF_NW=8 SV_WF_TH=48
  one o4_th24_$r $V SV_WF_NW=8
  one o4_th16_$r $V SV_WF_NW=8 SV_WF_TH=16
  one o4_th32_$r $V SV_WF_NW=8 SV_WF_TH=32
done
