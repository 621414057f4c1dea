set -u
mkdir -p gpurun_out/r11
SV_DEBUG_TIMING=1 timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r11/b.log 2>&1 || exit 3
cat gpurun_out/r11/b.log | grep "\[sv\]"
python -c "import json;d=json.loads(open('gpurun_out/r11/b.log').read().strip().splitlines()[-1]);print('base', round(d['value']/1e9,2),'G/s', round(d['roofline']['avg_launch_us'],1),'us', round(d['ms_per_step'],3), 'ms/step')"
