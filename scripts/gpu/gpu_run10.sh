set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r10
timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r10/b.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/r10/b.log').read().strip().splitlines()[-1]);print('base', round(d['value']/1e9,2),'G/s', round(d['roofline']['avg_launch_us'],1),'us', round(d['ms_per_step'],3), 'ms/step')"
for a in 1 2 3; do
SV_LIB_OVERRIDE=$PWD/scripts/libsvhip_ablate$a.so timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r10/a$a.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/r10/a$a.log').read().strip().splitlines()[-1]);print('ablate$a', round(d['value']/1e9,2),'G/s', round(d['roofline']['avg_launch_us'],1),'us', round(d['ms_per_step'],3), 'ms/step')"
done
