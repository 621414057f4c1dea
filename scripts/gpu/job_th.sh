# strip-height sweep for small lattices (measurement only)
source scripts/gpu/guard.sh
O=gpurun_out/${1:-r203}
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_domain.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
for L in 256 1024; do
  for TH in 4 8 12 16 24 32 52 auto; do
    if [ $TH = auto ]; then unset SV_FUSED_TH; else export SV_FUSED_TH=$TH; fi
    step b$L-$TH timeout -k 10 120 python bench.py --L $L --steps 1000 --warmup 50 --warmup-s 0.3 --no-cpu-baseline --no-copy-ceiling > $O/b_${L}_$TH.log 2>&1
    python -c "import json,sys; d=json.loads(open('$O/b_${L}_$TH.log').read().strip().splitlines()[-1]); print('$L $TH', round(d['value']/1e9,2), 'G/s', round(d['roofline']['avg_launch_us'],2), 'us/launch', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
unset SV_FUSED_TH
