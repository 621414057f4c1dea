# Round 4: the driver-form bench (python bench.py, as the round-end driver runs it) with the next batch planned while
# the device runs the current one (default) and without (SV_PREPLAN=0), two repetitions each; Villain parity first.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_preplan}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_villain.py tests/test_gpu_band.py > $O/test.log 2>&1 || { echo "[villain tests] failed"; tail -30 $O/test.log; exit 3; }
tail -1 $O/test.log
for rep in 1 2; do
  for p in 1 0; do
    SV_PREPLAN=$p timeout -k 10 300 python bench.py > $O/drv_p${p}_$rep.json 2> $O/drv_p${p}_$rep.err || { echo "[drv p=$p] failed"; tail -20 $O/drv_p${p}_$rep.err; exit 3; }
    echo "driver preplan=$p $rep $(python -c "import json; d=json.load(open('$O/drv_p${p}_$rep.json')); print(round(d['value']/1e9,3), 'G wall', round(d['ms_per_step']*1e3,2), 'us kernel', round(d['roofline']['avg_launch_us'],2))")"
  done
done
