# Round 4: headline-kernel micro-optimisations A/B (variants built by scripts/build_variant.sh): early row prefetch
# (SV_HOT_PF_EARLY), sign-extending n loads (SV_HOT_I16), one-shift u53 (SV_HOT_U53=2), per-lane word bases
# (SV_HOT_BSEL), all four; parity of the combined variant first.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_hot_ab}
mkdir -p $O
V=$PWD/supervillain_amd/variants
SV_LIB_OVERRIDE=$V/libsvhip_hall.so timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_worldline.py > $O/test_all.log 2>&1 || { echo "[tests hall] failed"; tail -30 $O/test_all.log; exit 3; }
tail -1 $O/test_all.log
for rep in 1 2; do
  for v in base hpf hi16 hu53 hbsel hall; do
    if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=$V/libsvhip_$v.so; fi
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/vh_${v}_$rep.json 2> $O/vh_${v}_$rep.err || { echo "[vh $v] failed"; tail -20 $O/vh_${v}_$rep.err; exit 3; }
    echo "vh $v $rep $(python -c "import json; d=json.load(open('$O/vh_${v}_$rep.json')); print(round(d['value']/1e9,3), round(d['roofline']['avg_launch_us'],2))")"
  done
done
