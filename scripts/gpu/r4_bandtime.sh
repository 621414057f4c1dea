# Round 4: per-sweep timeline of the band launches (wgtime variant), then the VALU ablation passes (r4_ablate.sh).
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_bandtime}
mkdir -p $O
SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 120 python -u scripts/perf/band_timeline.py 256 63 > $O/band_k7.log 2>&1 || { echo "[bandtime] failed"; tail -20 $O/band_k7.log; exit 3; }
SV_BAND_K=3 SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_wgtime.so timeout -k 10 120 python -u scripts/perf/band_timeline.py 256 63 > $O/band_k3.log 2>&1 || { echo "[bandtime k3] failed"; tail -20 $O/band_k3.log; exit 3; }
cat $O/band_k7.log $O/band_k3.log
OUT=r4_ablate bash scripts/gpu/r4_ablate.sh
