# 32-bit row offsets in tile mode: domain + Villain suites, then the N = 8 tile per-sweep time, cur vs off0 (64-bit).
# Usage: bash scripts/gpu/job_off32t.sh TAG
source scripts/gpu/guard.sh
T=${1:-off32t}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_domain.py tests/test_gpu_villain.py tests/test_gpu_replicas.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for r in 1 2; do
  for v in off0 cur; do
    SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so SV_SIZES=2048x1024 step t$v timeout -k 10 200 python -u scripts/perf/tile_th.py > $O/t_${v}_$r.log 2>&1
    echo "$v $r $(tail -1 $O/t_${v}_$r.log)"
  done
done
