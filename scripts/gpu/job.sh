source scripts/gpu/guard.sh
T=${1:-r371}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 1000 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_domain.py tests/test_gpu_replicas.py tests/test_gpu_philox.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
REPS="1 2 3" bash scripts/gpu/job_ab.sh $T "e0 e1"
for rep in 1 2; do for v in e0 e1; do
SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so SV_SIZES=2048x1024 step t$v timeout -k 10 300 python scripts/perf/tile_th.py "" > $O/t_${v}_$rep.log 2>&1
grep us/sweep $O/t_${v}_$rep.log | sed "s/^/$v /"
done; done
