source scripts/gpu/guard.sh
T=${1:-r379}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_s1.so step tests timeout -k 10 900 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_domain.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
REPS="1 2 3" bash scripts/gpu/job_ab.sh $T "s0 s1"
REPS="1 2" ABARGS="--steps 200" bash scripts/gpu/job_ab.sh ${T}r "s0 s1" --workload replicas
