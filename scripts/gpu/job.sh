source scripts/gpu/guard.sh
T=${1:-r358}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
REPS="1 2" bash scripts/gpu/job_ab.sh $T "d0 d1"
REPS="1" ABARGS="--steps 1000 --warmup 50" bash scripts/gpu/job_ab.sh ${T}w "d0 d1" --workload worldline
REPS="1" ABARGS="--steps 200" bash scripts/gpu/job_ab.sh ${T}r "d0 d1" --workload replicas
