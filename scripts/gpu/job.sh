source scripts/gpu/guard.sh
T=${1:-r374}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
REPS="1 2 3" bash scripts/gpu/job_ab.sh $T "prev cur"
REPS="1 2" bash scripts/gpu/job_ab.sh ${T}p "prev cur" --rng philox
