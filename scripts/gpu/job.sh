source scripts/gpu/guard.sh
T=${1:-r336}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_philox.py tests/test_gpu_replicas.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
REPS="1 2" bash scripts/gpu/job_ab.sh $T "p4 p5 p6" --rng philox
