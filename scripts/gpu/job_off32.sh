# villain_sweep_hot with 32-bit row offsets (default) vs 64-bit addressing (variant off0): suites, then A/B bench lines.
# Usage: bash scripts/gpu/job_off32.sh TAG
source scripts/gpu/guard.sh
T=${1:-off32}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_boundary.py tests/test_gpu_pipeline.py tests/test_gpu_replicas.py tests/test_gpu_philox.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
REPS="1 2 3" ABARGS="--steps 300 --warmup 20" bash scripts/gpu/job_ab.sh $T "off0 cur" || exit 1
