source scripts/gpu/guard.sh
mkdir -p gpurun_out/r51
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r51/tests.log 2>&1
tail -2 gpurun_out/r51/tests.log
step b1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r51/bench1.log 2>&1
step b2 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r51/bench2.log 2>&1
step b3 timeout -k 10 300 python bench.py --workload replicas --no-cpu-baseline > gpurun_out/r51/replicas.log 2>&1
