source scripts/gpu/guard.sh
mkdir -p gpurun_out/r24
export TMPDIR=/tmp
step tests bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_replicas.py tests/test_gpu_villain.py tests/test_gpu_domain.py -x -q > gpurun_out/r24/tests.log 2>&1'
tail -3 gpurun_out/r24/tests.log
step bench bash -c 'timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r24/bench.log 2>&1'
grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r24/bench.log
step bench_abl bash -c 'SV_LIB_OVERRIDE=scripts/libsvhip_ablate4.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r24/bench_abl4.log 2>&1'
grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r24/bench_abl4.log
step reps bash -c 'timeout -k 10 300 python scripts/replica_timing.py > gpurun_out/r24/reps.log 2>&1'
cat gpurun_out/r24/reps.log
step reps_abl bash -c 'SV_LIB_OVERRIDE=scripts/libsvhip_ablate4.so timeout -k 10 300 python scripts/replica_timing.py 128 128 0 64 256 0 > gpurun_out/r24/reps_abl.log 2>&1'
cat gpurun_out/r24/reps_abl.log
for th in 32 128; do
step reps_th$th bash -c "SV_FUSED_TH=$th timeout -k 10 300 python scripts/replica_timing.py 128 128 0 1024 128 0 64 256 0 > gpurun_out/r24/reps_th$th.log 2>&1"
cat gpurun_out/r24/reps_th$th.log
done
