source scripts/gpu/guard.sh
mkdir -p gpurun_out/r40
export TMPDIR=/tmp
step tests bash -c 'timeout -k 10 600 python -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py -x -q > gpurun_out/r40/tests.log 2>&1'
tail -2 gpurun_out/r40/tests.log
for a in 0 1 2 8 16 24 64; do
  if [ $a = 0 ]; then L=supervillain_amd/libsvhip.so; else L=scripts/libsvhip_ablate$a.so; fi
  step abl$a bash -c "SV_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r40/abl$a.log 2>&1"
  echo "ablate $a: $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r40/abl$a.log)"
done
