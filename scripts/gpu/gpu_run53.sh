source scripts/gpu/guard.sh
mkdir -p gpurun_out/r53
export TMPDIR=/tmp
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r53/tests.log 2>&1
tail -2 gpurun_out/r53/tests.log
for rep in 1 2; do
for v in nols ls; do
if [ $v = ls ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_$v.so; fi
step b$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r53/${v}_$rep.log 2>&1
done
done
