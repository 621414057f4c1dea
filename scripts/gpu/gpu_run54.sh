source scripts/gpu/guard.sh
mkdir -p gpurun_out/r54
export TMPDIR=/tmp
for rep in 1 2; do
for v in nols ls2 ls4w2; do
export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_$v.so
step b$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r54/${v}_$rep.log 2>&1
done
done
unset SV_LIB_OVERRIDE
export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_ls2.so
step tests timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r54/tests.log 2>&1
tail -2 gpurun_out/r54/tests.log
