source scripts/gpu/guard.sh
mkdir -p gpurun_out/r106
export TMPDIR=/tmp
for rep in 1 2; do
for v in base old; do
if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so; fi
step h$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/r106/h$v$rep.log 2>&1
echo HEAD $v $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r106/h$v$rep.log)
step r$v timeout -k 10 300 python bench.py --workload replicas --no-cpu-baseline --steps 100 > gpurun_out/r106/r$v$rep.log 2>&1
echo REPS $v $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r106/r$v$rep.log)
done
done
unset SV_LIB_OVERRIDE
step p timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU -d gpurun_out/r106/pmc -o pmc --output-format csv -- python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r106/pmc.log 2>&1
step t timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_replicas.py tests/test_gpu_domain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r106/tests.log 2>&1
tail -1 gpurun_out/r106/tests.log
