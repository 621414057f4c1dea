set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r8
echo "== pytest villain"; timeout -k 10 900 python -m pytest tests/test_gpu_villain.py -m gpu -q -x --timeout 600 -p no:cacheprovider > gpurun_out/r8/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r8/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline > gpurun_out/r8/b.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/r8/b.log').read().strip().splitlines()[-1]);print(round(d['value']/1e9,2),'G/s', round(d['roofline']['avg_launch_us'],1),'us', round(d['ms_per_step'],3), 'ms/step')"
P="timeout -k 10 300 rocprofv3 --kernel-include-regex villain_sweep_fused"
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline"
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/r8/pmc1 -o p --output-format csv -- $B > gpurun_out/r8/pmc1.log 2>&1 || echo pmc1 failed
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES -d gpurun_out/r8/pmc2 -o p --output-format csv -- $B > gpurun_out/r8/pmc2.log 2>&1 || echo pmc2 failed
$P --pmc SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 -d gpurun_out/r8/pmc5 -o p --output-format csv -- $B > gpurun_out/r8/pmc5.log 2>&1 || echo pmc5 failed
echo done
