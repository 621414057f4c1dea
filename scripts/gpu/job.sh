source scripts/gpu/guard.sh
T=${1:-r214}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --workload worldline --steps 20 --warmup 2 --warmup-s 0.2 --no-cpu-baseline --no-copy-ceiling"
step sq1 timeout -s KILL 120 rocprofv3 --kernel-include-regex worldline_step_fused --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $O/sq1 -o p --output-format csv -- $B > $O/sq1.log 2>&1
step sq2 timeout -s KILL 120 rocprofv3 --kernel-include-regex worldline_step_fused --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/sq2 -o p --output-format csv -- $B > $O/sq2.log 2>&1
step tr timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1
echo done
