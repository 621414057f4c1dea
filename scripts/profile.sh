#!/bin/bash
# Profile the bench workload on the GPU box and summarize into profiles/.
#   bash scripts/profile.sh <tag>
# Kernel trace + stats pass, then separate --pmc passes (counters never combined with tracing
# domains other than --kernel-trace), per MI355X_MICROARCH.md "rocprofv3 PMC slots".
set -u
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT profiles
B="python bench.py --no-cpu-baseline"  # the default command (200 + 20 sweeps) without the CPU leg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || exit 3
P="timeout -k 10 300 rocprofv3 --kernel-include-regex villain_sweep_hot"
Bs="python bench.py --steps 4 --warmup 1 --no-cpu-baseline"
$P --pmc FETCH_SIZE -d $OUT/fetch -o p --output-format csv -- $Bs > $OUT/fetch.log 2>&1 || exit 3
$P --pmc WRITE_SIZE -d $OUT/write -o p --output-format csv -- $Bs > $OUT/write.log 2>&1 || exit 3
$P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/sq1 -o p --output-format csv -- $Bs > $OUT/sq1.log 2>&1 || exit 3
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/sq2 -o p --output-format csv -- $Bs > $OUT/sq2.log 2>&1 || exit 3
python scripts/summarize_profile.py $OUT $TAG
# kernel-trace summaries of the other workloads (BASELINE configs 3 and 5)
for w in replicas worldline hammer wlhammer; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline > $OUT/trace_$w.log 2>&1 || exit 3
  cp $OUT/trace_$w/run_kernel_stats.csv profiles/${TAG}_kernel_stats_$w.csv
done
