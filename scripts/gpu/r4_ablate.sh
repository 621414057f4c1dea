# Round 4: where the VALU instructions of the two hot kernels go.  Ablation variants (fused.h SV_ABLATE: 1 no exp,
# 2 no PCG64 compositions, 8 no HBM stores, 16 no HBM loads, 32 no barriers) -- results wrong by construction, only
# counted and timed -- each under one rocprofv3 PMC pass per kernel.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_ablate}
mkdir -p $O
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for v in base a1 a2 a3 a24 a59; do
  if [ $v = base ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_$v.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-include-regex villain_sweep_hot --pmc $C -d $O/vh_$v -o p --output-format csv -- python bench.py --steps 12 --warmup 2 --no-cpu-baseline > $O/vh_$v.log 2>&1 || { echo "[vh $v] failed"; exit 3; }
  timeout -s KILL 120 rocprofv3 --kernel-include-regex worldline_step_fused --pmc $C -d $O/wf_$v -o p --output-format csv -- python bench.py --workload worldline --steps 12 --warmup 2 --no-cpu-baseline > $O/wf_$v.log 2>&1 || { echo "[wf $v] failed"; exit 3; }
  echo "[$v] done"
done
python scripts/perf/ablate_summary.py $O
