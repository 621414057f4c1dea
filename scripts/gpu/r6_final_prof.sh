# End-of-round evidence, part B: rocprofv3 kernel trace + stats of the default bench command and PMC passes for the
# headline kernel (scripts/profile.sh r06), worldline_step_fused PMC (VALU per plaquette-step)
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6_final}
mkdir -p $O
step prof timeout -k 10 900 bash scripts/profile.sh ${PTAG:-r06}
step wfpmc timeout -s KILL 120 rocprofv3 --kernel-include-regex worldline_step_fused --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/wf_pmc -o p --output-format csv -- python bench.py --workload worldline --steps 12 --warmup 2 --no-cpu-baseline > $O/wf_pmc.log 2>&1
echo done
# config 3's wall time again (part A's box read 41.2 us wall against 34.9 kernel)
for r in 1 2; do
  step wl$r timeout -k 10 120 python -u bench.py --workload worldline > $O/worldline_again_$r.json 2> $O/worldline_again_$r.err
done
for f in $O/worldline_again_*.json; do python scripts/summ_line.py $f; done
