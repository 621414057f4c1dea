# End-of-round evidence: full -m gpu suite (runtime error log on), smoke, bench lines, headline trace + PMC
# (scripts/profile.sh r05), worldline_step_fused PMC (VALU per plaquette-step).
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_final}
mkdir -p $O/bench
export AMD_LOG_LEVEL=1
if [ "${TESTS:-1}" = 1 ]; then
step tests timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
fi
unset AMD_LOG_LEVEL
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2 3; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench/driver_$r.json 2> $O/bench/driver_$r.err
done
step def timeout -k 10 300 python -u bench.py > $O/bench/default.json 2> $O/bench/default.err
step wl timeout -k 10 300 python -u bench.py --workload worldline > $O/bench/worldline.json 2> $O/bench/worldline.err
step wlref timeout -k 10 300 python -u bench.py --workload worldline --plaquette reference --steps 20 --warmup 3 > $O/bench/worldline_reference.json 2> $O/bench/worldline_reference.err
step l256 timeout -k 10 300 python -u bench.py --L 256 > $O/bench/l256.json 2> $O/bench/l256.err
step rep timeout -k 10 300 python -u bench.py --workload replicas > $O/bench/replicas.json 2> $O/bench/replicas.err
step t8w env SV_DOMAIN_PREDICT=1 timeout -k 10 300 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 3 --no-cpu-baseline > $O/bench/tiles2x4_weak.json 2> $O/bench/tiles2x4_weak.err
step t8 timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles2x4.json 2> $O/bench/tiles2x4.err
for f in $O/bench/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3), d['config'].get('lemire_rejections_in_timed_steps'))"; done
step prof timeout -k 10 900 bash scripts/profile.sh ${PTAG:-r05}
step wfpmc timeout -s KILL 120 rocprofv3 --kernel-include-regex worldline_step_fused --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/wf_pmc -o p --output-format csv -- python bench.py --workload worldline --steps 12 --warmup 2 --no-cpu-baseline > $O/wf_pmc.log 2>&1
mkdir -p $O/ab && cp -r $O/wf_pmc $O/ab/wf_base && python scripts/perf/ablate_summary.py $O/ab
