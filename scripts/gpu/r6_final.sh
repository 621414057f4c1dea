# End-of-round evidence, part A: full -m gpu suite (runtime error log on), smoke, the bench lines.
# Part B (scripts/gpu/r6_final_prof.sh): the rocprofv3 trace + PMC passes.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6_final}
mkdir -p $O/bench
export AMD_LOG_LEVEL=1
step tests timeout -k 10 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for r in 1 2 3; do
  step d$r timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench/driver_$r.json 2> $O/bench/driver_$r.err
done
step def timeout -k 10 200 python -u bench.py > $O/bench/default.json 2> $O/bench/default.err
step wl timeout -k 10 120 python -u bench.py --workload worldline > $O/bench/worldline.json 2> $O/bench/worldline.err
step wlref timeout -k 10 120 python -u bench.py --workload worldline --plaquette reference --steps 20 --warmup 3 > $O/bench/worldline_reference.json 2> $O/bench/worldline_reference.err
step l256 timeout -k 10 120 python -u bench.py --L 256 > $O/bench/l256.json 2> $O/bench/l256.err
step rep timeout -k 10 120 python -u bench.py --workload replicas > $O/bench/replicas.json 2> $O/bench/replicas.err
step t8 timeout -k 10 150 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles2x4.json 2> $O/bench/tiles2x4.err
step t8w timeout -k 10 200 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 3 --no-cpu-baseline > $O/bench/tiles2x4_weak.json 2> $O/bench/tiles2x4_weak.err
step t4 timeout -k 10 150 python -u bench.py --tiles 2x2 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles2x2.json 2> $O/bench/tiles2x2.err
step t2 timeout -k 10 150 python -u bench.py --tiles 1x2 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles1x2.json 2> $O/bench/tiles1x2.err
for f in $O/bench/*.json; do python scripts/summ_line.py $f; done
