# Round 6: the headline kernel's HBM path -- no row stores (SV_ABLATE=8) and no row loads (SV_ABLATE=16), timing only
# (results wrong by construction), and the row stores at a fixed count per row step (SV_FIXSTORE=1: junk slots past
# the lattice for rows with nothing to store, so the prefetch wait is vmcnt(6), not vmcnt(0)), against the tree;
# then the Villain / split / overflow suites on the fixed-count variant
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_ablate
mkdir -p $O
V=supervillain_amd/variants
for r in 1 2 3; do
  step b$r timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  step fix$r env SV_LIB_OVERRIDE=$V/libsvhip_fix.so timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/fix_$r.json 2> $O/fix_$r.err
done
for v in a8 a16; do
  step $v env SV_LIB_OVERRIDE=$V/libsvhip_$v.so timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/${v}.json 2> $O/${v}.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
step t env SV_LIB_OVERRIDE=$V/libsvhip_fix.so timeout -k 10 600 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_split.py tests/test_gpu_overflow.py tests/test_gpu_pipeline.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_fix.log 2>&1
tail -2 $O/tests_fix.log
