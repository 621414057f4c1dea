# Round 6: 16-byte row accesses in villain_sweep_hot (variants/libsvhip_wide.so, -DSV_WIDE=1; the tree: even strip
# boundaries, 8-byte accesses) -- headline, config 5, the 2x4 tile emulation, interleaved; then the Villain, split,
# overflow, domain, replica and observables suites on the wide variant
source scripts/gpu/guard.sh
export TMPDIR=/tmp
export SV_DOMAIN_PREDICT=0
O=gpurun_out/r6_wide
mkdir -p $O
W=supervillain_amd/variants/libsvhip_wide.so
for r in 1 2 3; do
  step hb$r timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/head_base_$r.json 2> $O/head_base_$r.err
  step hw$r env SV_LIB_OVERRIDE=$W timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/head_wide_$r.json 2> $O/head_wide_$r.err
done
for r in 1 2; do
  step rb$r timeout -k 10 120 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_base_$r.json 2> $O/rep_base_$r.err
  step rw$r env SV_LIB_OVERRIDE=$W timeout -k 10 120 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_wide_$r.json 2> $O/rep_wide_$r.err
  step tb$r timeout -k 10 150 python -u bench.py --tiles 2x4 --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t8_base_$r.json 2> $O/t8_base_$r.err
  step tw$r env SV_LIB_OVERRIDE=$W timeout -k 10 150 python -u bench.py --tiles 2x4 --steps 100 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/t8_wide_$r.json 2> $O/t8_wide_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
unset SV_DOMAIN_PREDICT
step t env SV_LIB_OVERRIDE=$W timeout -k 10 900 python -u -m pytest tests/test_gpu_villain.py tests/test_gpu_split.py tests/test_gpu_overflow.py tests/test_gpu_domain.py tests/test_gpu_replicas.py tests/test_gpu_observables.py tests/test_gpu_band.py tests/test_gpu_block.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_wide.log 2>&1
tail -3 $O/tests_wide.log
