# Round 6: the exact statistics (common.h) -- the full -m gpu suite, then the headline / config-5 / tile lines A/B
# against the round-5 kernels (variants/libsvhip_r5base.so = HEAD before the exact sums), and the domain E_N lines.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_exact
mkdir -p $O
B=supervillain_amd/variants/libsvhip_r5base.so
step suite timeout -k 10 1500 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
for r in 1 2; do
  step hn$r timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/head_new_$r.json 2> $O/head_new_$r.err
  step hb$r env SV_LIB_OVERRIDE=$B timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/head_base_$r.json 2> $O/head_base_$r.err
done
for r in 1 2; do
  step rn$r timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_new_$r.json 2> $O/rep_new_$r.err
  step rb$r env SV_LIB_OVERRIDE=$B timeout -k 10 200 python -u bench.py --workload replicas --no-cpu-baseline --no-copy-ceiling > $O/rep_base_$r.json 2> $O/rep_base_$r.err
  step wn$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
  step wb$r env SV_LIB_OVERRIDE=$B timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step ln$r timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline --no-copy-ceiling > $O/l256_new_$r.json 2> $O/l256_new_$r.err
done
for r in 1 2; do
  step ts$r timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/tiles_strong_$r.json 2> $O/tiles_strong_$r.err
  step tw$r timeout -k 10 300 python -u bench.py --tiles 2x4 --weak --steps 20 --warmup 5 --no-cpu-baseline --no-copy-ceiling > $O/tiles_weak_$r.json 2> $O/tiles_weak_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
