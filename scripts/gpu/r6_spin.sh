# Round 6: HIP's synchronization mode (SV_SPIN=1: hipDeviceScheduleSpin, 2: Yield, before the context's first work)
# against the default, on the lines whose wall exceeds their kernel time most: config 3, config 2, the headline
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_spin
mkdir -p $O
env SV_SPIN=1 SV_DEBUG_TIMING=1 timeout -k 10 60 python -u bench.py --workload worldline --steps 5 --warmup 1 --no-cpu-baseline --no-copy-ceiling 2>&1 | grep -m2 "hipSetDeviceFlags" || true
for r in 1 2; do
  for sp in 0 1 2; do
    step w$sp$r env SV_SPIN=$sp timeout -k 10 120 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_s${sp}_$r.json 2> $O/wl_s${sp}_$r.err
    step l$sp$r env SV_SPIN=$sp timeout -k 10 120 python -u bench.py --L 256 --no-cpu-baseline --no-copy-ceiling > $O/l256_s${sp}_$r.json 2> $O/l256_s${sp}_$r.err
    step h$sp$r env SV_SPIN=$sp timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-copy-ceiling > $O/head_s${sp}_$r.json 2> $O/head_s${sp}_$r.err
  done
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
