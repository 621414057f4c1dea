# villain_sweep_block: blocks dealt to the XCDs round-robin (0) or in contiguous runs (1), L=256, three repetitions
source scripts/gpu/guard.sh
O=gpurun_out/r4_xcd
mkdir -p $O
for rep in 1 2 3; do
  for x in 0 1; do
    step xcd$x env SV_BLOCK_XCD=$x timeout -k 10 200 python -u bench.py --L 256 --no-cpu-baseline > $O/l256_xcd${x}_$rep.json 2> $O/l256_xcd${x}_$rep.err
    python -c "import json; d=json.loads(open('$O/l256_xcd${x}_$rep.json').readline()); print('xcd$x', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"
  done
done
