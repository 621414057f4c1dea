# Gaps between hot launches vs the enqueue chunk (SV_CHUNK: 4 default, 16, 0 = the whole 64-sweep batch).
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3_chunk; mkdir -p $O
for ch in 4 16 0; do
  step c$ch env SV_CHUNK=$ch timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c$ch -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/c$ch.json 2> $O/c$ch.err
  python scripts/perf/gap_stats.py $O/c$ch/run_kernel_trace.csv
  python -c "import json; d=json.loads(open('$O/c$ch.json').readline()); print('chunk $ch', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), d['config']['lemire_rejections_in_timed_steps'])"
done
