# Reference-order Worldline bench line, and the L=256 kernel trace (kernel time vs gaps between launches).
source scripts/gpu/guard.sh
O=gpurun_out/r3_m1; mkdir -p $O
export TMPDIR=/tmp
step wlref timeout -k 10 300 python -u bench.py --workload worldline --L 1024 --plaquette reference --steps 10 --warmup 2 > $O/wlref.json 2> $O/wlref.err
cat $O/wlref.json; tail -3 $O/wlref.err
step l256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/l256 -o run --output-format csv -- python bench.py --L 256 --steps 2000 --warmup 100 --no-cpu-baseline --no-copy-ceiling > $O/l256.json 2> $O/l256.err
cat $O/l256.json
