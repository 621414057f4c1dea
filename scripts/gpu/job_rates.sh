# instruction-rate microbenchmark + copy ceiling (measurement only)
source scripts/gpu/guard.sh
O=gpurun_out/${1:-r202}
mkdir -p $O
step rates timeout -k 10 120 ./scripts/perf/isa_rates > $O/rates.log 2>&1
cat $O/rates.log
step copy timeout -k 10 120 python scripts/perf/copy_calibrate.py > $O/copy.log 2>&1
cat $O/copy.log
