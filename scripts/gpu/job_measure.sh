# round measurement: every bench line (headline default and driver-style, configs 2/3/5, 8(f) rows)
source scripts/gpu/guard.sh
T=${1:-r215}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1; shift; step $name timeout -k 10 400 python bench.py "$@" > $O/bench_$name.log 2>&1; grep '^{' $O/bench_$name.log | tail -1 > $O/bench_$name.json; echo $name $(cut -c1-160 $O/bench_$name.json); }
run default
run driver20 --gpus 1 --steps 20 --warmup 5
run l256 --L 256 --steps 2000 --warmup 100
run worldline --workload worldline --steps 200 --warmup 20
run replicas --workload replicas --steps 50 --warmup 5
run worms --workload worms --steps 200 --kappa 1.0 --no-cpu-baseline
run hammer --workload hammer --steps 50 --warmup 5 --no-cpu-baseline
run wlhammer --workload wlhammer --steps 50 --warmup 5 --no-cpu-baseline
echo done
