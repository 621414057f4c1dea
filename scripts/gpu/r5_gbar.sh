# grid-barrier microbenchmark (scripts/perf/grid_barrier.hip)
source scripts/gpu/guard.sh
O=${OUT:-gpurun_out/r5_gbar}
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/perf/grid_barrier.hip -o $O/grid_barrier || exit 1
step g225 timeout -k 10 60 $O/grid_barrier 225 2000 > $O/g225.log 2>&1
cat $O/g225.log
step g256 timeout -k 10 60 $O/grid_barrier 256 2000 > $O/g256.log 2>&1
cat $O/g256.log
