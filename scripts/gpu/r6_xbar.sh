# Round 6: the XCD-local barrier (32 workgroups per XCD, the band launches' form) against the device-wide one
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_xbar
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/perf/xcd_barrier.hip -o $O/xcd_barrier 2> $O/build.err || { echo build failed; exit 1; }
step xbar timeout -k 10 60 $O/xcd_barrier 2000 > $O/xbar.log 2>&1
cat $O/xbar.log
