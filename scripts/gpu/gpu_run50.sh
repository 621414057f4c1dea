source scripts/gpu/guard.sh
mkdir -p gpurun_out/r50
export TMPDIR=/tmp
for it in 1 2 4 8 16; do
for w in worldline site exact vortex; do
SV_GS_ITERS=$it step b$w$it timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r50/${w}_$it.log 2>&1
done
done
for it in 1 4 16; do
SV_GS_ITERS=$it step bl$it timeout -k 10 300 python bench.py --workload worldline --L 4096 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r50/wl4096_$it.log 2>&1
done
