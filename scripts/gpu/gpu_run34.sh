source scripts/gpu/guard.sh
mkdir -p gpurun_out/r34
export TMPDIR=/tmp
for th in 8 16 32 64; do
step reps$th bash -c "SV_FUSED_TH=$th timeout -k 10 300 python scripts/replica_timing.py 128 128 1 1024 128 1 64 256 1 > gpurun_out/r34/reps$th.log 2>&1"
cat gpurun_out/r34/reps$th.log
done
