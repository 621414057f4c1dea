source scripts/gpu/guard.sh
mkdir -p gpurun_out/r31
export TMPDIR=/tmp
for a in 0 1 2 8 16 24 64; do
  if [ $a = 0 ]; then L=supervillain_amd/libsvhip.so; else L=scripts/libsvhip_ablate$a.so; fi
  step abl$a bash -c "SV_LIB_OVERRIDE=$L timeout -k 10 200 python scripts/replica_timing.py 1024 128 0 > gpurun_out/r31/abl$a.log 2>&1"
  echo "ablate $a: $(cat gpurun_out/r31/abl$a.log)"
done
