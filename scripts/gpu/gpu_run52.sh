source scripts/gpu/guard.sh
mkdir -p gpurun_out/r52
export TMPDIR=/tmp
for rep in 1 2; do
for v in base k3 sw all; do
if [ $v = all ]; then unset SV_LIB_OVERRIDE; else export SV_LIB_OVERRIDE=$PWD/supervillain_amd/variants/libsvhip_$v.so; fi
step b$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/r52/${v}_$rep.log 2>&1
done
done
