# Round 6: n as int16 in HBM for the hot kernel's row loads and stores (SV_ABLATE=1024: timing only, cold start),
# against the tree -- the potential of an int16 n image kept for the length of a call
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_i16
mkdir -p $O
V=supervillain_amd/variants
for r in 1 2 3; do
  step b$r timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/base_$r.json 2> $O/base_$r.err
  step i$r env SV_LIB_OVERRIDE=$V/libsvhip_i16.so timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-copy-ceiling > $O/i16_$r.json 2> $O/i16_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
