# Round 6: config 3's step time by where the exact acceptance words live (SV_WFFX variants) against round 5's kernels
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_wfab
mkdir -p $O
V=supervillain_amd/variants
for r in 1 2 3; do
  step n$r timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_new_$r.json 2> $O/wl_new_$r.err
  step b$r env SV_LIB_OVERRIDE=$V/libsvhip_r5base.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_base_$r.json 2> $O/wl_base_$r.err
  step f1$r env SV_LIB_OVERRIDE=$V/libsvhip_wffx1.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_fx1_$r.json 2> $O/wl_fx1_$r.err
  step f2$r env SV_LIB_OVERRIDE=$V/libsvhip_wffx2.so timeout -k 10 200 python -u bench.py --workload worldline --no-cpu-baseline --no-copy-ceiling > $O/wl_fx2_$r.json 2> $O/wl_fx2_$r.err
done
for f in $O/*.json; do python scripts/summ_line.py $f; done
