# A/B: the domain tile's hot sweeps with write-through row stores (variants/libsvhip_tilesc1.so) vs plain stores:
# the 2048 x 1024 depth-4 tile alone and through RCCL loopback (deep_halo.py), the 2 x 4 emulation bench line
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tilesc1}
mkdir -p $O
V=supervillain_amd/variants/libsvhip_tilesc1.so
step t env SV_LIB_OVERRIDE=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_domain.py > $O/tests.log 2>&1
for r in 1 2; do
  step b$r env SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_base_$r.log 2>&1
  step s$r env SV_LIB_OVERRIDE=$V SV_SIZES=2048x1024 timeout -k 10 200 python -u scripts/perf/deep_halo.py 4 > $O/tile_sc1_$r.log 2>&1
  echo "base $r: $(tr '\n' ' ' < $O/tile_base_$r.log)"
  echo "sc1 $r: $(tr '\n' ' ' < $O/tile_sc1_$r.log)"
done
for r in 1 2; do
  step eb$r timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/t8_base_$r.json 2> $O/t8_base_$r.err
  step es$r env SV_LIB_OVERRIDE=$V timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/t8_sc1_$r.json 2> $O/t8_sc1_$r.err
done
for f in $O/t8_*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us/sweep')"; done
# config 2 (L=256): villain_sweep_block with write-through stores (variants/libsvhip_blksc1.so) vs plain
B=supervillain_amd/variants/libsvhip_blksc1.so
step bt env SV_LIB_OVERRIDE=$B timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_block.py > $O/tests_blk.log 2>&1
for r in 1 2 3; do
  step lb$r timeout -k 10 200 python -u bench.py --L 256 --steps 2000 --warmup 200 --no-cpu-baseline > $O/l256_base_$r.json 2> $O/l256_base_$r.err
  step ls$r env SV_LIB_OVERRIDE=$B timeout -k 10 200 python -u bench.py --L 256 --steps 2000 --warmup 200 --no-cpu-baseline > $O/l256_sc1_$r.json 2> $O/l256_sc1_$r.err
done
for f in $O/l256_*.json; do python -c "import json; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel')"; done
