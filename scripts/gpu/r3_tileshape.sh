# Tile shape and wave count for the config-4 per-GPU tile: 2048x1024 vs 1024x2048, 4- vs 8-wave workgroups.
source scripts/gpu/guard.sh
O=gpurun_out/r3_tileshape; mkdir -p $O
for sz in 2048x1024 1024x2048; do
  step a$sz env SV_SIZES=$sz timeout -k 10 200 python -u scripts/perf/tile_th.py "" 24 32 36 > $O/a$sz.log 2>&1
  step b$sz env SV_SIZES=$sz SV_HOT_NW=8 timeout -k 10 200 python -u scripts/perf/tile_th.py 64 72 80 > $O/b$sz.log 2>&1
done
cat $O/*.log
