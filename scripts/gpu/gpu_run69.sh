source scripts/gpu/guard.sh
mkdir -p gpurun_out/r69
SV_DEVICE=0 step two timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/perf/two_rank_same_gpu.py > gpurun_out/r69/two.log 2>&1
grep -i "two-rank\|error\|duplicate" gpurun_out/r69/two.log | head
