source scripts/gpu/guard.sh
mkdir -p gpurun_out/r21
export TMPDIR=/tmp
step tests timeout -k 10 900 python -m pytest tests -m gpu -x -q -o log_cli=false --junitxml=gpurun_out/r21/junit.xml > gpurun_out/r21/tests.log 2>&1
tail -5 gpurun_out/r21/tests.log
step bench1 bash -c 'timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/r21/bench1.log 2>&1'
tail -2 gpurun_out/r21/bench1.log
step torchfirst bash -c 'timeout -k 10 200 python scripts/check_torch_first.py > gpurun_out/r21/torchfirst.log 2>&1'
tail -3 gpurun_out/r21/torchfirst.log
step tiles12 bash -c 'timeout -k 10 300 python bench.py --tiles 1x2 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r21/bench_tiles12.log 2>&1'
tail -2 gpurun_out/r21/bench_tiles12.log
step probe2 bash -c 'SV_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 2 --L 1024 > gpurun_out/r21/probe2.log 2>&1'
tail -30 gpurun_out/r21/probe2.log
