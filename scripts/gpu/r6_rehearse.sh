# Round 6: the driver's N > 1 bench runs rehearsed with N real ranks on the one GPU (SV_DEVICE=0): bench.py --gpus N
# launches its own torch.distributed.run, halos over the hosted transport (RCCL refuses several ranks on one device).
# Not measurements: N processes share one GPU.  Config 4 at N = 2, 4, 8 and config 3 at N = 8.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
export SV_DEVICE=0
O=gpurun_out/r6_rehearse
mkdir -p $O
for n in 2 4 8; do
  step v$n timeout -k 10 300 python -u bench.py --gpus $n --transport host --steps 20 --warmup 2 --warmup-s 0.2 --no-cpu-baseline --no-copy-ceiling > $O/villain_n$n.json 2> $O/villain_n$n.err
done
step w8 timeout -k 10 300 python -u bench.py --gpus 8 --transport host --workload worldline --steps 20 --warmup 2 --warmup-s 0.2 --no-cpu-baseline --no-copy-ceiling > $O/worldline_n8.json 2> $O/worldline_n8.err
for f in $O/*.json; do python scripts/summ_line.py $f; done
