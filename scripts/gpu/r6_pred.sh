# Round 6: rejection prediction on the strong-scaled ranks -- the N = 8 tile through RCCL loopback at the real
# per-sweep rejection rate, prediction off / on
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r6_pred
mkdir -p $O
step pred timeout -k 10 400 python -u scripts/perf/domain_predict_cost.py 3 > $O/pred.log 2>&1
grep interval_n $O/pred.log
