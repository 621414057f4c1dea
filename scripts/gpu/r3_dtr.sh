source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3_dtr; mkdir -p $O
for sz in "4096 4096" "4096 2048"; do
  t=$(echo $sz | tr ' ' x)
  step $t env SV_DEBUG_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$t -o run --output-format csv -- python -u scripts/perf/domain_trace.py $sz 256 > $O/$t.log 2>&1
  grep "us/sweep" $O/$t.log
  python scripts/perf/gap_stats.py $O/$t/run_kernel_trace.csv
done
