# Round 4: PC sampling (rocprofv3 beta) of the two hot kernels -- where their issue slots go, by instruction.
set -u
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_pcs}
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d $O/vh_st -o p --output-format csv -- python bench.py --steps 40 --warmup 2 --no-cpu-baseline > $O/vh_st.log 2>&1
echo "stochastic rc=$?"; ls -R $O/vh_st 2>/dev/null | head; tail -5 $O/vh_st.log
if ! ls $O/vh_st/*/*pc_sampling* > /dev/null 2>&1 && ! ls $O/vh_st/*pc_sampling* > /dev/null 2>&1; then
  timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 10 -d $O/vh_ht -o p --output-format csv -- python bench.py --steps 40 --warmup 2 --no-cpu-baseline > $O/vh_ht.log 2>&1
  echo "host_trap rc=$?"; ls -R $O/vh_ht 2>/dev/null | head; tail -5 $O/vh_ht.log
fi
