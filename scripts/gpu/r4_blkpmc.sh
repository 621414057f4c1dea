# PMC passes on villain_sweep_block (config 2, L=256): instructions, busy / wait shares, LDS, HBM bytes
source scripts/gpu/guard.sh
O=gpurun_out/r4_blkpmc
mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --L 256 --steps 60 --warmup 3 --no-cpu-baseline"
step sq1 timeout -s KILL 120 rocprofv3 --kernel-include-regex villain_sweep_block --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/sq1 -o p --output-format csv -- $B > $O/sq1.log 2>&1
step sq2 timeout -s KILL 120 rocprofv3 --kernel-include-regex villain_sweep_block --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/sq2 -o p --output-format csv -- $B > $O/sq2.log 2>&1
step fetch timeout -s KILL 120 rocprofv3 --kernel-include-regex villain_sweep_block --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- $B > $O/fetch.log 2>&1
step write timeout -s KILL 120 rocprofv3 --kernel-include-regex villain_sweep_block --pmc WRITE_SIZE -d $O/write -o p --output-format csv -- $B > $O/write.log 2>&1
python scripts/perf/block_pmc.py $O > $O/summary.json; cat $O/summary.json
