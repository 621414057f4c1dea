# End-of-round evidence: headline trace + PMC passes (scripts/profile.sh), PMC passes of the config 2 / 3 / 5 kernels,
# traces of the reference-order Worldline step, L=256 and the N=8 tile, and the bench lines.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
TAG=r03
O=gpurun_out/prof_$TAG
step headline timeout -k 10 900 bash scripts/profile.sh $TAG
pmc() {  # NAME KERNEL -- bench args
  local name=$1 kern=$2; shift 3
  local P="timeout -s KILL 120 rocprofv3 --kernel-include-regex $kern"
  step ${name}_f $P --pmc FETCH_SIZE -d $O/$name/fetch -o p --output-format csv -- python bench.py "$@" > $O/${name}_f.log 2>&1
  step ${name}_w $P --pmc WRITE_SIZE -d $O/$name/write -o p --output-format csv -- python bench.py "$@" > $O/${name}_w.log 2>&1
  step ${name}_s1 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $O/$name/sq1 -o p --output-format csv -- python bench.py "$@" > $O/${name}_s1.log 2>&1
  step ${name}_s2 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES GRBM_GUI_ACTIVE -d $O/$name/sq2 -o p --output-format csv -- python bench.py "$@" > $O/${name}_s2.log 2>&1
}
B="--steps 4 --warmup 1 --warmup-s 0 --no-cpu-baseline --no-copy-ceiling"
pmc worldline worldline_step_fused -- --workload worldline $B
pmc replicas villain_sweep_hot_fr -- --workload replicas $B
pmc l256 villain_sweep_hot -- --L 256 $B
step tr_wlref timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_wlref -o run --output-format csv -- python bench.py --workload worldline --plaquette reference --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_wlref.log 2>&1
step tr_l256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_l256 -o run --output-format csv -- python bench.py --L 256 --steps 2000 --warmup 100 --no-cpu-baseline --no-copy-ceiling > $O/trace_l256.log 2>&1
step tr_tile timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_tile -o run --output-format csv -- python -u scripts/perf/domain_trace.py 2048 1024 256 > $O/trace_tile.log 2>&1
# bench lines (no tracer)
mkdir -p $O/bench
for r in 1 2 3; do
  step d$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench/driver_$r.json 2> $O/bench/driver_$r.err
done
step def timeout -k 10 300 python -u bench.py > $O/bench/default.json 2> $O/bench/default.err
step wl timeout -k 10 300 python -u bench.py --workload worldline > $O/bench/worldline.json 2> $O/bench/worldline.err
step wlref timeout -k 10 300 python -u bench.py --workload worldline --plaquette reference --steps 20 --warmup 2 > $O/bench/worldline_reference.json 2> $O/bench/worldline_reference.err
step l256 timeout -k 10 300 python -u bench.py --L 256 > $O/bench/l256.json 2> $O/bench/l256.err
step rep timeout -k 10 300 python -u bench.py --workload replicas > $O/bench/replicas.json 2> $O/bench/replicas.err
step t8 timeout -k 10 300 python -u bench.py --tiles 2x4 --steps 40 --warmup 5 --no-cpu-baseline > $O/bench/tiles2x4.json 2> $O/bench/tiles2x4.err
for f in $O/bench/*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), round(d['roofline']['frac'],3), d['config'].get('lemire_rejections_in_timed_steps'))"; done
