# Round-3 rocprofv3 evidence: the headline trace + PMC passes (scripts/profile.sh), then PMC passes of the other
# configs' kernels (config 3 worldline_step_fused, config 5 villain_sweep_hot_fr, config 2 villain_sweep_hot at L=256)
# and kernel traces of the reference-order Worldline step and of L=256.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
TAG=r03
step headline timeout -k 10 900 bash scripts/profile.sh $TAG
O=gpurun_out/prof_$TAG
pmc() {  # NAME KERNEL UNITS ALG MIN -- bench args
  local name=$1 kern=$2 units=$3 alg=$4 mn=$5; shift 6
  local P="timeout -s KILL 120 rocprofv3 --kernel-include-regex $kern"
  step ${name}_f $P --pmc FETCH_SIZE -d $O/$name/fetch -o p --output-format csv -- python bench.py "$@" > $O/${name}_f.log 2>&1
  step ${name}_w $P --pmc WRITE_SIZE -d $O/$name/write -o p --output-format csv -- python bench.py "$@" > $O/${name}_w.log 2>&1
  step ${name}_s1 $P --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $O/$name/sq1 -o p --output-format csv -- python bench.py "$@" > $O/${name}_s1.log 2>&1
  step ${name}_s2 $P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES GRBM_GUI_ACTIVE -d $O/$name/sq2 -o p --output-format csv -- python bench.py "$@" > $O/${name}_s2.log 2>&1
  python scripts/summarize_pmc.py $O/$name $TAG $name $kern $units $alg $mn
}
B="--steps 4 --warmup 1 --warmup-s 0 --no-cpu-baseline --no-copy-ceiling"
#pmc worldline worldline_step_fused 1048576 168 168 -- --workload worldline $B
#pmc replicas villain_sweep_hot_fr 16777216 88 48 -- --workload replicas $B
pmc l256 villain_sweep_hot 65536 88 48 -- --L 256 $B
step tr_wlref timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_wlref -o run --output-format csv -- python bench.py --workload worldline --plaquette reference --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_wlref.log 2>&1
cp $O/trace_wlref/run_kernel_stats.csv profiles/${TAG}_kernel_stats_worldline_reference.csv
step tr_l256 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_l256 -o run --output-format csv -- python bench.py --L 256 --steps 2000 --warmup 100 --no-cpu-baseline --no-copy-ceiling > $O/trace_l256.log 2>&1
cp $O/trace_l256/run_kernel_stats.csv profiles/${TAG}_kernel_stats_l256.csv
ls profiles/ | grep $TAG
# the config-4 per-GPU tile (2048 x 1024, one periodic 1x1 domain: the kernel the 8-GPU run uses per rank)
cat > /tmp/tile_run.py <<'PY'
import sys, numpy as np
sys.path.insert(0, '.')
from supervillain_amd.domain import VillainDomain
d = VillainDomain(2048, 1024, (1, 1), kappa=0.5, W=1); d.cold(); g = np.random.default_rng(0); d.run(64, g); d.run(256, g); d.close()
PY
step tr_tile timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_tile -o run --output-format csv -- python /tmp/tile_run.py > $O/trace_tile.log 2>&1
cp $O/trace_tile/run_kernel_stats.csv profiles/${TAG}_kernel_stats_tile2048x1024.csv
