# A/B timing of library variants: bash scripts/gpu/job_ab.sh TAG "v0 v1 ..." [bench args]
source scripts/gpu/guard.sh
T=$1; VARS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
for v in $VARS; do
  SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_$v.so step b$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-copy-ceiling ${ABARGS:---steps 300 --warmup 20} "$@" > $O/b_${v}_$rep.log 2>&1
  grep '^{' $O/b_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $rep, round(d['value']/1e9,2), round(d['roofline']['avg_launch_us'],1), d['ms_per_step'])"
done
done
