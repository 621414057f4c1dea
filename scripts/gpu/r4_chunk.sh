# Round 4, item 2: host pacing of single-lattice batches (SV_CHUNK=4, the round-3 default: chunks of 4 sweeps behind
# the host-mapped progress word) against whole batches enqueued at once (SV_CHUNK=0), in the driver's command form,
# and the cost of a NumPy Lemire rejection in a 20-sweep window (replays now on villain_sweep_hot_skip).
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4_chunk}
mkdir -p $O
for r in 1 2 3; do
  for ch in 4 0; do
    SV_CHUNK=$ch step d${ch}_$r timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/driver_ch${ch}_$r.json 2> $O/driver_ch${ch}_$r.err
  done
done
for ch in 4 0; do
  SV_CHUNK=$ch step rw$ch timeout -k 10 600 python -u scripts/perf/reject_window.py 4096 20 150 > $O/reject_window_ch$ch.log 2>&1
done
for f in $O/driver_*.json; do python -c "import json,sys; d=json.loads(open('$f').readline()); print('$f', round(d['value']/1e9,2), round(d['ms_per_step']*1e3,2), round(d['roofline']['avg_launch_us'],2), d['config'].get('lemire_rejections_in_timed_steps'))"; done
cat $O/reject_window_ch*.log
