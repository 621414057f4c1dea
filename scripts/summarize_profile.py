"""Fold a scripts/profile.sh run into profiles/<tag>_*.csv|json (committed evidence for bench.py)."""
import collections
import csv
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]
os.makedirs('profiles', exist_ok=True)
shutil.copy(os.path.join(out, 'trace', 'run_kernel_stats.csv'), f'profiles/{tag}_kernel_stats.csv')


def counters(d):
    rows = list(csv.DictReader(open(os.path.join(out, d, 'p_counter_collection.csv'))))
    agg = collections.defaultdict(float)
    disp = set()
    for r in rows:
        agg[r['Counter_Name']] += float(r['Counter_Value'])
        disp.add(r['Dispatch_Id'])
    return {k: v / len(disp) for k, v in agg.items()}, len(disp)


pmc = {}
for d in ('fetch', 'write', 'sq1', 'sq2'):
    c, n = counters(d)
    pmc.update(c)
# rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reads half
# the bytes of a WIDE (16 B/lane) coalesced stream; this kernel's loads are 8 B/lane, for which the
# guide gives no calibration -- both the raw and the x2-corrected read bytes are recorded.
fetch = pmc['FETCH_SIZE'] * 1024
write = pmc['WRITE_SIZE'] * 1024
stats = list(csv.DictReader(open(f'profiles/{tag}_kernel_stats.csv')))
fused = [r for r in stats if 'villain_sweep_fused' in r['Name']][0]
# launches that met a NumPy Lemire rejection make the rest of their batch exit at entry (a few us);
# the full-sweep average excludes those early exits, which is what bench.py's events time
trace = [r for r in csv.DictReader(open(os.path.join(out, 'trace', 'run_kernel_trace.csv')))
         if 'villain_sweep_fused' in r['Kernel_Name']]
dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in trace]
full = [x for x in dur if x > 0.1 * max(dur)]
L = 4096
# the profiled bench run's own JSON line: its live hipEvent average (measured under the tracer) is what the
# trace's full-sweep average must agree with; the tracer slows the kernel itself by ~10% against untraced runs
traced = None
for line in open(os.path.join(out, 'trace.log')):
    if line.startswith('{'):
        traced = json.loads(line)
summary = {
    f'villain_sweep_fused_L{L}': {
        'avg_duration_ns': float(fused['AverageNs']), 'calls': int(fused['Calls']),
        'full_sweep_avg_duration_ns': sum(full) / len(full), 'full_sweep_calls': len(full),
        'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch, 'write_bytes': write,
        'hbm_bytes_per_launch': 2 * fetch + write,
        'hbm_bytes_per_launch_raw': fetch + write,
        'algorithmic_bytes_per_launch': 88 * L * L,          # SURVEY.md 8(d), what bench.py's roofline uses
        'fused_min_bytes_per_launch': 48 * L * L,            # one read + one write of (phi, n) per sweep
        'counters_per_dispatch': pmc,
        'bench_avg_launch_us_same_run': traced['roofline']['avg_launch_us'] if traced else None,
        'bench_ms_per_step_same_run': traced['ms_per_step'] if traced else None,
    }
}
json.dump(summary, open('profiles/pmc_summary.json', 'w'), indent=1)
json.dump(summary, open(f'profiles/{tag}_pmc_summary.json', 'w'), indent=1)
print(json.dumps(summary, indent=1))
