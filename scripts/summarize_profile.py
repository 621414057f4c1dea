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
    """Per-dispatch averages of one --pmc pass over FULL sweeps only: launches queued behind a rejected sweep
    exit at entry (a few us, ~0 bytes) and would dilute the averages; they are told apart by duration."""
    rows = list(csv.DictReader(open(os.path.join(out, d, 'p_counter_collection.csv'))))
    dur = {r['Dispatch_Id']: int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows}
    longest = max(dur.values())
    keep = {k for k, v in dur.items() if v > 0.5 * longest}
    agg = collections.defaultdict(float)
    for r in rows:
        if r['Dispatch_Id'] in keep:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
    avg = {k: v / len(keep) for k, v in agg.items()}
    avg['_duration_ns'] = sum(dur[k] for k in keep) / len(keep)
    return avg, len(keep)


pmc = {}
pass_durations = {}
for d in ('fetch', 'write', 'sq1', 'sq2'):
    c, n = counters(d)
    pass_durations[d] = c.pop('_duration_ns')
    pmc.update(c)
# rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reads half
# the bytes of a WIDE (16 B/lane) coalesced stream; this kernel's loads are 8 B/lane, for which the
# guide gives no calibration -- both the raw and the x2-corrected read bytes are recorded.
fetch = pmc['FETCH_SIZE'] * 1024
write = pmc['WRITE_SIZE'] * 1024
stats = list(csv.DictReader(open(f'profiles/{tag}_kernel_stats.csv')))
# the headline sweep kernel (villain_sweep_hot since round 2; villain_sweep_fused runs the sweeps the hot kernel
# does not cover: a NumPy Lemire rejection known in the sweep's choice blocks)
KERNEL = 'villain_sweep_hot' if any('villain_sweep_hot' in r['Name'] for r in stats) else 'villain_sweep_fused'
fused = [r for r in stats if KERNEL in r['Name']][0]
# launches that met a NumPy Lemire rejection make the rest of their batch exit at entry (a few us);
# the full-sweep average excludes those early exits, which is what bench.py's events time
trace = [r for r in csv.DictReader(open(os.path.join(out, 'trace', 'run_kernel_trace.csv')))
         if KERNEL in r['Kernel_Name']]
dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in trace]
# launches queued behind a rejected sweep exit at entry ("drains", a few us each); they are counted and
# reported, and kept out of the full-sweep average (which is what bench.py's hipEvents time)
full = [x for x in dur if x > 0.1 * max(dur)]
drains = [x for x in dur if x <= 0.1 * max(dur)]
L = 4096
# the profiled bench run's own JSON line: its live hipEvent average (measured under the tracer) is what the
# trace's full-sweep average must agree with; the tracer slows the kernel itself by ~10% against untraced runs
traced = None
for line in open(os.path.join(out, 'trace.log')):
    if line.startswith('{'):
        traced = json.loads(line)
summary = {
    f'{KERNEL}_L{L}': {
        'kernel': KERNEL,
        'early_exit_drains': len(drains), 'early_exit_avg_ns': (sum(drains) / len(drains)) if drains else None,
        'avg_duration_ns': float(fused['AverageNs']), 'calls': int(fused['Calls']),
        'full_sweep_avg_duration_ns': sum(full) / len(full), 'full_sweep_calls': len(full),
        'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch, 'write_bytes': write,
        'hbm_bytes_per_launch': 2 * fetch + write,
        'hbm_bytes_per_launch_raw': fetch + write,
        'algorithmic_bytes_per_launch': 88 * L * L,          # SURVEY.md 8(d), what bench.py's roofline uses
        'fused_min_bytes_per_launch': 48 * L * L,            # one read + one write of (phi, n) per sweep
        'counters_per_dispatch': pmc,
        'pmc_pass_full_sweep_avg_ns': pass_durations,
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles (MI355X_MICROARCH.md, DVFS give-back)
        'effective_clock_GHz': (pmc['GRBM_GUI_ACTIVE'] / 8 / pass_durations['sq2']) if 'GRBM_GUI_ACTIVE' in pmc else None,
        'valu_instructions_per_site_update': pmc['SQ_INSTS_VALU'] * 64 / (L * L),
        'bench_avg_launch_us_same_run': traced['roofline']['avg_launch_us'] if traced else None,
        'bench_ms_per_step_same_run': traced['ms_per_step'] if traced else None,
    }
}
json.dump(summary, open('profiles/pmc_summary.json', 'w'), indent=1)
json.dump(summary, open(f'profiles/{tag}_pmc_summary.json', 'w'), indent=1)
print(json.dumps(summary, indent=1))
