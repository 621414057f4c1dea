"""Fold the --pmc passes of one kernel (scripts/gpu/r3_profile.sh) into profiles/<tag>_pmc_<name>.json.

Usage: summarize_pmc.py OUTDIR TAG NAME KERNEL_SUBSTRING UNITS_PER_LAUNCH ALG_BYTES_PER_UNIT MIN_BYTES_PER_UNIT
  OUTDIR holds one sub-directory per pass (fetch, write, sq1, sq2), each with p_counter_collection.csv.
Per-dispatch averages over full launches only (launches queued behind an aborted sweep exit at entry and are told
apart by duration, < half the median; a cold first launch above twice the median is dropped too).  FETCH_SIZE / WRITE_SIZE are KiB; MI355X_MICROARCH.md: on gfx950 FETCH_SIZE
counts half the bytes of a wide coalesced stream, so both the raw and the x2-corrected read bytes are recorded."""
import collections
import csv
import json
import os
import sys

out, tag, name, kernel = sys.argv[1:5]
units, alg, mn = int(sys.argv[5]), float(sys.argv[6]), float(sys.argv[7])


def counters(d):
    rows = [r for r in csv.DictReader(open(os.path.join(out, d, 'p_counter_collection.csv')))
            if kernel in r['Kernel_Name']]
    dur = {r['Dispatch_Id']: int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows}
    med = sorted(dur.values())[len(dur) // 2]
    keep = {k for k, v in dur.items() if 0.5 * med < v < 2 * med}  # (a cold first launch is not typical either)
    agg = collections.defaultdict(float)
    for r in rows:
        if r['Dispatch_Id'] in keep:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
    avg = {k: v / len(keep) for k, v in agg.items()}
    return avg, sum(dur[k] for k in keep) / len(keep), len(keep), rows[0]['Kernel_Name']


pmc, durations, calls = {}, {}, {}
kname = None
for d in ('fetch', 'write', 'sq1', 'sq2'):
    if not os.path.exists(os.path.join(out, d, 'p_counter_collection.csv')):
        continue
    c, t, n, kname = counters(d)
    pmc.update(c)
    durations[d] = t
    calls[d] = n
fetch = pmc.get('FETCH_SIZE', 0.0) * 1024
write = pmc.get('WRITE_SIZE', 0.0) * 1024
t_ns = durations.get('sq1') or next(iter(durations.values()))
summary = {
    'kernel': kname,
    'units_per_launch': units,
    'pmc_pass_avg_duration_ns': durations,
    'full_launches_per_pass': calls,
    'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch, 'write_bytes': write,
    'hbm_bytes_per_launch': 2 * fetch + write,
    'hbm_bytes_per_unit': (2 * fetch + write) / units,
    'algorithmic_bytes_per_launch': alg * units,
    'fused_min_bytes_per_launch': mn * units,
    'achieved_alg_GBps': alg * units / t_ns,
    'achieved_alg_frac_of_8TBps': alg * units / t_ns / 8000.0,
    'hbm_traffic_GBps': (2 * fetch + write) / t_ns,
    'valu_instructions_per_unit': pmc['SQ_INSTS_VALU'] * 64 / units if 'SQ_INSTS_VALU' in pmc else None,
    'valu_busy_frac': (pmc['SQ_ACTIVE_INST_VALU'] * 4 / (pmc['GRBM_GUI_ACTIVE'] / 8) / 1024)
    if 'SQ_ACTIVE_INST_VALU' in pmc and pmc.get('GRBM_GUI_ACTIVE') else None,
    'wait_any_frac_of_wave_cycles': pmc['SQ_WAIT_ANY'] / pmc['SQ_WAVE_CYCLES'] if 'SQ_WAIT_ANY' in pmc else None,
    'counters_per_dispatch': pmc,
}
os.makedirs('profiles', exist_ok=True)
json.dump(summary, open(f'profiles/{tag}_pmc_{name}.json', 'w'), indent=1)
print(name, json.dumps({k: v for k, v in summary.items() if k != 'counters_per_dispatch'}))
