"""Summarize scripts/gpu/r4_ablate.sh: per variant and kernel, the median dispatch duration and the PMC counts per
dispatch (VALU, SALU, LDS instructions; VALU busy and wait shares), and VALU lane-instructions per unit
(site-update for villain_sweep_hot at L=4096, plaquette-step for worldline_step_fused at L=1024)."""
import csv
import glob
import json
import os
import statistics
import sys

out = sys.argv[1]
UNITS = {'vh': 4096 * 4096, 'wf': 1024 * 1024}
res = {}
for d in sorted(glob.glob(os.path.join(out, '*_*'))):
    if not os.path.isdir(d):
        continue
    key = os.path.basename(d)
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        continue
    per = {}
    for r in csv.DictReader(open(files[0])):
        did = r.get('Dispatch_Id')
        per.setdefault(did, {'dur': None, 'kernel': r.get('Kernel_Name')})
        per[did][r['Counter_Name']] = per[did].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
        if r.get('Start_Timestamp') and r.get('End_Timestamp'):
            per[did]['dur'] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    # the most dispatched kernel (not a replay form), full dispatches only: early exits after an abort run a few us
    # and a few hundred thousand instructions
    kern = statistics.mode(p['kernel'] for p in per.values())
    mine = [p for p in per.values() if p['kernel'] == kern and p['dur']]
    top = max(p.get('SQ_INSTS_VALU', 0.0) for p in mine) if mine else 0.0
    full = [p for p in mine if p.get('SQ_INSTS_VALU', 0.0) > 0.5 * top]
    if not full:
        continue
    med = lambda k: statistics.median(p.get(k, 0.0) for p in full)  # noqa: E731
    unit = UNITS[key.split('_')[0]]
    gui = med('GRBM_GUI_ACTIVE')
    res[key] = {'kernel': kern, 'dispatches': len(full), 'dur_us': statistics.median(p['dur'] for p in full) / 1e3,
                'valu_per_unit': med('SQ_INSTS_VALU') * 64 / unit, 'salu_per_unit': med('SQ_INSTS_SALU') * 64 / unit,
                'lds_per_unit': med('SQ_INSTS_LDS') * 64 / unit,
                'valu_busy': med('SQ_ACTIVE_INST_VALU') * 4 / (gui / 8) / 1024 if gui else None,
                'wait_share': med('SQ_WAIT_INST_ANY') / med('SQ_WAVE_CYCLES') if med('SQ_WAVE_CYCLES') else None}
for k, v in res.items():
    print(k, json.dumps({a: (round(b, 3) if isinstance(b, float) else b) for a, b in v.items()}))
json.dump(res, open(os.path.join(out, 'summary.json'), 'w'), indent=1)
