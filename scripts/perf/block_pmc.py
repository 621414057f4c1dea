"""Summary of the PMC passes on villain_sweep_block (scripts/gpu/r4_blkpmc.sh): per-dispatch averages, VALU
instructions per owned site-update (K sweeps x N^2 per launch), VALU busy and wait shares, LDS bank-conflict share,
HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md's correction)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
L, K = int(os.environ.get('L', 256)), int(os.environ.get('K', 3))
acc, durs = {}, []
for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        if 'villain_sweep_block' not in r.get('Kernel_Name', ''):
            continue
        name, v = r['Counter_Name'], float(r['Counter_Value'])
        acc.setdefault(name, {}).setdefault(r['Dispatch_Id'], 0.0)
        acc[name][r['Dispatch_Id']] += v
c = {k: sum(v.values()) / max(len(v), 1) for k, v in acc.items()}
units = K * L * L
out = {'kernel': 'villain_sweep_block<8>', 'site_updates_per_launch': units, 'counters_per_dispatch': c}
if 'SQ_INSTS_VALU' in c:
    out['valu_per_site_update'] = c['SQ_INSTS_VALU'] * 64 / units
if 'SQ_ACTIVE_INST_VALU' in c and 'SQ_BUSY_CYCLES' in c and 'SQ_WAVE_CYCLES' in c:
    out['valu_busy_share_of_wave_cycles'] = c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']
    out['wait_share_of_wave_cycles'] = c.get('SQ_WAIT_INST_ANY', 0) / c['SQ_WAVE_CYCLES']
if 'SQ_LDS_BANK_CONFLICT' in c and 'SQ_LDS_IDX_ACTIVE' in c:
    out['lds_bank_conflict_share'] = c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']
if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
    out['hbm_bytes_per_launch'] = (2 * c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024
    out['hbm_bytes_per_site_update'] = out['hbm_bytes_per_launch'] / units
print(json.dumps(out, indent=1))
