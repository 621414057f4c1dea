"""The device timeline of the last sv_villain_run call of a bench run (rocprofv3 --kernel-trace --memory-copy-trace
CSVs): every kernel and copy of the call in order with its duration and the idle gap before it, and the totals --
where a call's wall time goes besides the sweep kernels."""
import csv
import glob
import os
import sys

d = sys.argv[1]
KEY = sys.argv[2] if len(sys.argv) > 2 else 'villain_sweep'  # the sweep kernels' name fragment
MINK = int(sys.argv[3]) if len(sys.argv) > 3 else 20       # a timed call has at least this many of them
ev = []
for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60]))
for f in glob.glob(os.path.join(d, '**', '*memory_copy_trace.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'copy ' + r.get('Direction', '?')))
ev.sort()
# calls: runs of events separated by > 200 us of idle; the timed call is the last one with >= 20 sweep kernels
calls, cur = [], []
for e in ev:
    if cur and e[0] - cur[-1][1] > 200_000:
        calls.append(cur)
        cur = []
    cur.append(e)
if cur:
    calls.append(cur)
hot = [c for c in calls if sum(KEY in x[2] for x in c) >= MINK]
c = hot[-1] if hot else calls[-1]
t0 = c[0][0]
busy = sum(e[1] - e[0] for e in c)
sweep = sum(e[1] - e[0] for e in c if KEY in e[2])
print(f'call: {len(c)} events, span {(c[-1][1] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, sweep kernels {sweep / 1e3:.1f} us '
      f'({sum(KEY in x[2] for x in c)} launches), idle {(c[-1][1] - t0 - busy) / 1e3:.1f} us')
prev = t0
for s, e, n in c:
    if 'villain_sweep' not in n or s - prev > 3000:
        print(f'  +{(s - t0) / 1e3:8.1f} us  gap {(s - prev) / 1e3:6.1f}  dur {(e - s) / 1e3:7.1f}  {n}')
    prev = e
print(f'between calls: ' + ', '.join(f'{(calls[i + 1][0][0] - calls[i][-1][1]) / 1e3:.0f} us' for i in range(max(0, len(calls) - 4), len(calls) - 1)))
