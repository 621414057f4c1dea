"""GPU idle time in a rocprofv3 kernel trace: the union of all kernels' busy intervals over the span from the first
to the last launch of KERNEL, the idle fraction, and the largest idle gaps with the kernels either side.
Usage: idle_gaps.py run_kernel_trace.csv KERNEL [top]"""
import csv
import sys

KERNEL = sys.argv[2]
TOP = int(sys.argv[3]) if len(sys.argv) > 3 else 12
tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(tr) if KERNEL in r['Kernel_Name']]
# the last 60% of the KERNEL launches (skips warmup and setup)
first = idx[int(0.4 * len(idx))]
last = idx[-1]
ev = tr[first:last + 1]
busy_end = int(ev[0]['Start_Timestamp'])
idle, gaps = 0, []
for i, r in enumerate(ev):
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if s > busy_end:
        g = s - busy_end
        idle += g
        gaps.append((g, ev[i - 1]['Kernel_Name'][:60] if i else '', r['Kernel_Name'][:60]))
    busy_end = max(busy_end, e)
span = busy_end - int(ev[0]['Start_Timestamp'])
n = sum(1 for r in ev if KERNEL in r['Kernel_Name'])
print(f'{n} {KERNEL} launches over {span / 1e6:.2f} ms: idle {idle / 1e6:.3f} ms ({100 * idle / span:.1f}%), '
      f'{len(gaps)} gaps, {sum(1 for g in gaps if g[0] > 20000)} over 20 us')
for g, a, b in sorted(gaps, reverse=True)[:TOP]:
    print(f'  {g / 1e3:9.1f} us  after {a}  before {b}')
