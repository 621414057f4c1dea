"""Gaps between consecutive launches of one kernel in a rocprofv3 kernel trace: count, mean, p90, and the spacing
(in launches) of the gaps above 3 us.  Usage: gap_stats.py run_kernel_trace.csv [kernel substring]"""
import collections
import csv
import statistics
import sys

KERNEL = sys.argv[2] if len(sys.argv) > 2 else 'villain_sweep_hot'
tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
hot = [i for i, r in enumerate(tr) if KERNEL in r['Kernel_Name']]
gaps, big = [], []
for j, i in enumerate(hot[:-1]):
    if hot[j + 1] == i + 1:
        g = int(tr[i + 1]['Start_Timestamp']) - int(tr[i]['End_Timestamp'])
        if g < 1e6:
            gaps.append(g)
            if g > 3000:
                big.append(j)
sp = collections.Counter(big[k + 1] - big[k] for k in range(len(big) - 1))
dur = [int(tr[i]['End_Timestamp']) - int(tr[i]['Start_Timestamp']) for i in hot]
full = [d for d in dur if d > 0.5 * statistics.median(dur)]
print(f'{sys.argv[1]}: {len(gaps)} gaps, mean {statistics.mean(gaps) / 1e3:.2f} us, p90 {sorted(gaps)[int(0.9 * len(gaps))] / 1e3:.2f} us; '
      f'large gaps every {sp.most_common(3)} launches; full sweeps {len(full)} x {statistics.mean(full) / 1e3:.1f} us, '
      f'drains {len(dur) - len(full)}', flush=True)
