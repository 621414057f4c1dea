"""Where a NumPy Lemire rejection's cost goes, from a rocprofv3 kernel trace of scripts/perf/reject_window.py:
for every split replay launch (villain_sweep_hot_split) or general-kernel replay (villain_sweep_fused), the failing
hot sweep before it, the early-exit drains behind it, the idle GPU time between the last drain and the replay's first
kernel (the host's round trip), the replay itself and the hot sweep's median for comparison.
Usage: reject_trace.py run_kernel_trace.csv"""
import csv
import statistics
import sys

tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
ev = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in tr]
dur = lambda e: (e[2] - e[1]) / 1e3  # noqa: E731
hot = [dur(e) for e in ev if 'villain_sweep_hot<' in e[0] or 'villain_sweep_hotILb' in e[0]]
full = statistics.median([d for d in hot if d > 50]) if hot else 0.0
rows = []
for i, e in enumerate(ev):
    if not ('hot_split' in e[0] or 'villain_sweep_fused' in e[0]):
        continue
    # walk back: kernels between the previous full hot sweep and this replay
    j = i - 1
    drains, other = [], []
    while j >= 0 and not (('villain_sweep_hot' in ev[j][0]) and dur(ev[j]) > 50):
        (drains if 'villain_sweep_hot' in ev[j][0] else other).append(ev[j])
        j -= 1
    if j < 0:
        continue
    fail = ev[j]
    last_before = max((x[2] for x in ev[j:i]), default=fail[2])
    first_after = min(x[1] for x in ev[j + 1:i + 1] if x[1] >= last_before) if i > j else e[1]
    gap = (e[1] - last_before) / 1e3
    rows.append(dict(fail=dur(fail), drains=len(drains), drain_us=sum(dur(d) for d in drains),
                     other=[x[0][:30] for x in other], gap=gap, replay=dur(e), kind='split' if 'split' in e[0] else 'fused'))
print(f'hot sweep median {full:.1f} us; {len(rows)} replays')
for r in rows:
    print(f"  fail {r['fail']:6.1f}  drains {r['drains']:2d} ({r['drain_us']:6.1f} us)  idle before replay {r['gap']:6.1f}  "
          f"{r['kind']} {r['replay']:6.1f} us  other: {','.join(sorted(set(r['other'])))}")
if rows:
    m = lambda k: statistics.mean(r[k] for r in rows)  # noqa: E731
    print(f"mean: fail {m('fail'):.1f} us, drains {m('drains'):.1f} ({m('drain_us'):.1f} us), idle {m('gap'):.1f} us, "
          f"replay {m('replay'):.1f} us (hot {full:.1f})")
