"""Kernel timeline around each replay of a rejected config-2 sweep (rocprofv3 kernel trace of
scripts/perf/reject_cost_small.py): the launches before and after every villain_sweep_fused / _hot_split launch (the
failing sweep's replay), with their start times relative to the replay, durations and the idle gaps between them.
Usage: reject_trace_small.py run_kernel_trace.csv [before=10] [after=4]"""
import csv
import sys

tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
before = int(sys.argv[2]) if len(sys.argv) > 2 else 10
after = int(sys.argv[3]) if len(sys.argv) > 3 else 4
ev = [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in tr]
short = lambda n: n.replace('void ', '').replace('sv::', '').split('(')[0][:34]  # noqa: E731
for i, e in enumerate(ev):
    if not ('villain_sweep_fused' in e[0] or 'hot_split' in e[0]):
        continue
    print(f'--- replay at trace index {i}')
    prev_end = None
    for j in range(max(0, i - before), min(len(ev), i + after + 1)):
        n, s, t = ev[j]
        gap = '' if prev_end is None else f'gap {(s - prev_end) / 1e3:7.1f}'
        print(f'  {(s - e[1]) / 1e3:9.1f} us  {short(n):34s} {(t - s) / 1e3:7.1f} us  {gap}')
        prev_end = t
