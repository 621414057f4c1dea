# summarize bench logs and kernel stats of a gpurun_out/rNN directory
d=$1
for f in $d/*.log; do python3 -c "
import json,sys
ls=[l for l in open('$f') if l.startswith('{')]
if ls:
    d=json.loads(ls[-1]); print('%-12s %10.3g %8.3f ms %9.1f us frac %.3f acc %.4f' % ('$(basename $f .log)', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['config']['acceptance_rate']))"; done
for f in $(find $d -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print('%-70s %5s %10.1f us avg %6.2f%%' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, float(r['Percentage'])))"; done
