"""One line per bench JSON: value, wall and kernel time per step, E_N, rejections, metric (GPU-run summaries)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).readline())
    except Exception as e:  # (a run that printed nothing)
        print(path, 'no line:', e)
        continue
    s = d['config'].get('scaling_reference', {})
    print(path, f"{d['value'] / 1e9:.3f} G", f"{d['ms_per_step'] * 1e3:.2f} us wall",
          f"{d['roofline']['avg_launch_us']:.2f} us kernel", 'E_N', s.get('E_N'), 'E_single',
          s.get('E_N_vs_single_lattice'), 'R1', s.get('R1'), 'single', s.get('single_lattice_rate'), 'rej',
          d['config'].get('lemire_rejections_in_timed_steps'), '|', d['metric'])
