"""Measurement only: Ensemble-style emission of kept configurations at L=4096 -- the asynchronous emission path
(device snapshot + copy stream into page-locked storage) against a synchronous download per configuration.
   python scripts/perf/emit_overlap.py [--L 4096] [--keep 32] [--steps 8]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import supervillain_amd as sv  # noqa: E402
from supervillain_amd.generator import villain as gv  # noqa: E402
from supervillain_amd.generator.combining import KeepEvery  # noqa: E402
from supervillain_amd.pipeline import DeviceChain, device_program, pinned_empty  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--L', type=int, default=4096)
ap.add_argument('--keep', type=int, default=32)
ap.add_argument('--steps', type=int, default=8)
a = ap.parse_args()
S = sv.Villain(sv.Lattice2D(a.L), 0.5, 1)
t = time.perf_counter()
phi = pinned_empty((a.steps, 1, a.L, a.L), np.float64)
n = pinned_empty((a.steps, 2, a.L, a.L), np.int64)
t_pin = time.perf_counter() - t
res = {'L': a.L, 'keep_every': a.keep, 'configs': a.steps, 'pin_s': t_pin}
for mode in ('advance_only', 'download', 'emit', 'advance_only'):
    G = gv.NeighborhoodUpdate(S)
    G.rng = np.random.default_rng(0)
    ch = DeviceChain(S, device_program(KeepEvery(a.keep, G)))
    ch.upload(S.configurations(1)[0])
    ch.advance()  # warm: tables, buffers
    t = time.perf_counter()
    for i in range(a.steps):
        ch.advance()
        if mode == 'download':
            d = ch.download()
            phi[i], n[i] = d['phi'], d['n']
        elif mode == 'emit':
            ch.emit(phi[i], n[i])
    if mode == 'emit':
        ch.emit_wait()
    res[mode + '_ms_per_config'] = (time.perf_counter() - t) / a.steps * 1e3
    ch.close()
res['bytes_per_config'] = int(phi[0].nbytes + n[0].nbytes)
print(json.dumps(res))
