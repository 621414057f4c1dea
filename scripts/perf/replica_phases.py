"""Where the config-5 whole-job time goes: Python around VillainReplicas.run vs the C++ batch loop.
  SV_DEBUG_TIMING=1 python scripts/perf/replica_phases.py [sweeps]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd.replicas import VillainReplicas, STATS_DTYPE  # noqa: E402
import supervillain_amd._abi as abi  # noqa: E402

R, N = 1024, 128
sweeps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B = VillainReplicas(R, N, 0.5, 2)
B.cold()
gens = [np.random.default_rng(r) for r in range(R)]
B.run(20, gens, inline=True)
for rep in range(2):
    t0 = time.perf_counter()
    stats, obs = B.run(sweeps, gens, inline=True)
    t1 = time.perf_counter()
    print(f'run({sweeps}): {(t1 - t0) * 1e3:.1f} ms = {(t1 - t0) / sweeps * 1e6:.1f} us/sweep', flush=True)
# the same call taken apart
T = {}
t = time.perf_counter()
r, a = abi.rngs_from_numpy(gens)
T['rng in'] = time.perf_counter() - t
t = time.perf_counter()
st = np.zeros((R, sweeps), dtype=STATS_DTYPE)
ob = np.zeros((R, sweeps, 4))
T['alloc'] = time.perf_counter() - t
t = time.perf_counter()
B.ctx.check(_native.lib().sv_replicas_run(B.handle, B.kappa, B.W, B.interval_phi, B.interval_n, sweeps, r,
                                          _native.ptr(st), _native.ptr(ob)), 'run')
T['C call'] = time.perf_counter() - t
t = time.perf_counter()
abi.rngs_to_numpy(r, gens, a)
T['rng out'] = time.perf_counter() - t
t = time.perf_counter()
V = N * N
x = {'accepted': st['accepted'].copy(), 'acceptance': st['acceptance_sum'] / V, 'rejections': st['rejections'].copy()}
S = B.kappa / 2 * ob[..., 0]
y = {'ActionDensity': S / V, 'InternalEnergyDensity': S / (V * B.kappa), 'WindingSquared': ob[..., 1] / V,
     'TorusWrapping': ob[..., 2:4].astype(np.int64)}
T['post'] = time.perf_counter() - t
print({k: round(v * 1e3, 2) for k, v in T.items()}, 'ms', flush=True)
B.close()
