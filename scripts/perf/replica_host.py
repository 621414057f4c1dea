"""Where a config-5 call's wall time goes outside the sweep kernels: VillainReplicas.run's phases timed one by one
(generator states in, result arrays allocated, the library call -- kernels, planning, copies -- and the Python
post-processing), against the kernel time the context's events record.  Usage: python scripts/perf/replica_host.py"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rngs_from_numpy, rngs_to_numpy  # noqa: E402
from supervillain_amd.replicas import STATS_DTYPE, VillainReplicas  # noqa: E402

R, L, sweeps = 1024, 128, 200
B = VillainReplicas(R, L, 0.5, 2)
B.cold()
gens = [np.random.default_rng(r) for r in range(R)]
Lib = _native.lib()
B.run(20, gens, inline=True)
for rep in range(4):
    Lib.sv_ctx_set_timing(B.ctx.handle, 1)
    t0 = time.perf_counter()
    r, addrs = rngs_from_numpy(gens)
    t1 = time.perf_counter()
    st = np.zeros((R, sweeps), dtype=STATS_DTYPE)
    obs = np.zeros((R, sweeps, 4))
    t2 = time.perf_counter()
    B.ctx.check(Lib.sv_replicas_run(B.handle, B.kappa, B.W, B.interval_phi, B.interval_n, sweeps, r, _native.ptr(st),
                                    _native.ptr(obs)), 'run')
    t3 = time.perf_counter()
    rngs_to_numpy(r, gens, addrs)
    V = L * L
    stats = {'accepted': st['accepted'], 'acceptance': st['acceptance_sum'] / V, 'rejections': st['rejections']}
    S = obs[..., 0] * (B.kappa / 2)
    action = S / V
    np.divide(S, V * B.kappa, out=S)
    w2 = obs[..., 1] / V
    tw = obs[..., 2:4].astype(np.int64)
    t4 = time.perf_counter()
    ms = lambda a, b: (b - a) * 1e3
    print(f'rep {rep}: rng in {ms(t0, t1):.2f} ms, alloc {ms(t1, t2):.2f}, call {ms(t2, t3):.2f}, post {ms(t3, t4):.2f}, '
          f'total {ms(t0, t4):.2f} ms = {ms(t0, t4) * 1e3 / sweeps:.1f} us/sweep')
    t5 = time.perf_counter()
    B.run(sweeps, gens, inline=True)
    t6 = time.perf_counter()
    print(f'       VillainReplicas.run: {ms(t5, t6):.2f} ms = {ms(t5, t6) * 1e3 / sweeps:.1f} us/sweep')
B.close()
