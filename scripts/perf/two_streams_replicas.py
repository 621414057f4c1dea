"""Tail-recovery potential for config 5: the 1024 replicas (L=128, W=2, inline observables) as one batch on one stream,
against two batches of 512 on two contexts (streams) driven from two host threads.  If the pair's replica-sweeps per
second beat the one batch, the batch launches' tails are what the difference costs."""
import sys
import threading
import time

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd.replicas import VillainReplicas  # noqa: E402

L, R = 128, 1024
sweeps = int(sys.argv[1]) if len(sys.argv) > 1 else 200


def batch(r, seed, ctx):
    saved = _native.context
    _native.context = lambda device=None: ctx  # bind this batch to its own context (stream)
    try:
        b = VillainReplicas(r, L, 0.5, 2)
    finally:
        _native.context = saved
    gens = [np.random.default_rng(seed + i) for i in range(r)]
    return b, gens


one, g1 = batch(R, 0, _native.Context(0))
ha, ga = batch(R // 2, 10_000, _native.Context(0))
hb, gb = batch(R // 2, 20_000, _native.Context(0))
one.run(10, g1, inline=True)
ha.run(10, ga, inline=True)
hb.run(10, gb, inline=True)
for rep in range(3):
    t0 = time.perf_counter()
    one.run(sweeps, g1, inline=True)
    t1 = time.perf_counter()
    ths = [threading.Thread(target=b.run, args=(sweeps, g), kwargs={'inline': True}) for b, g in ((ha, ga), (hb, gb))]
    t2 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t3 = time.perf_counter()
    print(f'{R} x L={L}: one batch {(t1 - t0) / sweeps * 1e6:.1f} us per sweep ({R * L * L * sweeps / (t1 - t0) / 1e9:.2f} G); '
          f'two half-batches on two streams {(t3 - t2) / sweeps * 1e6:.1f} us per sweep '
          f'({R * L * L * sweeps / (t3 - t2) / 1e9:.2f} G)', flush=True)
