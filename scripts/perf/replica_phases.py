"""Where the config-5 whole-job time goes: Python around VillainReplicas.run vs the C++ batch loop."""
import os, sys, time
import numpy as np
sys.path.insert(0, '.')
os.environ['SV_DEBUG_TIMING'] = '1'
from supervillain_amd.replicas import VillainReplicas
import supervillain_amd._abi as abi
R, N = 1024, 128
B = VillainReplicas(R, N, 0.5, 2)
B.cold()
gens = [np.random.default_rng(r) for r in range(R)]
B.run(20, gens, inline=True)
for rep in range(2):
    t0 = time.perf_counter()
    stats, obs = B.run(200, gens, inline=True)
    t1 = time.perf_counter()
    print(f'run(200): {(t1 - t0) * 1e3:.1f} ms', flush=True)
t0 = time.perf_counter(); r, a = abi.rngs_from_numpy(gens); abi.rngs_to_numpy(r, gens, a); print('rng conv', (time.perf_counter() - t0) * 1e3, 'ms')
