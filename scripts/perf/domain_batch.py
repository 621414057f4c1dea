"""Batch size vs rejection cost.  (a) 2x4 tiles of 4096^2 emulated on one GPU (q = 12.5% per sweep, no RCCL);
(b) one 4096^2 tile exchanging through RCCL loopback with interval_n = 6 (choice over 13 values: Lemire
threshold 9, q = 14% per sweep -- the 8-GPU rejection rate with a real RCCL exchange in every sweep)."""
import os, sys, time, subprocess
import numpy as np
sys.path.insert(0, '.')
if len(sys.argv) == 1:
    for mode in ('emul', 'rccl'):
        for b in ['64', '16', '8', '4', '']:
            env = dict(os.environ)
            if b:
                env['SV_DOMAIN_BATCH'] = b
            subprocess.run([sys.executable, __file__, mode, b or 'auto'], env=env, check=True, timeout=240)
    sys.exit(0)
from supervillain_amd.domain import VillainDomain, unique_id
L = 4096
if sys.argv[1] == 'emul':
    dom, tiles, K = VillainDomain(2 * L, 4 * L, (2, 4), kappa=0.5, W=1), 8, 100
else:
    dom, tiles, K = VillainDomain(L, L, (1, 1), kappa=0.5, W=1, interval_n=6, unique_id=unique_id()), 1, 300
dom.cold()
g = np.random.default_rng(0)
dom.run(10, g)
t0 = time.perf_counter(); st = dom.run(K, g); t1 = time.perf_counter()
print(f'{sys.argv[1]} batch {sys.argv[2]}: per tile-sweep {(t1 - t0) / K / tiles * 1e6:.1f} us, '
      f'rejections {sum(s.rejections for s in st)} in {K} sweeps', flush=True)
