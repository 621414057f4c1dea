"""Quick timing of replica batches (config 5 shape: L=128, W=2, inline observables).
  python scripts/replica_timing.py [R N inline] ..."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from supervillain_amd.replicas import VillainReplicas  # noqa: E402

cases = [(128, 128, True), (128, 128, False), (1024, 128, True), (64, 256, True)]
if len(sys.argv) > 1:
    a = sys.argv[1:]
    cases = [(int(a[i]), int(a[i + 1]), a[i + 2] == '1') for i in range(0, len(a), 3)]
for R, N, inline in cases:
    B = VillainReplicas(R, N, 0.5, 2)
    B.cold()
    gens = [np.random.default_rng(r) for r in range(R)]
    B.run(10, gens, inline=inline)
    sweeps = 200
    t = time.perf_counter()
    B.run(sweeps, gens, inline=inline)
    dt = time.perf_counter() - t
    print(f'TH={os.environ.get("SV_FUSED_TH", "64")} R={R} N={N} inline={inline}: {sweeps / dt:.1f} sweeps/s, '
          f'{R * N * N * sweeps / dt / 1e9:.2f} G replica-site updates/s', flush=True)
    B.close()
