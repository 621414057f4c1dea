"""Integrated autocorrelation time (Sokal window, c = 5) of ActionDensity for the Villain chains of
tests/test_gpu_statparity.py: the counter-based NeighborhoodUpdate alone and the reference's Link + Site + Exact +
Cohomology suite, per (N, kappa).  Sets the thinning the statistical comparison needs."""
import sys

import numpy as np

sys.path.insert(0, '.')
from tests.test_gpu_statparity import villain_chain  # noqa: E402


def tau_int(x, c=5.0):
    x = np.asarray(x, float) - np.mean(x)
    n = len(x)
    f = np.fft.rfft(x, 2 * n)
    acf = np.fft.irfft(f * np.conj(f))[:n]
    acf /= acf[0] if acf[0] > 0 else 1
    tau = 0.5
    for m in range(1, n):
        tau += acf[m]
        if m >= c * tau:
            break
    return tau


steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
for N in (8, 16):
    for kappa in (0.25, 0.5, 1.0):
        out = []
        for suite in ('philox', 'pcg64'):
            o = villain_chain(N, kappa, suite, steps, 1)[steps // 10:, 0]
            out.append(f'{suite}: mean {o.mean():.4f} tau {tau_int(o):.1f}')
        print(f'N={N} kappa={kappa}: ' + '; '.join(out), flush=True)
