import numpy as np, ctypes, sys
sys.path.insert(0, '.')
import supervillain_amd as sv
from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy
from oracle import oracle as O
N = 4
S = sv.Villain(sv.Lattice2D(N), 0.5, 1)
G = sv.generator.villain.CohomologyUpdate(S)
for sweeps in (1, 2):
    G.rng = np.random.default_rng(5)
    r = rng_from_numpy(G.rng)
    print('in ', r.state_hi, r.state_lo, r.inc_hi, r.inc_lo, r.has_uint32, r.uinteger)
    ctx, _, h = G._state()
    st = _native.stats_array(sweeps)
    phi = np.zeros((N, N)); n = np.zeros((2, N, N), dtype=np.int64)
    L = _native.lib()
    ctx.check(L.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'up')
    ctx.check(L.sv_villain_cohomology_run(h, 0.5, 1, sweeps, ctypes.byref(r), st), 'run')
    print('dev', r.state_hi, r.state_lo, r.has_uint32, r.uinteger, [(s.accepted, s.acceptance_sum) for s in st])
    g = np.random.default_rng(5)
    stt = O.villain_generator('CohomologyUpdate', N, 0.5, 1, phi.copy(), n.copy(), sweeps, g)
    r2 = rng_from_numpy(g)
    print('ora', r2.state_hi, r2.state_lo, r2.has_uint32, r2.uinteger, [(s.accepted, s.acceptance_sum) for s in stt])
