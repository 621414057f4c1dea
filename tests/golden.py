"""Loader for the golden fixtures in tests/golden/ (made by tools/make_golden.py from the reference)."""
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def cases(name):
    z = np.load(os.path.join(HERE, name), allow_pickle=False)
    out = []
    for i in range(int(z['count'])):
        prefix = f'{i}/'
        c = {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}
        for k, v in list(c.items()):
            if v.shape == () and v.dtype.kind in 'iuf':
                c[k] = v.item()
            elif v.shape == () and v.dtype.kind == 'U':
                c[k] = str(v)
        out.append(c)
    return out


def generator_from(state):
    """A NumPy Generator(PCG64) positioned at a recorded state (6 uint64: s_hi s_lo inc_hi inc_lo has buf)."""
    s = [int(x) for x in state]
    g = np.random.Generator(np.random.PCG64())
    st = g.bit_generator.state
    st['state'] = {'state': (s[0] << 64) | s[1], 'inc': (s[2] << 64) | s[3]}
    st['has_uint32'] = s[4]
    st['uinteger'] = s[5]
    g.bit_generator.state = st
    return g


def state_of(gen):
    st = gen.bit_generator.state
    s, inc = st['state']['state'], st['state']['inc']
    return np.array([s >> 64, s & ((1 << 64) - 1), inc >> 64, inc & ((1 << 64) - 1), st['has_uint32'],
                     st['uinteger']], dtype=np.uint64)


_MULT = 0x2360ED051FC65DA44385DF649FCCF645
_MINV = pow(_MULT, -1, 1 << 128)
_M128 = (1 << 128) - 1


def crafted_generator(seed, position, half):
    """A Generator(PCG64) whose raw output `position` has its low (half=0) or high (half=1) 32 bits
    zero, forcing a NumPy Lemire rejection there (natural rate 2^-32 per draw)."""
    gen = np.random.default_rng(seed)
    inc = gen.bit_generator.state['state']['inc']
    hi = (0x0123456789ABCDEF ^ (seed * 0x9E3779B1)) & ((1 << 58) - 1)
    out = 0xDEADBEEF00000000 if half == 0 else 0x00000000DEADBEEF
    s = (hi << 64) | (hi ^ out)
    for _ in range(position + 1):
        s = ((s - inc) * _MINV) & _M128
    st = gen.bit_generator.state
    st['state']['state'] = s
    st['has_uint32'] = 0
    st['uinteger'] = 0
    gen.bit_generator.state = st
    return gen


def observable_start(c):
    """The starting fields of a villain_observables.npz chain (tools/make_golden_observables.hot_start: cold, or phi
    uniform in [-pi, pi) and n in W * {-2..2} from the chain's hot-start seed)."""
    N, W = c['N'], c['W']
    if c['hot_seed'] < 0:
        return np.zeros((N, N)), np.zeros((2, N, N), dtype=np.int64)
    r = np.random.default_rng(c['hot_seed'])
    return r.uniform(-np.pi, np.pi, (1, N, N))[0], (W * r.integers(-2, 3, (2, N, N))).astype(np.int64)


def observable_groups():
    """villain_observables.npz chains by group (one N, kappa, W per group: a replica batch)."""
    groups = {}
    for c in cases('villain_observables.npz'):
        groups.setdefault(c['group'], []).append(c)
    return groups
