"""Generator persistence: the reference pickles its generators -- rng included -- into the h5
file (supervillain/h5/data.py:75,88) and resumes a chain with Ensemble.continue_from (ensemble.py:103).  A hot-path
generator pickled after k device sweeps and unpickled must continue exactly as the uninterrupted chain: the same
fields, counters, reports and NumPy rng states; the device handle (`_dev`) is never in the pickle (DeviceState)."""
import pickle

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.batch import Batch
from supervillain_amd.generator import villain as gv, worldline as gw
from supervillain_amd.generator.combining import KeepEvery, Sequentially

N = 16
SV = sv.Villain(sv.Lattice2D(N), 0.5, 1)
SW = sv.Worldline(sv.Lattice2D(N), 0.5, 1)

FACTORY = {
    'neighborhood': (SV, lambda: gv.NeighborhoodUpdate(SV)),
    'neighborhood_inline': (SV, lambda: gv.NeighborhoodUpdate(SV, inline=True)),
    'neighborhood_philox': (SV, lambda: gv.NeighborhoodUpdate(SV, philox=5)),
    'neighborhood_keepevery': (SV, lambda: KeepEvery(3, gv.NeighborhoodUpdate(SV))),
    'villain_hammer': (SV, lambda: gv.Hammer(SV)),
    'coexact': (SW, lambda: gw.CoexactUpdate(SW)),
    'plaquette_checkerboard': (SW, lambda: gw.PlaquetteUpdate(SW, mode='checkerboard')),
    'plaquette_reference': (SW, lambda: gw.PlaquetteUpdate(SW, mode='reference')),
    'worldline_hammer': (SW, lambda: gw.Hammer(SW)),
}
FIELDS = {id(SV): ('phi', 'n'), id(SW): ('m', 'v')}


def leaves(G):
    if isinstance(G, Sequentially):
        return [x for g in G.generators for x in leaves(g)]
    if isinstance(G, KeepEvery):
        return leaves(G.generator)
    return [G]


def seeded(make, seed=100):
    np.random.seed(11)  # the reference-order Plaquette's visit orders come from NumPy's global RandomState
    G = make()
    for i, g in enumerate(leaves(G)):
        g.rng = np.random.default_rng(seed + i)
    return G


def counters(G):
    out = []
    for g in leaves(G):
        d = {k: getattr(g, k) for k in ('accepted', 'proposed', 'acceptance', 'sweeps', 'philox_counter')
             if hasattr(g, k)}
        if hasattr(g, 'worm_lengths'):
            d['worm_lengths'] = list(g.worm_lengths)
        d['rng'] = g.rng.bit_generator.state
        out.append(d)
    return out


def assert_same_cfg(a, b, fields):
    for f in fields:
        assert (np.asarray(a[f]) == np.asarray(b[f])).all(), f


def test_pickle_drops_the_device_handle():
    """CPU: a generator whose device state is set pickles without it (an unpicklable stand-in for the handle)."""
    for name, (S, make) in FACTORY.items():
        G = seeded(make)
        for g in leaves(G):
            g._dev = lambda: None  # not picklable: pickling fails if the handle is kept
        blob = pickle.dumps(G)
        assert b'_dev' not in blob, name
        H = pickle.loads(blob)
        for g, h in zip(leaves(G), leaves(H)):
            assert '_dev' not in h.__dict__, name
            assert h.rng.bit_generator.state == g.rng.bit_generator.state, name
            g._dev = None


@pytest.mark.gpu
@pytest.mark.parametrize('name', sorted(FACTORY))
def test_pickled_generator_continues_the_chain(name):
    S, make = FACTORY[name]
    fields = FIELDS[id(S)]
    k, m = 3, 4
    A = seeded(make)
    cfg = S.configurations(1)[0]
    for _ in range(k):
        cfg = A.step(cfg)
    assert any(g.__dict__.get('_dev') is not None for g in leaves(A))  # the chain ran on the device
    blob = pickle.dumps(A)
    assert b'_dev' not in blob
    B = pickle.loads(blob)
    assert counters(B) == counters(A)
    for _ in range(m):
        cfg = B.step(cfg)

    R = seeded(make)
    ref = S.configurations(1)[0]
    for _ in range(k + m):
        ref = R.step(ref)
    assert_same_cfg(cfg, ref, fields)
    assert counters(B) == counters(R)
    assert B.report() == R.report()


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['neighborhood', 'neighborhood_inline', 'villain_hammer', 'plaquette_reference',
                                  'worldline_hammer', 'neighborhood_keepevery'])
def test_continue_from_a_pickled_generator(name):
    """Ensemble.generate(k), the generator pickled and restored (as the reference's h5 round trip does), then
    Ensemble.continue_from(m): the same m draws and indices as draws k .. k + m of one uninterrupted generate."""
    S, make = FACTORY[name]
    k, m = 4, 5
    E = sv.Ensemble(S).generate(k, seeded(make))
    E.generator = pickle.loads(pickle.dumps(E.generator))
    E2 = sv.Ensemble.continue_from(E, m)
    R = seeded(make)
    ER = sv.Ensemble(S).generate(k + m, R)
    for f in E2.configuration.fields:
        a = np.asarray(Batch.as_array(E2.configuration.fields[f]))
        b = np.asarray(Batch.as_array(ER.configuration.fields[f]))[k:]
        assert (a == b).all(), f
    assert (np.asarray(Batch.as_array(E2.index)) == k + np.arange(m)).all()
    assert counters(E2.generator) == counters(R)
