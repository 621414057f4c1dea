"""Device-resident Ensemble.generate (supervillain_amd/pipeline.py) against the per-step
host loop it replaces (supervillain/ensemble.py:74-98): identical storage, rng states, counters and reports."""
import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.generator import villain as gv, worldline as gw
from supervillain_amd.generator.combining import KeepEvery, Sequentially
from supervillain_amd.pipeline import device_program

pytestmark = pytest.mark.gpu


def villain_hammer(S, seeds):
    H = gv.Hammer(S)
    for G, s in zip(H.generators, seeds):
        G.rng = np.random.default_rng(s)
    return H


def both(make, S, steps, fields):
    out = []
    for resident in (False, True):
        G = make()
        E = sv.Ensemble(S).generate(steps, G, device_resident=resident)
        out.append((E, G))
    (E0, G0), (E1, G1) = out
    for f in fields:
        a = np.asarray(getattr(E0, f).array if hasattr(getattr(E0, f), 'array') else getattr(E0, f))
        b = np.asarray(getattr(E1, f).array if hasattr(getattr(E1, f), 'array') else getattr(E1, f))
        assert (a == b).all(), f  # (the device's float observables are exact sums: common.h)
    assert G0.report() == G1.report()
    return G0, G1


def rng_states(G):
    gens = G.generators if isinstance(G, Sequentially) else [G.generator] if isinstance(G, KeepEvery) else [G]
    out = []
    for g in gens:
        if isinstance(g, Sequentially):
            out += rng_states(g)
        else:
            out.append(g.rng.bit_generator.state)
    return out


def test_program_flattening():
    S = sv.Villain(sv.Lattice2D(8), 0.5, 1)
    a, b = gv.SiteUpdate(S), gv.ExactUpdate(S)
    p = device_program(KeepEvery(3, Sequentially((a, b))))
    assert [(g, k) for g, k in p] == [(a, 1), (b, 1)] * 3
    p = device_program(Sequentially((KeepEvery(4, a), b, b)))
    assert p == [(a, 4), (b, 2)]
    n = gv.NeighborhoodUpdate(S, inline=True)
    assert device_program(KeepEvery(2, n)) is None            # blocked inline observables: host loop
    assert device_program(KeepEvery(2, n, blocked_inline=False)) == [(n, 2)]


@pytest.mark.parametrize('N,W', [(16, 1), (9, 2), (32, 3)])
def test_villain_hammer_resident(N, W):
    S = sv.Villain(sv.Lattice2D(N), 0.4, W)
    G0, G1 = both(lambda: villain_hammer(S, [1, 2, 3, 4, 5]), S, 12, ['phi', 'n', 'Vortex_Vortex', 'Worm_Length'])
    assert rng_states(G0) == rng_states(G1)


def test_keepevery_neighborhood_inline_resident():
    S = sv.Villain(sv.Lattice2D(16), 0.3, 1)

    def make():
        G = gv.NeighborhoodUpdate(S, inline=True)
        G.rng = np.random.default_rng(5)
        return KeepEvery(3, G, blocked_inline=False)
    both(make, S, 7, ['phi', 'n', 'ActionDensity', 'InternalEnergyDensity', 'WindingSquared', 'TorusWrapping'])


@pytest.mark.parametrize('W', [1, 2, float('inf')])
def test_worldline_hammer_resident(W):
    S = sv.Worldline(sv.Lattice2D(12), 0.5, W)

    def make():
        H = gw.Hammer(S)
        for G, s in zip(H.generators, [7, 8, 9, 10]):
            G.rng = np.random.default_rng(s)
        return H
    G0, G1 = both(make, S, 10, ['m', 'v', 'Spin_Spin', 'Worm_Length'])
    assert rng_states(G0) == rng_states(G1)


def test_plaquette_reference_order_resident():
    """PlaquetteUpdate draws its visit order from NumPy's global RandomState (plaquette.py:63)."""
    S = sv.Worldline(sv.Lattice2D(8), 0.5, 1)
    res = []
    for resident in (False, True):
        np.random.seed(123)
        G = gw.PlaquetteUpdate(S)
        G.rng = np.random.default_rng(4)
        C = gw.CoexactUpdate(S)
        C.rng = np.random.default_rng(5)
        E = sv.Ensemble(S).generate(6, Sequentially((G, C)), device_resident=resident)
        res.append((np.asarray(E.m.array if hasattr(E.m, 'array') else E.m).copy(), G.report()))
    assert (res[0][0] == res[1][0]).all() and res[0][1] == res[1][1]


def test_villain_hammer_worms_keepevery():
    """Hammer(S, worms=3): the worm inside KeepEvery (blocked inline observables averaged, combining.py:100-112)
    keeps the host loop; Hammer(S, worm=False) is the worm-free program."""
    S = sv.Villain(sv.Lattice2D(8), 0.5, 2)
    H = gv.Hammer(S, worms=3)
    assert isinstance(H.generators[-1], KeepEvery) and device_program(H) is None
    assert device_program(gv.Hammer(S, worm=False)) is not None
    for G, s in zip(H.generators[:-1], [1, 2, 3, 4]):
        G.rng = np.random.default_rng(s)
    H.generators[-1].generator.rng = np.random.default_rng(5)
    E = sv.Ensemble(S).generate(4, H)
    assert np.asarray(E.Vortex_Vortex.array if hasattr(E.Vortex_Vortex, 'array') else E.Vortex_Vortex).shape == (4, 8, 8)


def test_emissions_in_flight():
    """Three emissions over the two device buffers before one wait: each host array holds its own step."""
    from supervillain_amd.pipeline import DeviceChain
    S = sv.Villain(sv.Lattice2D(64), 0.5, 1)
    ref = []
    for emit in (False, True):
        G = gv.NeighborhoodUpdate(S)
        G.rng = np.random.default_rng(11)
        ch = DeviceChain(S, device_program(KeepEvery(2, G)))
        try:
            ch.upload(S.configurations(1)[0])
            outs = []
            for _ in range(3):
                ch.advance()
                if emit:
                    a, b = np.empty_like(ch.a), np.empty_like(ch.b)
                    ch.emit(a, b)
                    outs.append((a, b))
                else:
                    d = ch.download()
                    outs.append((d['phi'].copy(), d['n'].copy()))
            if emit:
                ch.emit_wait()
        finally:
            ch.close()
        ref.append(outs)
    for (a0, b0), (a1, b1) in zip(*ref):
        assert (a0 == a1).all() and (b0 == b1).all()


@pytest.mark.parametrize('N,resident', [(256, True), (48, False)])
def test_generate_stream_resident(tmp_path, N, resident):
    """Ensemble.generate(stream=...) with the emission path (pinned storage, copy stream) and the host loop: the
    store equals the ensemble, and the chain equals the per-step loop."""
    from supervillain_amd.store import ExtendableStore
    S = sv.Villain(sv.Lattice2D(N), 0.5, 1)
    out = []
    for dev, path in ((False, None), (resident, tmp_path / 's')):
        G = gv.NeighborhoodUpdate(S)
        G.rng = np.random.default_rng(21)
        E = sv.Ensemble(S).generate(9, KeepEvery(2, G), device_resident=dev, stream=path, stream_every=4)
        out.append(E)
    st = ExtendableStore(tmp_path / 's', create=False)
    assert len(st) == 9
    for f in ('phi', 'n'):
        a = getattr(out[0].configuration, f).array
        assert (getattr(out[1].configuration, f).array == a).all() and (st.read(f) == a).all()
