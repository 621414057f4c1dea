"""ExtendableStore (supervillain_amd/store.py) and Ensemble streaming: the role of the reference's extendable
HDF5 datasets (supervillain/h5/extendable.py:62-74, Ensemble.extend_h5) without HDF5.  CPU only: the chain
comes from the oracle-backed generator of test_host (test infrastructure)."""
import json
import os

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.store import ExtendableStore
from test_host import OracleNeighborhood


def test_store_extend_and_read(tmp_path):
    s = ExtendableStore(tmp_path / 'a')
    assert len(s) == 0
    x = np.arange(24.0).reshape(3, 2, 4)
    i = np.arange(3, dtype=np.int64)
    s.extend({'x': x, 'i': i})
    s.extend({'x': x[:1] + 100, 'i': i[:1] + 7})
    r = ExtendableStore(tmp_path / 'a', create=False)
    assert len(r) == 4 and sorted(r.columns()) == ['i', 'x']
    assert (r.read('x')[:3] == x).all() and (r.read('x')[3] == x[0] + 100).all()
    assert r.read('i').tolist() == [0, 1, 2, 7]
    with pytest.raises(KeyError):
        r.extend({'x': x})
    with pytest.raises(ValueError):
        r.extend({'x': x.astype(np.float32), 'i': i})
    with pytest.raises(ValueError):
        r.extend({'x': x[:, :1], 'i': i})
    with pytest.raises(ValueError):
        r.extend({'x': x, 'i': i[:2]})
    with pytest.raises(FileNotFoundError):
        ExtendableStore(tmp_path / 'none', create=False)


def test_store_drops_a_torn_tail(tmp_path):
    """Bytes past the manifest's draw count (an extend cut short) are overwritten by the next extend."""
    s = ExtendableStore(tmp_path / 'a').extend({'x': np.ones((2, 3))})
    with open(os.path.join(s.path, 'x.bin'), 'ab') as f:
        f.write(b'\xff' * 11)
    s = ExtendableStore(tmp_path / 'a')
    s.extend({'x': np.full((1, 3), 5.0)})
    assert s.read('x').tolist() == [[1, 1, 1], [1, 1, 1], [5, 5, 5]]
    assert os.path.getsize(os.path.join(s.path, 'x.bin')) == 3 * 3 * 8
    assert json.load(open(os.path.join(s.path, 'manifest.json')))['draws'] == 3


def chain(oracle_lib, N=8, seed=3):
    S = sv.Villain(sv.Lattice2D(N), 0.5, 1)
    G = OracleNeighborhood(S, oracle_lib)
    G.rng = np.random.default_rng(seed)
    return S, G


@pytest.mark.parametrize('every', [1, 3, 64])
def test_generate_streams_to_store(tmp_path, oracle_lib, every):
    S, G = chain(oracle_lib)
    E = sv.Ensemble(S).generate(7, G, stream=tmp_path / 's', stream_every=every, starting_index=10, index_stride=2)
    st = ExtendableStore(tmp_path / 's', create=False)
    assert len(st) == 7
    assert (st.read('phi') == E.configuration.phi.array).all() and (st.read('n') == E.configuration.n.array).all()
    assert st.read('index').tolist() == list(range(10, 24, 2)) and (st.read('weight') == 1).all()
    F = sv.Ensemble.from_store(S, st)
    assert (F.configuration.phi.array == E.configuration.phi.array).all() and F.index_stride == 2


def test_extend_store_continues(tmp_path, oracle_lib):
    S, G = chain(oracle_lib)
    E = sv.Ensemble(S).generate(4, G)
    st = E.to_store(tmp_path / 's')
    with pytest.raises(FileExistsError):
        E.to_store(tmp_path / 's')
    E2 = sv.Ensemble.continue_from(E, 3)
    E2.extend_store(tmp_path / 's')
    S2, G2 = chain(oracle_lib)
    whole = sv.Ensemble(S2).generate(7, G2)
    st = ExtendableStore(tmp_path / 's', create=False)
    assert (st.read('phi') == whole.configuration.phi.array).all() and (st.read('n') == whole.configuration.n.array).all()
    assert st.read('index').tolist() == list(range(7))
