"""Host-side mirror of the reference interface (CPU): lattice, forms, actions, storage, composition.

The Ensemble/KeepEvery/Sequentially logic is exercised with an oracle-backed stand-in generator
(test-only) and compared with golden vectors captured from the reference's own Ensemble.generate."""
import os

import numpy as np
import pytest

import supervillain_amd as sv
from supervillain_amd.batch import Batch
from supervillain_amd.lattice import d, delta
from tests.golden import cases


def test_checkerboarding_matches_reference():
    for c in cases('checkerboarding.npz'):
        L = sv.Lattice2D(c['N'])
        cid = np.full((c['N'], c['N']), -1)
        for i, color in enumerate(L.checkerboarding):
            cid[color] = i
        assert (cid == c['colors']).all()


def test_colours_have_no_same_colour_neighbours():
    for N in range(2, 14):
        L = sv.Lattice2D(N)
        cid = np.full((N, N), -1)
        for i, color in enumerate(L.checkerboarding):
            cid[color] = i
        if N > 2:
            assert (cid != np.roll(cid, 1, 0)).all() and (cid != np.roll(cid, 1, 1)).all()


def test_d_delta_nilpotent_and_dtypes():
    L = sv.Lattice(3, 4)
    rng = np.random.default_rng(0)
    f0 = sv.Form(rng.integers(-3, 4, (1, 4, 4, 4)), degree=0, lattice=L)
    f2 = sv.Form(rng.integers(-3, 4, (3, 4, 4, 4)), degree=2, lattice=L)
    assert (d(d(f0)) == 0).all()
    assert (delta(delta(f2)) == 0).all()
    assert np.asarray(d(f0)).dtype == np.int64 and np.asarray(delta(f2)).dtype == np.int64


def test_villain_action_matches_golden(oracle_lib):
    for c in cases('villain_neighborhood.npz'):
        L = sv.Lattice2D(c['N'])
        S = sv.Villain(L, c['kappa'], c['W'])
        phi = sv.Form(c['phi'][None], degree=0, lattice=L)
        n = sv.Form(c['n'], degree=1, lattice=L)
        np.testing.assert_allclose(S(phi, n), c['action'], rtol=1e-12)
        assert S.valid({'n': n})


def test_worldline_action_matches_golden():
    for c in cases('worldline_coexact.npz'):
        L = sv.Lattice2D(c['N'])
        S = sv.Worldline(L, c['kappa'], c['W'])
        m = sv.Form(c['m'], degree=1, lattice=L)
        v = sv.Form(c['v'][None], degree=2, lattice=L)
        assert S.valid({'m': m})
        np.testing.assert_allclose(S(m, v), c['action'], rtol=1e-12)
    L = sv.Lattice2D(4)
    S = sv.Worldline(L, 0.5, 1)
    bad = L.zeros(1, dtype=int)
    bad[0, 0, 0] = 1
    with pytest.raises(ValueError):
        S(bad, L.zeros(2, dtype=int))


def test_batch_rejects_lossy_casts():
    b = Batch(3, shape=(2,), dtype=int)
    b[0] = np.array([1.0, 2.0])
    with pytest.raises(TypeError):
        b[1] = np.array([1.5, 2.0])


def test_generators_reject_wrong_action():
    L = sv.Lattice2D(4)
    with pytest.raises(ValueError):
        sv.generator.villain.NeighborhoodUpdate(sv.Worldline(L, 0.5, 1))
    with pytest.raises(ValueError):
        sv.generator.worldline.CoexactUpdate(sv.Villain(L, 0.5, 1))
    with pytest.raises(ValueError):
        sv.generator.worldline.PlaquetteUpdate(sv.Villain(L, 0.5, 1))


class OracleNeighborhood(sv.generator.Generator):
    """Test-only stand-in with NeighborhoodUpdate's contract, backed by the CPU oracle."""

    def __init__(self, S, oracle, interval_phi=np.pi):
        self.Action, self.O, self.interval_phi = S, oracle, interval_phi
        self.rng = np.random.default_rng()
        self.accepted = self.proposed = self.sweeps = 0
        self.acceptance = 0.

    def step(self, cfg):
        N = self.Action.Lattice.N
        phi = np.array(cfg['phi'], dtype=float).reshape(N, N).copy()
        n = np.array(cfg['n'], dtype=np.int64).copy()
        st = self.O.villain_neighborhood(N, self.Action.kappa, self.Action.W, phi, n, 1, self.rng,
                                         interval_phi=self.interval_phi)
        V = N * N
        self.sweeps += 1
        self.proposed += V
        self.acceptance += st[0].acceptance_sum / V
        self.accepted += st[0].accepted
        L = self.Action.Lattice
        return cfg | {'phi': sv.Form(phi[None], degree=0, lattice=L), 'n': sv.Form(n, degree=1, lattice=L)}

    def report(self):
        return (f'There were {self.accepted} neighborhood proposals accepted of {self.proposed} proposed updates.'
                + '\n' + f'    {self.accepted/self.proposed:.6f} acceptance rate' + '\n'
                + f'    {self.acceptance / self.sweeps:.6f} average Metropolis acceptance probability.')


def test_ensemble_generate_matches_golden(oracle_lib):
    c = [x for x in cases('ensemble.npz') if x['kind'] == 'villain_generate'][0]
    L = sv.Lattice2D(c['N'])
    S = sv.Villain(L, c['kappa'], c['W'])
    G = OracleNeighborhood(S, oracle_lib)
    G.rng = np.random.default_rng(c['seed'])
    E = sv.Ensemble(S).generate(c['steps'], G, starting_index=c['starting_index'], index_stride=c['index_stride'])
    assert E.configuration.phi.array.shape == c['phi'].shape and E.configuration.phi.dtype == np.float64
    assert E.configuration.n.dtype == np.int64
    assert (E.configuration.phi.array == c['phi']).all() and (E.configuration.n.array == c['n']).all()
    assert (E.index.array == c['index']).all() and (E.weight.array == c['weight']).all()
    assert G.report() == c['report']
    e2 = E.cut(2).every(2)
    assert len(e2) == len(range(2, c['steps'], 2))
    assert isinstance(e2.generator, sv.generator.KeepEvery)


def test_keepevery_sequentially_matches_golden(oracle_lib):
    c = [x for x in cases('ensemble.npz') if x['kind'] == 'keepevery_sequentially'][0]
    L = sv.Lattice2D(c['N'])
    S = sv.Villain(L, c['kappa'], c['W'])
    a, b = OracleNeighborhood(S, oracle_lib), OracleNeighborhood(S, oracle_lib, interval_phi=1.0)
    a.rng, b.rng = np.random.default_rng(8), np.random.default_rng(9)
    G = sv.generator.KeepEvery(3, sv.generator.Sequentially((a, b)))
    E = sv.Ensemble(S).generate(c['steps'], G)
    assert (E.configuration.phi.array == c['phi']).all() and (E.configuration.n.array == c['n']).all()
    assert G.report() == c['report']


def test_worm_wrong_action_raises():
    with pytest.raises(ValueError):
        __import__('supervillain_amd.generator.villain', fromlist=['Worm']).Worm(sv.Worldline(sv.Lattice2D(4), 0.5, 1))
    with pytest.raises(ValueError):
        __import__('supervillain_amd.generator.worldline', fromlist=['Worm']).Worm(sv.Villain(sv.Lattice2D(4), 0.5, 1))


def test_hammer_composition_matches_reference():
    """Hammer(S, worms) as supervillain/generator/{villain,worldline}/__init__.py build it: the worm is always
    the last member in D = 2 (worms = 0 and 1 alike), inside KeepEvery only when worms > 1; LinkUpdate is
    left out at W = infinity; worm=False (an extension) drops the worm."""
    from supervillain_amd.generator import villain as gv, worldline as gw
    from supervillain_amd.generator.combining import KeepEvery
    L = sv.Lattice2D(4)
    for W, names in ((1, ['SiteUpdate', 'LinkUpdate', 'ExactUpdate', 'CohomologyUpdate']),
                     (float('inf'), ['SiteUpdate', 'ExactUpdate', 'CohomologyUpdate'])):
        S = sv.Villain(L, 0.5, W)
        for worms in (0, 1):
            H = gv.Hammer(S, worms)
            assert [type(g).__name__ for g in H.generators] == names + ['ClassicWorm']
        H = gv.Hammer(S, 3)
        assert isinstance(H.generators[-1], KeepEvery) and H.generators[-1].stride == 3
        assert [type(g).__name__ for g in gv.Hammer(S, worm=False).generators] == names
    Sw = sv.Worldline(L, 0.5, 1)
    for worms in (0, 1):
        assert [type(g).__name__ for g in gw.Hammer(Sw, worms).generators] == \
            ['VortexUpdate', 'CoexactUpdate', 'WrappingUpdate', 'ClassicWorm']
    assert isinstance(gw.Hammer(Sw, 2).generators[-1], KeepEvery)
    assert len(gw.Hammer(Sw, worm=False).generators) == 3


def test_rng_batch_roundtrip():
    """sv_rng_gather / sv_rng_scatter (host-only C-ABI) read and write NumPy's PCG64 states exactly like the
    public state dict, including the half-word buffer."""
    from supervillain_amd._abi import rng_from_numpy, rngs_from_numpy, rngs_to_numpy
    gens = [np.random.default_rng(s) for s in range(37)]
    for i, g in enumerate(gens):
        g.integers(0, 3, i % 5)  # odd counts leave a buffered half-word
    arr, addrs = rngs_from_numpy(gens)
    assert addrs is not None
    for x, g in zip(arr, gens):
        y = rng_from_numpy(g)
        assert (x.state_hi, x.state_lo, x.inc_hi, x.inc_lo, x.has_uint32, x.uinteger) == \
               (y.state_hi, y.state_lo, y.inc_hi, y.inc_lo, y.has_uint32, y.uinteger)
    twins = [np.random.default_rng(99) for _ in gens]
    rngs_to_numpy(arr, twins, rngs_from_numpy(twins)[1])
    for a, b in zip(gens, twins):
        assert a.bit_generator.state == b.bit_generator.state
        assert (a.integers(0, 7, 9) == b.integers(0, 7, 9)).all()


def test_bench_json_contract(capsys):
    """bench.py's report line carries every field the driver and the judge read (CPU-only: synthetic timings,
    the CPU baseline on a small lattice)."""
    import json
    import types
    import bench
    args = types.SimpleNamespace(steps=10, warmup=2, strong=False, no_cpu_baseline=False, L=64, kappa=0.5, W=1,
                                 cpu_sweeps=2)
    bench.report(args, 1, 4096 * 4096, 4096 * 4096, 3.2e-3, 0.004, 3.2e-4,
                 {'workload': 'L=4096 test', 'L': 4096, 'parallelism': 'single GPU'}, 4096)
    d = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline'):
        assert k in d, k
    assert d['config']['workload'] and d['higher_is_better'] is True and d['scaling'] == 'weak'
    r = d['roofline']
    assert r['bound'] == 'hbm' and r['unit'] == 'GB/s' and abs(r['frac'] - r['achieved'] / r['peak']) < 1e-12
    assert r['traffic'] and r['traffic'] > 0.5 * 48 * 4096 * 4096  # the committed PMC summary
    c = d['cpu_baseline']
    assert c['cores'] >= 1 and c['kind'] == 'port' and c['value'] > 0 and c['value_1core'] > 0
    assert abs(d['value'] - 10 * 4096 * 4096 / 3.2e-3) < 1e-3 * d['value']


def test_bench_metric_names_the_lattice(capsys, monkeypatch):
    """a line's metric names the lattice the run swept -- BASELINE.json's metric verbatim for one
    L=4096 lattice (N = 1 and config 4's tiles of it, the default for --gpus N), the (ty L) x (tx L) lattice for
    --weak -- and report() refuses a line whose metric and config.lattice disagree."""
    import json
    import sys
    import types
    import bench
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'BASELINE.json')) as f:
        baseline_metric = json.load(f)['metric']
    assert bench.lattice_metric(4096, 4096) == bench.HEADLINE_METRIC == baseline_metric
    assert bench.metric_lattice(baseline_metric) == (4096, 4096)
    weak = bench.lattice_metric(8192, 16384, weak_tile=[4096, 4096])
    assert bench.metric_lattice(weak) == (8192, 16384) and 'L=4096' not in weak
    assert bench.metric_lattice(bench.lattice_metric(256, 256)) == (256, 256)
    wl = bench.lattice_metric(2048, 4096, 'Worldline', [1024, 1024], head='plaquette-steps/sec (x)', tail=', W=1')
    assert bench.metric_lattice(wl) == (2048, 4096)
    # the scaling default: config 4 (strong) for --gpus N unless --weak
    for argv, strong in ((['--gpus', '8'], True), (['--gpus', '8', '--weak'], False), (['--tiles', '2x4'], True),
                         (['--tiles', '2x4', '--weak'], False), ([], True)):
        monkeypatch.setattr(sys, 'argv', ['bench.py'] + argv)
        assert bench.parse().strong is strong, argv
    args = types.SimpleNamespace(steps=10, warmup=2, strong=True, no_cpu_baseline=True, L=4096, kappa=0.5, W=1)
    with pytest.raises(ValueError):
        bench.report(args, 8, 8192 * 16384, 4096 * 4096, 1.0, 0.004, 3e-4, {'workload': 'x', 'lattice': [8192, 16384]},
                     4096)  # the headline metric on the weak lattice
    bench.report(args, 8, 4096 * 4096, 2048 * 1024, 1.0, 0.004, 3e-5, {'workload': 'x', 'lattice': [4096, 4096]}, 2048)
    d = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert d['metric'] == baseline_metric and d['scaling'] == 'strong' and d['n_gpus'] == 8
    # an efficiency above 1.02 is flagged
    ref = bench.scaling_reference(8.5e11, 8, 1.0e11, [2048, 1024], 7.0e10, 0)
    assert ref['E_N_suspect'] and abs(ref['E_N'] - 1.0625) < 1e-12
    assert 'suspect' in capsys.readouterr().err
    ref = bench.scaling_reference(6.0e11, 8, 1.0e11, [2048, 1024], 7.0e10, 0)
    assert not ref['E_N_suspect'] and abs(ref['E_N_vs_single_lattice'] - 6.0e11 / 5.6e11) < 1e-12
