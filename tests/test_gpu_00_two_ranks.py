"""Two real ranks on one GPU: the multi-rank domain code (per-peer halo messages between two processes, the
batch-summary all-gather over two ranks, the abort / replay decision taken on every rank) against the single-process
tile emulation, bit for bit, for a Villain and a Worldline 1 x 2 decomposition (config 4 and config 3 as two GPUs would
run them), with NumPy Lemire rejections forced into the chain (the abort spreading across real ranks).  transport
'rccl': RCCL's ncclSend / ncclRecv and ncclAllGather; 'host': the same two collectives through host memory over the
gloo group (HostTransport, sv_domain_create_hosted) -- every other part of the multi-rank path (one tile per process,
pack / unpack kernels, the message layout per peer, the gathered summaries, rejection prediction) is the RCCL run's.

This file sorts FIRST among the -m gpu tests on purpose: the two ranks are started (spawn: fresh interpreters) before
the test process itself has touched the GPU -- a process that has initialised the GPU must not start new programs.
If RCCL refuses two ranks on one device, the ranks record its exact error and the test is marked xfail with it."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model, transport, predict, out, tiles=(1, 2)):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), SV_DEVICE='0', SV_DOMAIN_BATCH='4')
    if predict is not None:  # rejection prediction (on by default with several ranks) or the abort / replay protocol
        os.environ['SV_DOMAIN_PREDICT'] = predict
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from supervillain_amd.domain import VillainDomain, WorldlineDomain
        from tests.golden import crafted_generator
        if model == 'villain':
            Nt, Nx, steps = 64, 128, 9
            V = Nt * Nx
            pos = 4 * V + 3 * V + V // 3  # sweep 1's colour-1 choice words: a rejection there
            gen = lambda: crafted_generator(pos, pos, 1)  # noqa: E731
            phi0 = np.random.default_rng(4).uniform(-np.pi, np.pi, (Nt, Nx))
            n0 = np.random.default_rng(5).integers(-2, 3, (2, Nt, Nx)).astype(np.int64)
            make = lambda **kw: VillainDomain(Nt, Nx, tiles, kappa=0.5, W=1, **kw)  # noqa: E731
            dist_make = lambda: VillainDomain.distributed(Nt, Nx, tiles, kappa=0.5, W=1, transport=transport)  # noqa: E731
        else:
            Nt, Nx, steps = 64, 128, 6
            V = Nt * Nx
            pos = (2 * V + V + V // 2) + V + 3 * V // 4 + 5  # step 1's colour-1 change_v block
            gen = lambda: crafted_generator(pos, pos, 1)  # noqa: E731
            phi0 = np.random.default_rng(6).integers(-3, 4, (Nt, Nx)).astype(np.int64)
            n0 = np.zeros((2, Nt, Nx), dtype=np.int64)
            make = lambda **kw: WorldlineDomain(Nt, Nx, tiles, kappa=0.5, W=1, **kw)  # noqa: E731
            dist_make = lambda: WorldlineDomain.distributed(Nt, Nx, tiles, kappa=0.5, W=1, transport=transport)  # noqa: E731
        try:
            dom = dist_make()
        except Exception as e:  # RCCL refusing two ranks on one device lands here (ncclCommInitRank)
            if transport != 'rccl':
                raise
            with open(f'{out}.refused', 'w') as f:
                f.write(f'rank {rank}: {e}')
            return
        try:
            if model == 'villain':
                dom.upload(phi0, n0)
            else:
                dom.upload(n0, phi0)
            g = gen()
            st = dom.run(steps, g)
            a, b = dom.download()
        finally:
            dom.close()
        res = [None] * world
        dist.all_gather_object(res, (a, b, [(s.accepted, s.rejections) for s in st], g.bit_generator.state))
        if rank == 0:
            a = res[0][0].copy()
            b = res[0][1].copy()
            Ht, Wt = Nt // tiles[0], Nx // tiles[1]
            for r in range(1, world):  # rank r owns tile r (row-major): rows [iy Ht, +Ht), columns [ix Wt, +Wt)
                ys = slice(r // tiles[1] * Ht, (r // tiles[1] + 1) * Ht)
                xs = slice(r % tiles[1] * Wt, (r % tiles[1] + 1) * Wt)
                if model == 'villain':  # phi (Nt, Nx), n (2, Nt, Nx)
                    a[ys, xs] = res[r][0][ys, xs]
                    b[:, ys, xs] = res[r][1][:, ys, xs]
                else:  # m (2, Nt, Nx), v (Nt, Nx)
                    a[:, ys, xs] = res[r][0][:, ys, xs]
                    b[ys, xs] = res[r][1][ys, xs]
            ref = make()
            try:
                if model == 'villain':
                    ref.upload(phi0, n0)
                else:
                    ref.upload(n0, phi0)
                g2 = gen()
                st2 = ref.run(steps, g2)
                a2, b2 = ref.download()
            finally:
                ref.close()
            ok = ((a == a2).all() and (b == b2).all() and res[0][2] == [(s.accepted, s.rejections) for s in st2]
                  and all(res[r][2] == res[0][2] and res[r][3] == g2.bit_generator.state for r in range(world))
                  and sum(r for _, r in res[0][2]) >= 1)
            with open(f'{out}.result', 'w') as f:
                f.write('ok' if ok else f'mismatch: stats {res[0][2]} vs {[(s.accepted, s.rejections) for s in st2]}')
    except Exception as e:
        with open(f'{out}.error', 'a') as f:
            f.write(f'rank {rank}: {e!r}\n')
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('transport,predict', [('rccl', None), ('host', '0'), ('host', '1')])
@pytest.mark.parametrize('model', ['villain', 'worldline'])
def test_two_ranks_one_gpu(model, transport, predict, tmp_path):
    """predict '0': the forced rejection aborts the batch on the rank that meets it, the abort reaches the other rank
    in the halo messages and the gathered summaries, and both replay; '1': the scan split over the two ranks finds it
    first and both plan around it."""
    import time

    import torch.multiprocessing as mp
    out = str(tmp_path / model)
    ctx = mp.start_processes(_worker, args=(2, _free_port(), model, transport, predict, out), nprocs=2, join=False,
                             start_method='spawn')
    deadline = time.time() + 240  # a rendezvous that never completes must not hang the suite
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                p.kill()
            pytest.fail('two-rank run did not finish in 240 s')
    if transport == 'rccl' and os.path.exists(f'{out}.refused'):
        pytest.xfail('RCCL refused two ranks on one device: ' + open(f'{out}.refused').read())
    assert not os.path.exists(f'{out}.error'), open(f'{out}.error').read()
    assert open(f'{out}.result').read() == 'ok'


@pytest.mark.parametrize('tiles', [(2, 2), (2, 4)])
@pytest.mark.parametrize('model', ['villain', 'worldline'])
def test_more_ranks_one_gpu_hosted(model, tiles, tmp_path):
    """The same with 4 and 8 ranks (2 x 2, 2 x 4: every rank exchanges with several peers, corners included, the
    8-rank layout of BASELINE config 4) over the hosted transport, rejection prediction on (the multi-rank default)."""
    import time

    import torch.multiprocessing as mp
    out = str(tmp_path / model)
    world = tiles[0] * tiles[1]
    ctx = mp.start_processes(_worker, args=(world, _free_port(), model, 'host', None, out, tiles), nprocs=world,
                             join=False, start_method='spawn')
    deadline = time.time() + 240
    while not ctx.join(timeout=5):
        if time.time() > deadline:
            for p in ctx.processes:
                p.kill()
            pytest.fail(f'{world}-rank run did not finish in 240 s')
    assert not os.path.exists(f'{out}.error'), open(f'{out}.error').read()
    assert open(f'{out}.result').read() == 'ok'


@pytest.mark.parametrize('workload', ['villain', 'worldline'])
def test_bench_two_ranks_hosted(workload):
    """`bench.py --gpus 2` end to end -- its own torch.distributed.run launch, one rank per process, the domain line,
    R1 and the single-lattice reference on every rank, max over ranks, rank 0's JSON line -- with both ranks on the one
    GPU (SV_DEVICE=0) and the halos over the hosted transport (RCCL refuses two ranks on one device).  A rehearsal of
    the driver's N > 1 runs, not a measurement.  (Started, like the test above, before this process touches the GPU.)"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SV_DEVICE='0', MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--transport', 'host', '--steps', '4',
           '--warmup', '1', '--warmup-s', '0', '--no-cpu-baseline', '--no-copy-ceiling', '--L', '512',
           '--workload', workload]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([s for s in p.stdout.splitlines() if s.startswith('{')][-1])
    assert line['n_gpus'] == 2 and line['steps'] == 4 and line['value'] > 0
    cfg = line['config']
    assert cfg['halo_transport'] == 'host' and cfg['tiles'] == [1, 2] and cfg['lattice'] == [512, 512]
    assert '512' in line['metric'] and cfg['scaling_reference']['R1'] > 0
