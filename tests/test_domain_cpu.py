"""Domain decomposition host logic (CPU): the halo plan computed by libsvhip.so fills every ghost cell
with the right periodic neighbour value, its send/receive order matches pairwise (the RCCL
point-to-point matching rule), and a real 2-rank exchange over torch.distributed (gloo) executed
from that plan reproduces the ghost frames -- for the Villain decomposition (2/3-wide ghost frame) and the
Worldline one (5/4-wide).  The device kernels are covered by test_gpu_domain.py and test_gpu_wdomain.py."""
import os
import socket

import numpy as np
import pytest

from supervillain_amd.domain import GHOSTS, exchange_plan, ghost_frame, message_layout, tile_grid

MODELS = list(GHOSTS)


def test_tile_grid():
    assert [tile_grid(n) for n in (1, 2, 4, 8, 6, 3)] == [(1, 1), (1, 2), (2, 2), (2, 4), (2, 3), (1, 3)]


def padded_tile(G, tiles, rank, model):
    """Tile `rank` of global array G with an unfilled (NaN) ghost frame."""
    GT, GB, GL, GR = ghost_frame(*G.shape, tiles, model)
    Nt, Nx = G.shape
    ty, tx = tiles
    Ht, Wt = Nt // ty, Nx // tx
    iy, ix = divmod(rank, tx)
    P = np.full((Ht + GT + GB, Wt + GL + GR), np.nan)
    P[GT:GT + Ht, GL:GL + Wt] = G[iy * Ht:(iy + 1) * Ht, ix * Wt:(ix + 1) * Wt]
    return P


def expected_frame(G, tiles, rank, model):
    GT, GB, GL, GR = ghost_frame(*G.shape, tiles, model)
    Nt, Nx = G.shape
    ty, tx = tiles
    Ht, Wt = Nt // ty, Nx // tx
    iy, ix = divmod(rank, tx)
    rows = (np.arange(-GT, Ht + GB) + iy * Ht) % Nt
    cols = (np.arange(-GL, Wt + GR) + ix * Wt) % Nx
    return G[np.ix_(rows, cols)]


def message(P, m, model, ghost):
    GT, GB, GL, GR = ghost
    (r0, c0), (h, w) = m['src'], m['shape']
    return P[GT + r0:GT + r0 + h, GL + c0:GL + c0 + w].copy()


def place(P, m, block, model, ghost):
    GT, GB, GL, GR = ghost
    (r0, c0), (h, w) = m['dst'], m['shape']
    P[GT + r0:GT + r0 + h, GL + c0:GL + c0 + w] = block


GRIDS = [(1, 1), (1, 2), (2, 1), (2, 2), (2, 4), (3, 2), (1, 8), (4, 4)]


@pytest.mark.parametrize('model', MODELS)
@pytest.mark.parametrize('tiles', GRIDS)
@pytest.mark.parametrize('size', [(8, 6), (24, 24)])  # small tiles clamp the Villain depth, 24 x 24 tiles take K = 4
def test_plan_fills_every_ghost(tiles, model, size):
    ty, tx = tiles
    Nt, Nx = size[0] * ty, size[1] * tx
    G = np.random.default_rng(0).normal(size=(Nt, Nx))
    gh = ghost_frame(Nt, Nx, tiles, model)
    ntiles = ty * tx
    plans = [exchange_plan(Nt, Nx, tiles, r, model) for r in range(ntiles)]
    P = [padded_tile(G, tiles, r, model) for r in range(ntiles)]
    sent = {}
    for r in range(ntiles):
        for s, m in enumerate(plans[r]):
            sent[(r, m['send_to'], s)] = message(P[r], m, model, gh)
    for r in range(ntiles):
        for s, m in enumerate(plans[r]):
            place(P[r], m, sent[(m['recv_from'], r, s)], model, gh)
    for r in range(ntiles):
        np.testing.assert_array_equal(P[r], expected_frame(G, tiles, r, model))


@pytest.mark.parametrize('model', MODELS)
@pytest.mark.parametrize('tiles', GRIDS)
def test_plan_pairwise_order_matches(tiles, model):
    """ncclSend/ncclRecv between one pair of ranks match in call order: rank a's sends to b (in send
    order) must be b's receives from a (in receive order), message by message."""
    ty, tx = tiles
    Nt, Nx = 8 * ty, 6 * tx
    ntiles = ty * tx
    plans = [exchange_plan(Nt, Nx, tiles, r, model) for r in range(ntiles)]
    for a in range(ntiles):
        for b in range(ntiles):
            if a == b:
                continue
            sends = [s for s, m in enumerate(plans[a]) if m['send_to'] == b]
            recvs = [s for s, m in enumerate(plans[b]) if m['recv_from'] == a]
            assert sends == recvs
            for s in sends:
                assert plans[a][s]['shape'] == plans[b][s]['shape']


def test_plan_rejects_bad_decompositions():
    with pytest.raises(ValueError):
        exchange_plan(10, 12, (4, 1), 0)   # does not divide
    with pytest.raises(ValueError):
        exchange_plan(6, 12, (2, 2), 0)    # odd tile extent
    with pytest.raises(ValueError):
        exchange_plan(4, 4, (2, 2), 0)     # 2 x 2 tiles are too small
    with pytest.raises(ValueError):
        exchange_plan(8, 8, (2, 2), 0, 'worldline')  # 4 x 4 tiles are smaller than the 5-wide ghost frame


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _exchange_worker(rank, world, port, tiles, Nt, Nx, errfile, model):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        G = np.random.default_rng(1).normal(size=(Nt, Nx))
        gh = ghost_frame(Nt, Nx, tiles, model)
        plan = exchange_plan(Nt, Nx, tiles, rank, model)
        lay = message_layout(Nt, Nx, tiles, rank, model)
        P = padded_tile(G, tiles, rank, model)
        # the C++ RCCL loop: a send buffer laid out per peer (message s at soff[s] = [flag, pad, phi, n0, n1]),
        # one send per distinct peer, one receive per distinct source; self messages stay local
        send = np.zeros(lay['msg_words'])
        for s, m in enumerate(plan):
            blk = message(P, m, model, gh).ravel()
            o = lay['soff'][s]
            assert lay['words'][s] == 2 + 3 * blk.size
            send[o + 2:o + 2 + blk.size] = blk
        recvbuf = torch.zeros(lay['msg_words'], dtype=torch.float64)
        ops = [dist.P2POp(dist.isend, torch.from_numpy(send[o:o + w].copy()), peer) for peer, o, w in lay['sends']]
        ops += [dist.P2POp(dist.irecv, recvbuf[o:o + w], peer) for peer, o, w in lay['recvs']]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        remote = {s for s, m in enumerate(plan) if m['recv_from'] != rank}
        for s, m in enumerate(plan):
            cnt = int(np.prod(m['shape']))
            if s in remote:
                o = lay['roff'][s]
                block = recvbuf.numpy()[o + 2:o + 2 + cnt].reshape(m['shape'])
            else:
                block = message(P, plan[s], model, gh)
            place(P, m, block, model, gh)
        np.testing.assert_array_equal(P, expected_frame(G, tiles, rank, model))
    except Exception as e:  # report to the parent
        with open(errfile, 'a') as f:
            f.write(f'rank {rank}: {e!r}\n')
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('model', MODELS)
@pytest.mark.parametrize('tiles', [(1, 2), (2, 1), (2, 2)])
def test_two_rank_gloo_exchange(tiles, model, tmp_path):
    import torch.multiprocessing as mp
    errfile = str(tmp_path / 'err.txt')
    Nt, Nx = 24 * tiles[0], 24 * tiles[1]  # Villain tiles of 24 x 24: depth 4, the 8 / 12-deep frame
    world = tiles[0] * tiles[1]
    mp.start_processes(_exchange_worker, args=(world, _free_port(), tiles, Nt, Nx, errfile, model), nprocs=world,
                       join=True, start_method='spawn')
    assert not os.path.exists(errfile), open(errfile).read()


@pytest.mark.parametrize('model', MODELS)
@pytest.mark.parametrize('tiles', GRIDS)
@pytest.mark.parametrize('size', [(8, 6), (24, 24)])
def test_rccl_blocks_line_up(tiles, model, size):
    """The per-peer message blocks libsvhip.so sends (one ncclSend / ncclRecv per distinct peer): rank a's block
    for b and rank b's block from a have the same size, and every message s sits at the same offset inside
    both blocks, so the receiver's ghost block s gets exactly the sender's message s."""
    from supervillain_amd.domain import exchange_plan, message_layout
    ty, tx = tiles
    Nt, Nx = size[0] * ty, size[1] * tx
    ntiles = ty * tx
    lay = [message_layout(Nt, Nx, tiles, r, model) for r in range(ntiles)]
    plans = [exchange_plan(Nt, Nx, tiles, r, model) for r in range(ntiles)]
    for a in range(ntiles):
        L = lay[a]
        # blocks are disjoint, inside the buffer, and one per distinct remote peer
        spans = sorted((o, o + w) for _, o, w in L['sends'])
        assert all(e0 <= s1 for (_, e0), (s1, _) in zip(spans, spans[1:]))
        assert all(e <= L['msg_words'] for _, e in spans)
        assert len({p for p, _, _ in L['sends']}) == len(L['sends'])
        assert {p for p, _, _ in L['sends']} == {m['send_to'] for m in plans[a] if m['send_to'] != a}
        for b, off, words in L['sends']:
            rb = [x for x in lay[b]['recvs'] if x[0] == a]
            assert len(rb) == 1 and rb[0][2] == words
            roff = rb[0][1]
            dirs = [s for s in range(8) if plans[a][s]['send_to'] == b]
            assert dirs == [s for s in range(8) if plans[b][s]['recv_from'] == a]
            assert sum(L['words'][s] for s in dirs) == words
            for s in dirs:
                assert L['soff'][s] - off == lay[b]['roff'][s] - roff


def _hosted_worker(rank, world, port, tiles, errfile):
    import ctypes

    import torch.distributed as dist
    from supervillain_amd.domain import HostTransport
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        Nt, Nx = 24 * tiles[0], 24 * tiles[1]
        lay = message_layout(Nt, Nx, tiles, rank)
        t = HostTransport()
        # the library's call: this rank's messages {peer, offset, words} over host buffers, through the C callback
        send = np.zeros(lay['msg_words'], dtype=np.uint64)
        for peer, o, w in lay['sends']:
            send[o:o + w] = (np.uint64(rank) << np.uint64(48)) + (np.uint64(peer) << np.uint64(32)) + np.arange(w, dtype=np.uint64)
        recv = np.zeros(lay['msg_words'], dtype=np.uint64)
        flat = lambda lst: (ctypes.c_int64 * max(1, 3 * len(lst)))(*[v for m in lst for v in m])  # noqa: E731
        rc = t.xfer(None, len(lay['sends']), flat(lay['sends']), send.ctypes.data, len(lay['recvs']),
                    flat(lay['recvs']), recv.ctypes.data)
        assert rc == 0 and t.error is None, t.error
        for peer, o, w in lay['recvs']:  # what the peer sent to this rank, in its own layout
            exp = (np.uint64(peer) << np.uint64(48)) + (np.uint64(rank) << np.uint64(32)) + np.arange(w, dtype=np.uint64)
            np.testing.assert_array_equal(recv[o:o + w], exp)
        # the batch-summary all-gather: every rank's bytes, in rank order
        nbytes = 40
        mine = np.full(nbytes, rank + 1, dtype=np.uint8)
        out = np.zeros(world * nbytes, dtype=np.uint8)
        assert t.gather(None, mine.ctypes.data, out.ctypes.data, nbytes) == 0
        np.testing.assert_array_equal(out, np.repeat(np.arange(1, world + 1, dtype=np.uint8), nbytes))
    except Exception as e:
        with open(errfile, 'a') as f:
            f.write(f'rank {rank}: {e!r}\n')
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('tiles', [(1, 2), (2, 2)])
def test_host_transport_callbacks(tiles, tmp_path):
    """HostTransport (sv_domain_create_hosted's callbacks over gloo) moves each rank's per-peer messages to the offsets
    the receivers' layout names, and all-gathers the batch summaries in rank order -- driven through the same ctypes
    function pointers the library calls (the GPU suite runs it inside real multi-rank domains)."""
    import torch.multiprocessing as mp
    errfile = str(tmp_path / 'err.txt')
    world = tiles[0] * tiles[1]
    mp.start_processes(_hosted_worker, args=(world, _free_port(), tiles, errfile), nprocs=world, join=True,
                       start_method='spawn')
    assert not os.path.exists(errfile), open(errfile).read()
