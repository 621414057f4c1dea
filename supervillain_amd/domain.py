"""Villain NeighborhoodUpdate, and the Worldline Plaquette + Coexact step, on a domain-decomposed lattice
(multi-GPU; SURVEY.md 8e, BASELINE configs 4 and 3).

The reference runs one lattice in one process (generator/villain/neighborhood.py:59-137); this is the
same chain with the lattice cut into tiles (sv_domain_* in include/supervillain_amd.h).  One rank per
GPU owns one tile; halos travel over RCCL inside libsvhip.so.  With a single rank every tile lives on
one GPU -- the same code path minus RCCL, which is how the decomposition is checked bit-for-bit.

    dom = VillainDomain(4096, 8192, tiles=(1, 2), kappa=0.5)            # one GPU, two tiles
    dom = VillainDomain.distributed(8192, 16384, tiles=(2, 4), kappa=0.5)  # one rank per GPU
    dom.upload(phi, n)      # or dom.cold()
    stats = dom.run(100, rng)   # rng: numpy Generator(PCG64), advanced exactly as the reference would
"""
import ctypes

import numpy as np

from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy

UNIQUE_ID_BYTES = 128


def tile_grid(nranks):
    """Tile grid (tiles_t, tiles_x) for n ranks: 1x1, 1x2, 2x2, 2x4, ... (x gets the larger factor)."""
    if nranks < 1:
        raise ValueError('nranks must be >= 1')
    t = int(np.floor(np.sqrt(nranks)))
    while nranks % t:
        t -= 1
    return t, nranks // t


GHOSTS = {'villain': (2, 3, 2, 3), 'worldline': (5, 4, 5, 4)}  # ghost rows above / below, columns left / right


def exchange_plan(Nt, Nx, tiles, rank, model='villain'):
    """The halo messages of tile `rank` as computed by libsvhip.so (host-only; no GPU needed), for a Villain or a
    Worldline decomposition (their ghost frames differ: GHOSTS).

    Returns a list of 8 dicts in send order: dy, dx, send_to, src (row0, col0), shape (rows, cols),
    recv_from, dst (row0, col0) -- tile-local coordinates, ghosts outside [0, Ht) x [0, Wt)."""
    out = (ctypes.c_int64 * 80)()
    fn = _native.lib().sv_domain_exchange_plan_worldline if model == 'worldline' else _native.lib().sv_domain_exchange_plan
    rc = fn(int(Nt), int(Nx), int(tiles[0]), int(tiles[1]), int(rank), out)
    if rc != 0:
        raise ValueError(f'invalid decomposition {Nt}x{Nx} into {tiles} (rank {rank})')
    plan = []
    for s in range(8):
        o = [int(v) for v in out[10 * s:10 * s + 10]]
        plan.append({'dy': o[0], 'dx': o[1], 'send_to': o[2], 'src': (o[3], o[4]), 'shape': (o[5], o[6]),
                     'recv_from': o[7], 'dst': (o[8], o[9])})
    return plan


def ghost_frame(Nt, Nx, tiles, model='villain'):
    """(rows above, below, columns left, right) of the ghost frame libsvhip.so gives this decomposition: GHOSTS for
    the Worldline and for Villain at depth 1, K times the Villain frame when K sweeps run per halo exchange (deep
    halos, SV_DOMAIN_DEPTH).  Read off the exchange plan: the message toward (dy, dx) = (1, 0) fills
    the receiver's rows above, and so on."""
    plan = exchange_plan(Nt, Nx, tiles, 0, model)
    shape = {(m['dy'], m['dx']): m['shape'] for m in plan}
    return shape[(1, 0)][0], shape[(-1, 0)][0], shape[(0, 1)][1], shape[(0, -1)][1]


def message_layout(Nt, Nx, tiles, rank, model='villain'):
    """The RCCL message layout libsvhip.so uses for `rank` when every tile is a rank (host-only).

    Returns dict: sends / recvs = [(peer, offset, words)], soff / roff = per-direction word offsets of
    message s in the send / receive buffer, words = per-direction message size, msg_words = buffer size."""
    out = (ctypes.c_int64 * 128)()
    fn = (_native.lib().sv_domain_message_layout_worldline if model == 'worldline'
          else _native.lib().sv_domain_message_layout)
    rc = fn(int(Nt), int(Nx), int(tiles[0]), int(tiles[1]), int(rank), out)
    if rc != 0:
        raise ValueError(f'invalid decomposition {Nt}x{Nx} into {tiles} (rank {rank})')
    o = [int(v) for v in out]
    ns, nr = o[0], o[1]
    p = 2
    sends = [tuple(o[p + 3 * i:p + 3 * i + 3]) for i in range(ns)]
    p += 3 * ns
    recvs = [tuple(o[p + 3 * i:p + 3 * i + 3]) for i in range(nr)]
    p += 3 * nr
    return {'sends': sends, 'recvs': recvs, 'soff': o[p:p + 8], 'roff': o[p + 8:p + 16],
            'words': o[p + 16:p + 24], 'msg_words': o[p + 24]}


class HostTransport:
    """The two collectives of a multi-rank domain carried by torch.distributed on host memory instead of RCCL
    (sv_domain_create_hosted): the halo messages as one isend / irecv per distinct peer, the batch summaries as an
    all_gather.  Any backend that moves CPU tensors will do (gloo).  For checking the multi-rank protocol where RCCL
    cannot run -- two ranks on one GPU -- not for speed.  Default process group only (peers are its ranks)."""

    def __init__(self):
        import torch
        import torch.distributed as dist
        self._torch, self._dist = torch, dist
        self.error = None  # the first exception a callback met (the library then fails the run)
        self.xfer = _native.XFER_FN(self._xfer)
        self.gather = _native.GATHER_FN(self._gather)

    def _xfer(self, user, nsend, sends, sendbuf, nrecv, recvs, recvbuf):
        try:
            torch, dist = self._torch, self._dist
            reqs, landed = [], []
            for i in range(nsend):
                peer, off, words = sends[3 * i], sends[3 * i + 1], sends[3 * i + 2]
                msg = np.frombuffer((ctypes.c_int64 * words).from_address(sendbuf + 8 * off), dtype=np.int64).copy()
                reqs.append(dist.isend(torch.from_numpy(msg), dst=int(peer)))
            for i in range(nrecv):
                peer, off, words = recvs[3 * i], recvs[3 * i + 1], recvs[3 * i + 2]
                t = torch.empty(int(words), dtype=torch.int64)
                reqs.append(dist.irecv(t, src=int(peer)))
                landed.append((off, words, t))
            for r in reqs:
                r.wait()
            for off, words, t in landed:
                ctypes.memmove(recvbuf + 8 * off, t.numpy().ctypes.data, 8 * words)
            return 0
        except Exception as e:  # (an exception cannot cross the C frames: report it, fail the run)
            self.error = self.error or e
            return 1

    def _gather(self, user, local, out, nbytes):
        try:
            torch, dist = self._torch, self._dist
            mine = torch.from_numpy(np.frombuffer((ctypes.c_uint8 * nbytes).from_address(local), dtype=np.uint8).copy())
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(dist.get_world_size())]
            dist.all_gather(parts, mine)
            for r, t in enumerate(parts):
                ctypes.memmove(out + r * nbytes, t.numpy().ctypes.data, nbytes)
            return 0
        except Exception as e:
            self.error = self.error or e
            return 1


class VillainDomain:
    """An Nt x Nx Villain (phi, n) state cut into tiles, resident in HBM."""
    _model = 0  # sv_domain_create_hosted's model

    def __init__(self, Nt, Nx=None, tiles=(1, 1), kappa=0.5, W=1, interval_phi=np.pi, interval_n=1, *,
                 device=None, nranks=1, rank=0, unique_id=None, transport=None):
        Nx = Nt if Nx is None else Nx
        self.Nt, self.Nx, self.tiles = int(Nt), int(Nx), (int(tiles[0]), int(tiles[1]))
        self.kappa, self.W, self.interval_phi, self.interval_n = float(kappa), int(W), float(interval_phi), int(interval_n)
        self.nranks, self.rank = int(nranks), int(rank)
        self.ctx = _native.context(_native.default_device() if device is None else device)
        self._create(unique_id, transport, 'sv_domain_create')

    def _create(self, unique_id, transport, name):
        h = ctypes.c_void_p()
        self._transport = transport  # (the callbacks must outlive the domain)
        if transport is not None:
            rc = _native.lib().sv_domain_create_hosted(self.ctx.handle, self._model, self.Nt, self.Nx, self.tiles[0],
                                                       self.tiles[1], self.nranks, self.rank, transport.xfer,
                                                       transport.gather, None, ctypes.byref(h))
            self.ctx.check(rc, 'sv_domain_create_hosted')
        else:
            uid = None
            if unique_id is not None:
                uid = (ctypes.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(bytes(unique_id))
            self.ctx.check(getattr(_native.lib(), name)(self.ctx.handle, self.Nt, self.Nx, self.tiles[0], self.tiles[1],
                                                        self.nranks, self.rank, uid, ctypes.byref(h)), name)
        self.handle = h

    def _check_run(self, rc, name):
        t = getattr(self, '_transport', None)
        if rc != 0 and t is not None and t.error is not None:
            raise _native.NativeError(f'{name}: the host transport failed: {t.error!r}') from t.error
        self.ctx.check(rc, name)

    @classmethod
    def distributed(cls, Nt, Nx=None, tiles=None, group=None, transport='rccl', **kw):
        """One tile per rank of the (already initialised) default torch.distributed group.  transport='rccl': halos
        over RCCL (any backend for the group: gloo is enough, it only carries the 128-byte RCCL id); 'host': both
        collectives over the group itself through host memory (HostTransport; default group only)."""
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        tiles = tile_grid(world) if tiles is None else tiles
        if transport == 'host':
            if group is not None:
                raise ValueError('the host transport runs on the default process group')
            return cls(Nt, Nx, tiles, nranks=world, rank=rank, transport=HostTransport(), **kw)
        if transport != 'rccl':
            raise ValueError(f"transport must be 'rccl' or 'host', not {transport!r}")
        box = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        return cls(Nt, Nx, tiles, nranks=world, rank=rank, unique_id=box[0], **kw)

    def close(self, _in_del=False):
        if getattr(self, 'handle', None) is not None and _native._LIB is not None:
            h, self.handle = self.handle, None
            _native.destroy(_native._LIB.sv_domain_destroy, h, 'sv_domain_destroy (' + type(self).__name__ + ')',
                            self.ctx, _in_del)

    def __del__(self):
        self.close(_in_del=True)

    def cold(self):
        self.ctx.check(_native.lib().sv_domain_upload(self.handle, None, None), 'sv_domain_upload')

    def upload(self, phi, n):
        phi = np.ascontiguousarray(phi, dtype=np.float64).reshape(self.Nt, self.Nx)
        n = np.ascontiguousarray(n, dtype=np.int64).reshape(2, self.Nt, self.Nx)
        self.ctx.check(_native.lib().sv_domain_upload(self.handle, _native.ptr(phi), _native.ptr(n)), 'sv_domain_upload')

    def download(self, phi=None, n=None):
        """Copy this rank's tiles into global (Nt, Nx) arrays (other ranks' regions are left as given)."""
        phi = np.zeros((self.Nt, self.Nx)) if phi is None else phi
        n = np.zeros((2, self.Nt, self.Nx), dtype=np.int64) if n is None else n
        self.ctx.check(_native.lib().sv_domain_download(self.handle, _native.ptr(phi), _native.ptr(n)),
                       'sv_domain_download')
        return phi, n

    def run(self, sweeps, rng):
        """`sweeps` NeighborhoodUpdate sweeps; advances `rng` (NumPy Generator) like the reference.
        Collective when nranks > 1.  Returns per-sweep global stats."""
        r = rng_from_numpy(rng)
        st = _native.stats_array(max(sweeps, 1))
        self._check_run(_native.lib().sv_domain_run(self.handle, self.kappa, self.W, self.interval_phi, self.interval_n,
                                                    int(sweeps), ctypes.byref(r), st), 'sv_domain_run')
        rng_to_numpy(r, rng)
        return [st[i] for i in range(sweeps)]


class WorldlineDomain(VillainDomain):
    """An Nt x Nx Worldline (m, v) state cut into tiles: one step = the checkerboard PlaquetteUpdate sweep and
    the CoexactUpdate sweep of sv_worldline_plaquette_coexact_run (the config-3 step), one halo exchange per
    step (sv_domain_*_worldline).  Integer v; W a power of two."""

    _model = 1

    def __init__(self, Nt, Nx=None, tiles=(1, 1), kappa=0.5, W=1, interval_t=1, *, device=None, nranks=1, rank=0,
                 unique_id=None, transport=None):
        Nx = Nt if Nx is None else Nx
        self.Nt, self.Nx, self.tiles = int(Nt), int(Nx), (int(tiles[0]), int(tiles[1]))
        self.kappa, self.W, self.interval_t = float(kappa), float(W), int(interval_t)
        self.nranks, self.rank = int(nranks), int(rank)
        self.ctx = _native.context(_native.default_device() if device is None else device)
        self._create(unique_id, transport, 'sv_domain_create_worldline')

    def cold(self):
        self.ctx.check(_native.lib().sv_domain_upload_worldline(self.handle, None, None), 'sv_domain_upload_worldline')

    def upload(self, m, v):
        m = np.ascontiguousarray(m, dtype=np.int64).reshape(2, self.Nt, self.Nx)
        v = np.ascontiguousarray(v, dtype=np.int64).reshape(self.Nt, self.Nx)
        self.ctx.check(_native.lib().sv_domain_upload_worldline(self.handle, _native.ptr(m), _native.ptr(v)),
                       'sv_domain_upload_worldline')

    def download(self, m=None, v=None):
        m = np.zeros((2, self.Nt, self.Nx), dtype=np.int64) if m is None else m
        v = np.zeros((self.Nt, self.Nx), dtype=np.int64) if v is None else v
        self.ctx.check(_native.lib().sv_domain_download_worldline(self.handle, _native.ptr(m), _native.ptr(v)),
                       'sv_domain_download_worldline')
        return m, v

    def run(self, steps, rng):
        """`steps` Plaquette + Coexact steps; advances `rng` like the reference's shared Generator.  Returns
        2 * steps global stats ({Plaquette, Coexact} per step)."""
        r = rng_from_numpy(rng)
        st = _native.stats_array(max(2 * steps, 1))
        self._check_run(_native.lib().sv_domain_run_worldline(self.handle, self.kappa, self.W, self.interval_t,
                                                              int(steps), ctypes.byref(r), st),
                        'sv_domain_run_worldline')
        rng_to_numpy(r, rng)
        return [st[i] for i in range(2 * steps)]


def unique_id():
    """A fresh RCCL unique id (bytes), to be created on rank 0 and shared with every rank."""
    buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    if _native.lib().sv_domain_unique_id(buf) != 0:
        raise _native.NativeError('ncclGetUniqueId failed')
    return bytes(buf)
