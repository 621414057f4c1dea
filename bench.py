"""Benchmark of the hot path: L=4096 Villain NeighborhoodUpdate sweeps (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--L 4096]

A "step" is one NeighborhoodUpdate sweep (neighborhood.py:59-137) of the whole L x L lattice, in the
reference's own chain semantics (NumPy PCG64 stream replayed on the device, bit-exact parity mode),
with the fields resident in HBM.  One process per GPU (torch.distributed.run for N>1); each rank runs
its own L x L chain (seed = rank): weak scaling, no data-path collective (Multi-GPU).
Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ALG_BYTES_PER_SITE = 48      # one read + one write of phi (f64) and n (2 x i64) per sweep
SURVEY_BYTES_PER_SITE = 88   # two separate colour passes
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--L', type=int, default=4096)
    ap.add_argument('--kappa', type=float, default=0.5)
    ap.add_argument('--W', type=int, default=1)
    ap.add_argument('--path', type=int, default=2, help='0 auto, 1 per-colour kernels, 2 fused sweep kernel')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sweeps', type=int, default=5)
    return ap.parse_args()


def traffic_from_profiles(L):
    """HBM bytes per launch of the fused kernel from a committed rocprofv3 --pmc summary, if any."""
    path = os.path.join(ROOT, 'profiles', 'pmc_summary.json')
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f'villain_sweep_fused_L{L}')
        return None if e is None else float(e['hbm_bytes_per_launch'])
    except Exception:
        return None


def cpu_baseline(L, kappa, W, sweeps):
    """The CPU oracle (C restatement of the reference path, 1 core) on a bounded sample of the same
    workload.  Test infrastructure used only as the reported baseline."""
    from oracle import oracle as O
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    g = np.random.default_rng(0)
    O.villain_neighborhood(L, kappa, W, phi, n, 1, g)  # warm
    t = time.perf_counter()
    O.villain_neighborhood(L, kappa, W, phi, n, sweeps, g)
    dt = time.perf_counter() - t
    return {'value': sweeps * L * L / dt, 'unit': 'lattice-site updates/s', 'cores': 1, 'kind': 'port',
            'sample': f'{sweeps} sweeps of L={L} Villain NeighborhoodUpdate (kappa={kappa}, W={W}), cold start, '
                      'oracle/sv_oracle.c single-threaded'}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('gloo', rank=rank, world_size=world)

    from supervillain_amd import _native
    from supervillain_amd._abi import SvRng, rng_from_numpy

    Lib = _native.lib()
    ctx = _native.context(local)
    L = args.L
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'sv_villain_create')
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
    r = rng_from_numpy(np.random.default_rng(rank))

    def run(k):
        st = _native.stats_array(k)
        ctx.check(Lib.sv_villain_run(h, args.kappa, args.W, float(np.pi), 1, k, ctypes.byref(r), st, args.path),
                  'sv_villain_run')
        return st

    if args.warmup:
        run(args.warmup)
    Lib.sv_ctx_set_timing(ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    st = run(args.steps)  # synchronous on return (stream synchronized)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    ms = ctypes.c_double()
    launches = ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(launches))
    Lib.sv_ctx_set_timing(ctx.handle, 0)
    acc = sum(st[i].accepted for i in range(args.steps)) / (args.steps * L * L)
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        value = world * args.steps * L * L / elapsed
        avg_launch_s = ms.value / 1e3 / max(launches.value, 1)
        achieved = ALG_BYTES_PER_SITE * L * L / avg_launch_s / 1e9
        traffic = traffic_from_profiles(L)
        out = {
            'metric': 'lattice-site updates/sec (sweeps/s × L²), L=4096 Villain, 1→8 MI355X',
            'value': value,
            'unit': 'lattice-site updates/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f64+int64',
            'data': 'synthetic (cold start, NumPy PCG64 seed = rank)',
            'config': {'workload': f'L={L} Villain NeighborhoodUpdate sweep, kappa={args.kappa}, W={args.W}, '
                                   'bit-exact reference chain (PCG64 replay), fused two-colour sweep kernel',
                       'L': L, 'kappa': args.kappa, 'W': args.W, 'path': args.path,
                       'parallelism': f'{world} independent chains (one per GPU)',
                       'acceptance_rate': acc},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'kernel': 'villain_sweep_fused', 'avg_launch_us': avg_launch_s * 1e6,
                         'alg_bytes_per_site': ALG_BYTES_PER_SITE,
                         'survey_effective_GBps': SURVEY_BYTES_PER_SITE * L * L / avg_launch_s / 1e9},
            'cpu_baseline': None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(L, args.kappa, args.W, args.cpu_sweeps)
        print(json.dumps(out), flush=True)
    Lib.sv_villain_destroy(h)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
