"""Benchmark of the hot path: L=4096 Villain NeighborhoodUpdate sweeps (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--L 4096]

A "step" is one NeighborhoodUpdate sweep (neighborhood.py:59-137) of the whole lattice, in the
reference's own chain semantics (NumPy PCG64 stream replayed on the device, bit-exact parity mode),
with the fields resident in HBM.

  N = 1: one L x L lattice on one GPU (the single-lattice fused sweep kernel).
  N > 1: one process per GPU (torch.distributed.run; `python bench.py --gpus N` launches it itself when
         WORLD_SIZE is unset, before anything touches a GPU).  BASELINE config 4 (the default): the ONE L x L
         lattice the metric names (L=4096) cut into ty x tx tiles (1x2, 2x2, 2x4 for N = 2, 4, 8), one per GPU,
         with RCCL halo exchanges (strong scaling; the chain is bit-identical to the 1-GPU chain).  --weak: an
         L x L tile per GPU of a (ty L) x (tx L) lattice instead (north_star's weak-scaling efficiency), and the
         metric names that lattice.  --tiles TYxTX on one GPU emulates a decomposition.
         Every domain line also carries, under config.scaling_reference, rates timed after the same warm-up as
         the main run (warm_up: W steps, then --warmup-s seconds) over max(--steps, 100) sweeps: R1 = this rank's
         tile alone as a periodic lattice (E_N = R_N / (N R1)), and the single-lattice headline
         path on one L x L lattice (the N = 1 line's kernel: for --weak the per-GPU R1, for strong the 1-GPU
         rate of the whole problem).  An E_N above 1.02 is flagged (E_N_suspect) and printed to stderr.
Rank 0 prints one JSON line.

Secondary workloads (not the headline line; BASELINE.json configs 5 and 3):
  --workload replicas   1024 independent L=128 Villain chains, W=2, inline observables, split over
                        the N ranks (config 5; replicas need no collectives)
  --workload worldline  L=1024 Worldline: one checkerboard PlaquetteUpdate + one CoexactUpdate sweep
                        per step, W=1 (config 3); N > 1 (or --tiles) decomposes the lattice into tiles, one per
                        GPU, with a (v, m) halo exchange per step
  --workload site|link|exact|cohomology|hammer
                        SURVEY.md 8(f) rows at L=4096: one sweep of SiteUpdate / LinkUpdate / ExactUpdate /
                        CohomologyUpdate per step, or one Villain Hammer step (Site, Link, Exact, Cohomology,
                        each with its own stream, as the reference's Hammer minus its worm); device-resident
                        fields; N > 1 runs independent chains
  --workload worms      SURVEY.md 8(f) row 4: 1024 independent L=128 Villain chains (W=2, config-5 shape),
                        thermalized by 100 NeighborhoodUpdate sweeps, then one ClassicWorm per chain per
                        step (one GPU lane per chain); reported as worm moves/s over all chains
  --workload vortex|wrapping|wlhammer
                        the same for the Worldline rows: VortexUpdate, WrappingUpdate, or one Worldline
                        Hammer step (Vortex, Coexact, Wrapping) at L=4096, W=1
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

# roofline.achieved uses SURVEY.md 8(d)'s algorithmic bytes per unit (the task's definition): 88 B per Villain
# site-update (two colour passes at the reference dtypes).  The fused kernel's own compulsory traffic -- one read
# and one write of phi (f64) and n (2 x i64) per sweep, 48 B -- is reported beside it (fused_min_*).
SURVEY_BYTES_PER_SITE = 88
FUSED_MIN_BYTES_PER_SITE = 48
WORLDLINE_BYTES = 168        # Plaquette (88) + Coexact (80) per plaquette-step
# SURVEY.md 8(f) rows, compulsory HBM bytes per site and sweep: Site reads phi and n and
# writes phi (8 + 16 + 8); Exact reads phi and n and writes n (8 + 16 + 16); Link the same per site
# (2 links); Cohomology touches 2 N links (reported per site of the slice sum, not a roofline workload)
LOCAL_BYTES = {'site': 32, 'exact': 40, 'link': 40, 'hammer': 32 + 40 + 40,
               # Worldline: Vortex reads m and v and writes v (16 + 8 + 8); Wrapping reads m and v (16 + 8);
               # the Worldline Hammer adds Coexact's 80
               'vortex': 32, 'wrapping': 24, 'wlhammer': 32 + 80 + 24}
WORLDLINE_KINDS = ('vortex', 'wrapping', 'wlhammer')
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='number of GPUs (ranks); N > 1 without WORLD_SIZE launches torch.distributed.run itself')
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--L', type=int, default=4096)
    ap.add_argument('--kappa', type=float, default=0.5)
    ap.add_argument('--W', type=int, default=1)
    ap.add_argument('--path', type=int, default=2, help='0 auto, 1 per-colour kernels, 2 fused sweep kernel')
    ap.add_argument('--rng', default='pcg64', choices=['pcg64', 'philox'],
                    help='villain workload: pcg64 = the reference chain (NumPy stream replay, the headline); philox = '
                         'the optional counter-based mode (SURVEY.md 8(b) sv_rng mode 1, a different chain)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sweeps', type=int, default=5)
    ap.add_argument('--weak', action='store_true', help='an L x L tile per GPU of a (ty L) x (tx L) lattice (weak '
                                                        'scaling; with --tiles on one GPU, emulate that layout); the '
                                                        'metric then names that lattice')
    ap.add_argument('--strong', action='store_true', help='(the default) one L x L lattice decomposed over the N GPUs '
                                                          '(BASELINE config 4, strong scaling)')
    ap.add_argument('--warmup-s', type=float, default=1.0,
                    help='after the W warmup steps, keep warming (untimed) until this many seconds have passed: '
                         'clocks and page mappings reach steady state before the timed region')
    ap.add_argument('--no-copy-ceiling', action='store_true', help='skip the measured copy-kernel HBM ceiling')
    ap.add_argument('--tiles', default=None, help='tile grid TYxTX (default from N); with N=1 emulates the '
                                                   'decomposition on one GPU')
    ap.add_argument('--transport', default='rccl', choices=['rccl', 'host'],
                    help="N > 1 domain lines: halos over RCCL (the default), or 'host' (sv_domain_create_hosted over the "
                         'gloo group: a rehearsal of the N-rank path where RCCL cannot run, e.g. N ranks on one GPU '
                         'with SV_DEVICE=0; not a performance line)')
    ap.add_argument('--workload', default='villain', choices=['villain', 'replicas', 'worldline', 'site', 'link', 'exact',
                                                              'cohomology', 'hammer', 'vortex', 'wrapping', 'wlhammer',
                                                              'worms', 'ranks'])
    ap.add_argument('--event-timing', default='batch', choices=['launch', 'batch'],
                    help='hipEvents around each batch of 64 fused launches (default) or around every launch')
    ap.add_argument('--plaquette', default='checkerboard', choices=['checkerboard', 'reference'],
                    help='worldline workload: the checkerboard Plaquette chain (one fused launch per step) or the '
                         'bit-exact reference visit order (plaquette.py:63; level-scheduled)')
    ap.add_argument('--replicas', type=int, default=1024, help='replicas workload: total replica count')
    ap.add_argument('--streams', type=int, default=None, help='replicas workload: part-batches on their own HIP '
                                                              'streams (default: VillainReplicas\' choice, 2 from 256)')
    args = ap.parse_args()
    if args.strong and args.weak:
        ap.error('--strong and --weak exclude each other')
    # BASELINE config 4 (one L x L lattice over the GPUs, strong scaling) unless --weak
    args.strong = not args.weak
    if args.workload in ('replicas', 'worms'):
        args.L = 128 if args.L == 4096 else args.L
        args.W = 2 if args.W == 1 else args.W
    if args.workload == 'worldline':
        args.L = 1024 if args.L == 4096 else args.L
    return args


def traffic_from_profiles(L):
    """HBM bytes per launch of the fused kernel from a committed rocprofv3 --pmc summary, if any."""
    path = os.path.join(ROOT, 'profiles', 'pmc_summary.json')
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(f'villain_sweep_hot_L{L}') or d.get(f'villain_sweep_fused_L{L}')
        return None if e is None else float(e['hbm_bytes_per_launch'])
    except Exception:
        return None


def cpu_baseline(L, kappa, W, sweeps):
    """The CPU oracle (C restatement of the reference path) on a bounded sample of the same workload, on all
    of this process's host cores (OpenMP: jump-ahead draws + parallel per-site work, the same chain) and on
    one core.  Test infrastructure used only as the reported baseline."""
    from oracle import oracle as O
    cores = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or min(16, os.cpu_count() or 1)
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    g = np.random.default_rng(0)
    O.villain_neighborhood_mt(L, kappa, W, phi, n, 1, g, cores)  # warm
    t = time.perf_counter()
    O.villain_neighborhood_mt(L, kappa, W, phi, n, sweeps, g, cores)
    dt_mt = time.perf_counter() - t
    t = time.perf_counter()
    O.villain_neighborhood(L, kappa, W, phi, n, sweeps, g)
    dt_1 = time.perf_counter() - t
    return {'value': sweeps * L * L / dt_mt, 'unit': 'lattice-site updates/s', 'cores': cores, 'kind': 'port',
            'value_1core': sweeps * L * L / dt_1,
            'sample': f'{sweeps} sweeps of L={L} Villain NeighborhoodUpdate (kappa={kappa}, W={W}) on {cores} '
                      f'OpenMP threads (oracle/sv_oracle.c sv_o_villain_neighborhood_mt), then {sweeps} more on '
                      '1 core (the sequential restatement: value_1core)'}


def warm_up(run, args, dist=None):
    """Untimed warmup: the W steps the driver asks for, then more until --warmup-s seconds have passed (GPU
    clocks and page mappings at steady state).  Collective runs agree on the extra step count (max over ranks)."""
    t0 = time.perf_counter()
    if args.warmup:
        run(args.warmup)
    if args.warmup_s <= 0:
        return
    t1 = time.perf_counter()
    run(1)
    per = max(time.perf_counter() - t1, 1e-6)
    extra = int(max(0.0, args.warmup_s - (time.perf_counter() - t0)) / per) if args.warmup_s > 0 else 0
    extra = int(max_over_ranks(dist, float(min(extra, 100000))))
    while extra > 0:
        k = min(extra, 4096)
        run(k)
        extra -= k


def copy_ceiling(ctx):
    """Measured HBM ceiling on this GPU: a streaming copy of two 1 GiB buffers (16-B lanes), read + write bytes
    per second (report the roofline fraction against it as well as against the 8 TB/s spec)."""
    from supervillain_amd import _native
    g = ctypes.c_double()
    if _native.lib().sv_hbm_copy(ctx.handle, 1 << 30, 16, 20, ctypes.byref(g)) != 0:
        return None
    return g.value


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def kernel_time(Lib, ctx):
    ms = ctypes.c_double()
    launches = ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(launches))
    Lib.sv_ctx_set_timing(ctx.handle, 0)
    return ms.value / 1e3 / max(launches.value, 1)


HEADLINE_METRIC = 'lattice-site updates/sec (sweeps/s × L²), L=4096 Villain, 1→8 MI355X'  # BASELINE.json


def lattice_metric(Nt, Nx, model='Villain', weak_tile=None,
                   head='lattice-site updates/sec (sweeps/s × L²)', tail=', 1→8 MI355X'):
    """The metric string of a line, naming the lattice it actually sweeps: BASELINE.json's metric verbatim for one
    4096 x 4096 Villain lattice (the N = 1 headline and config 4's tiles of it), the same words with `L=N` for another
    square lattice, and `NtxNx` (plus the per-GPU tile) for the weak-scaled lattices."""
    if Nt == Nx and weak_tile is None:
        return f'{head}, L={Nt} {model}{tail}'
    what = f'{Nt}x{Nx} {model}'
    if weak_tile is not None:
        what += f' (weak scaling: one {weak_tile[0]}x{weak_tile[1]} tile per GPU)'
    return f'{head.replace("L²", "Nt·Nx")}, {what}{tail}'


def metric_lattice(metric):
    """(Nt, Nx) named by a metric string (`L=N <model>` or `NtxNx <model>`), or None."""
    import re
    m = re.search(r'L=(\d+) (?:Villain|Worldline)', metric)
    if m:
        return int(m.group(1)), int(m.group(1))
    m = re.search(r'(\d+)x(\d+) (?:Villain|Worldline)', metric)
    return (int(m.group(1)), int(m.group(2))) if m else None


def report(args, world, sites_per_step, sites_per_launch, elapsed, acc, avg_launch_s, config, traffic_L,
           metric=HEADLINE_METRIC,
           unit='lattice-site updates/s', kernel='villain_sweep_hot', alg_bytes=SURVEY_BYTES_PER_SITE,
           min_bytes=FUSED_MIN_BYTES_PER_SITE, baseline=None, ctx=None, scaling=None):
    timing_source = 'hipEvents around the sweep launches'
    if not avg_launch_s or avg_launch_s <= 0:
        # no timed launch survived (every timed segment ended behind a NumPy Lemire rejection's abort): the roofline
        # falls back to the wall-clock time per step, an upper bound on the kernel's
        avg_launch_s = elapsed / max(args.steps, 1)
        timing_source = 'wall clock per step (no timed launch survived the rejections)'
    achieved = alg_bytes * sites_per_launch / avg_launch_s / 1e9
    lat = config.get('lattice')
    named = metric_lattice(metric)
    if lat is not None and named is not None and tuple(lat) != named:
        raise ValueError(f'bench.py: the metric names a {named[0]}x{named[1]} lattice but the run swept '
                         f'{lat[0]}x{lat[1]}: {metric}')
    ceiling = copy_ceiling(ctx) if ctx is not None and not getattr(args, 'no_copy_ceiling', False) else None
    out = {
        'metric': metric,
        'value': args.steps * sites_per_step / elapsed,
        'unit': unit,
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': scaling or ('strong' if args.strong else 'weak'),
        'vs_baseline': None,
        'dtype': 'f64+int64',
        'data': 'synthetic (cold start, NumPy PCG64 seed 0)',
        'config': dict(config, kappa=args.kappa, W=args.W, acceptance_rate=acc),
        'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': achieved / HBM_PEAK_GBS,
                     'traffic': traffic_from_profiles(traffic_L) if kernel == 'villain_sweep_hot' else None,
                     # (PMC counters cannot be read inside this process: they come from scripts/profile.sh's separate
                     # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same command, per the guide's gfx950
                     # corrections, folded into profiles/pmc_summary.json)
                     'traffic_source': 'profiles/pmc_summary.json (rocprofv3 --pmc passes of this command, '
                                       'scripts/profile.sh)' if kernel == 'villain_sweep_hot' else None,
                     'kernel': kernel, 'avg_launch_us': avg_launch_s * 1e6, 'launch_time_source': timing_source,
                     'alg_bytes_per_unit': alg_bytes,
                     'fused_min_bytes_per_unit': min_bytes,
                     'fused_min_GBps': min_bytes * sites_per_launch / avg_launch_s / 1e9,
                     'fused_min_frac': min_bytes * sites_per_launch / avg_launch_s / 1e9 / HBM_PEAK_GBS,
                     'copy_ceiling_GBps': ceiling,
                     'frac_of_copy_ceiling': achieved / ceiling if ceiling else None},
        'cpu_baseline': None,
    }
    if world == 1 and not args.no_cpu_baseline:
        out['cpu_baseline'] = (baseline or (lambda: cpu_baseline(args.L, args.kappa, args.W, args.cpu_sweeps)))()
    print(json.dumps(out), flush=True)


def run_replicas(args, world, rank, dist):
    """BASELINE config 5: independent L x L replica chains (seed = global replica index), W=2, inline
    observables fused into the sweep kernel; the replicas are split over the ranks, no collective."""
    from supervillain_amd import _native
    from supervillain_amd.replicas import VillainReplicas
    L, Rt = args.L, args.replicas
    per = Rt // world
    first = rank * per
    B = VillainReplicas(per, L, args.kappa, args.W, streams=args.streams)
    B.cold()
    gens = [np.random.default_rng(first + r) for r in range(per)]
    Lib = _native.lib()
    warm_up(lambda k: B.run(k, gens, inline=True), args, dist)
    for c in B.contexts:
        Lib.sv_ctx_set_timing(c.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    stats, obs = B.run(args.steps, gens, inline=True)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    # each part-batch's launches are timed on its own stream: the mean launch duration over the streams
    ms_tot, n_tot = 0.0, 0
    for c in B.contexts:
        ms, nl = ctypes.c_double(), ctypes.c_int64()
        Lib.sv_ctx_kernel_time(c.handle, ctypes.byref(ms), ctypes.byref(nl))
        Lib.sv_ctx_set_timing(c.handle, 0)
        ms_tot, n_tot = ms_tot + ms.value, n_tot + nl.value
    launches_s = ms_tot / 1e3 / max(n_tot, 1)
    nparts = len(B.contexts)
    acc = float(stats['accepted'].sum()) / (args.steps * per * L * L)

    def baseline():
        from oracle import oracle as O
        sweeps, n = 20, 8
        t = time.perf_counter()
        for r in range(n):
            phi, nn = np.zeros((L, L)), np.zeros((2, L, L), dtype=np.int64)
            O.villain_neighborhood(L, args.kappa, args.W, phi, nn, sweeps, np.random.default_rng(r))
        dt = time.perf_counter() - t
        return {'value': n * sweeps * L * L / dt, 'unit': 'replica-site updates/s', 'cores': 1, 'kind': 'port',
                'sample': f'{n} replicas x {sweeps} sweeps of L={L} Villain NeighborhoodUpdate (W={args.W}), '
                          'oracle/sv_oracle.c single-threaded (no observables)'}

    if rank == 0:
        config = {'workload': f'{Rt} independent L={L} Villain NeighborhoodUpdate replica chains (W={args.W}), '
                              'inline ActionDensity/InternalEnergyDensity/WindingSquared/TorusWrapping, '
                              f'{per} replicas per GPU as {nparts} part-batch(es) on {nparts} HIP stream(s) (bit-identical '
                              'to one batch), one full-row villain_sweep_hot_fr launch per sweep and part (two when a '
                              'known NumPy Lemire rejection splits off the replicas that replay it)',
                  'L': L, 'replicas': Rt, 'replicas_per_gpu': per, 'path': 'replicas', 'streams': nparts,
                  'parallelism': f'{world} GPU(s), replicas sharded, no collectives',
                  'roofline_note': 'avg_launch_us is the mean duration of one part-batch launch on its own stream; '
                                   f'the {nparts} streams overlap, so the per-launch rate understates the aggregate: '
                                   f'{SURVEY_BYTES_PER_SITE * Rt * L * L * args.steps / elapsed / 1e9 / world:.1f} GB/s '
                                   'per GPU over the wall clock'}
        report(args, world, Rt * L * L, per * L * L // nparts, elapsed, acc, launches_s, config, L,
               metric=f'replica-site updates/sec, {Rt} x L={L} Villain replicas, W={args.W}, inline observables',
               unit='replica-site updates/s', kernel='villain_sweep_hot_fr (obs)', baseline=baseline, ctx=B.ctx,
               scaling='strong')
    B.close()


def run_worms(args, world, rank, dist):
    """batched Villain ClassicWorms (supervillain/generator/villain/worm.py:85-183) on
    config-5-shaped replicas; a step is one worm of every chain, the unit one worm move."""
    from supervillain_amd import _native
    from supervillain_amd.replicas import VillainReplicas
    L, Rt = args.L, args.replicas
    per = Rt // world
    first = rank * per
    B = VillainReplicas(per, L, args.kappa, args.W, streams=1)
    B.cold()
    gens = [np.random.default_rng(first + r) for r in range(per)]
    B.run(100, gens)  # thermalize: worms on a cold start are short
    wgens = [np.random.default_rng(10 ** 6 + first + r) for r in range(per)]
    Lib = _native.lib()
    warm_up(lambda k: B.worm(wgens, worms=k), args, dist)
    Lib.sv_ctx_set_timing(B.ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    _, lengths = B.worm(wgens, worms=args.steps)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    launch_s = kernel_time(Lib, B.ctx)
    moves = float(lengths.sum())
    if dist:
        import torch
        t = torch.tensor([moves], dtype=torch.float64)
        dist.all_reduce(t)
        moves = float(t.item())
    phi, n = B.download() if rank == 0 else (None, None)

    def baseline():
        from oracle import oracle as O
        t, done, k = time.perf_counter(), 0, 0
        while time.perf_counter() - t < 10 and k < per:
            nn = n[k].copy()
            _, l = O.villain_worm(L, args.kappa, args.W, phi[k], nn, 20, np.random.default_rng(7 + k))
            done += int(l.sum())
            k += 1
        dt = time.perf_counter() - t
        return {'value': done / dt, 'unit': 'worm moves/s', 'cores': 1, 'kind': 'port',
                'sample': f'20 worms on each of {k} thermalized L={L} chains (W={args.W}), oracle/sv_oracle.c '
                          'single-threaded'}

    if rank == 0:
        mean_len = moves / (args.steps * Rt)
        config = {'workload': f'{Rt} independent L={L} Villain chains (W={args.W}), one ClassicWorm per chain per '
                              f'step, one GPU lane per chain ({per} per GPU), Vortex_Vortex histogram of the last '
                              'worm, thermalized by 100 NeighborhoodUpdate sweeps',
                  'L': L, 'replicas': Rt, 'replicas_per_gpu': per, 'path': 'worms', 'mean_worm_length': mean_len,
                  'parallelism': f'{world} GPU(s), chains sharded, no collectives'}
        # bytes per move: n of the crossed link + the two phi of d(phi) on it (8 + 16), the conditional n store
        # and the histogram increment (8 + 8); a latency-bound walk, the roofline fraction is informational
        report(args, world, moves / args.steps, moves / world, elapsed, 0.0, launch_s, config, L,
               metric=f'worm moves/sec, {Rt} x L={L} Villain ClassicWorm chains, W={args.W}', unit='worm moves/s',
               kernel='villain_worm', alg_bytes=40, min_bytes=40, baseline=baseline, ctx=B.ctx, scaling='strong')
    B.close()


def run_worldline_domain(args, world, rank, dist):
    """Config 3 decomposed: one L x L Worldline lattice cut into ty x tx tiles (one per GPU;
    --weak: an L x L tile per GPU), one (v, m) halo exchange per Plaquette + Coexact step; R1 = one GPU running
    one periodic tile alone, as for config 4 (timed after the same warm-up, over max(--steps, 100) steps)."""
    from supervillain_amd import _native
    from supervillain_amd.domain import WorldlineDomain, tile_grid
    L = args.L
    if args.tiles:
        ty, tx = (int(v) for v in args.tiles.lower().split('x'))
    else:
        ty, tx = tile_grid(world)
    Nt, Nx = (L, L) if args.strong else (ty * L, tx * L)
    Ht, Wt = Nt // ty, Nx // tx
    kw = dict(kappa=args.kappa, W=args.W)
    dom = (WorldlineDomain.distributed(Nt, Nx, (ty, tx), transport=args.transport, **kw) if world > 1
           else WorldlineDomain(Nt, Nx, (ty, tx), **kw))
    dom.cold()
    gen = np.random.default_rng(0)
    Lib = _native.lib()
    warm_up(lambda k: dom.run(k, gen), args, dist)
    Lib.sv_ctx_set_timing(dom.ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    st = dom.run(args.steps, gen)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    avg_launch_s = kernel_time(Lib, dom.ctx)
    acc = sum(st[2 * i].accepted for i in range(args.steps)) / (args.steps * Nt * Nx)
    rej = sum(s.rejections for s in st)
    ctx = dom.ctx
    dom.close()
    one = WorldlineDomain(Ht, Wt, (1, 1), **kw)
    one.cold()
    g1 = np.random.default_rng(1)
    r1, _ = timed_rate(lambda k: one.run(k, g1), Ht * Wt, args, dist)
    one.close()
    r1_mean = r1 if dist is None else _mean_over_ranks(dist, r1)
    if rank == 0:
        value = args.steps * Nt * Nx / elapsed
        config = {'workload': f'{Nt}x{Nx} Worldline: checkerboard PlaquetteUpdate + CoexactUpdate sweep per step, '
                              f'W={args.W}, kappa={args.kappa}, domain-decomposed into {ty}x{tx} tiles of {Ht}x{Wt} '
                              '(one per GPU), (v, m) halo exchange per step, bit-exact PCG64 replay',
                  'L': L, 'lattice': [Nt, Nx], 'tiles': [ty, tx], 'path': 'worldline-domain',
                  'halo_transport': args.transport if world > 1 else 'none (one process)',
                  'parallelism': f'{ty}x{tx} domain decomposition over {world} GPU(s)',
                  'lemire_rejections_in_timed_steps': int(rej),
                  'scaling_reference': scaling_reference(value, world, r1_mean, [Ht, Wt], None, None, 'steps')}
        report(args, world, Nt * Nx, Nt * Nx // world, elapsed, acc, avg_launch_s, config, Ht,
               metric=lattice_metric(Nt, Nx, 'Worldline', None if args.strong else [Ht, Wt],
                                     head='plaquette-steps/sec (Plaquette + Coexact sweep)', tail=f', W={args.W}'),
               unit='plaquette-steps/s', kernel='worldline_step_fused', alg_bytes=WORLDLINE_BYTES,
               min_bytes=WORLDLINE_BYTES, ctx=ctx)


def run_worldline(args, world, rank, dist):
    """BASELINE config 3: L x L Worldline, one checkerboard PlaquetteUpdate sweep + one CoexactUpdate
    sweep per step (one worldline_step_fused launch), m = v = 0 cold start; N > 1 (or --tiles) decomposes
    the lattice (run_worldline_domain)."""
    if world > 1 or args.tiles:
        return run_worldline_domain(args, world, rank, dist)
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy
    L = args.L
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_worldline_create(ctx.handle, L, 0, ctypes.byref(h)), 'sv_worldline_create')
    m = np.zeros((2, L, L), dtype=np.int64)
    v = np.zeros((L, L), dtype=np.int64)
    ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'sv_worldline_upload')
    r = rng_from_numpy(np.random.default_rng(rank))
    Weff = float(args.W)

    reference = args.plaquette == 'reference'
    # the reference's global-RandomState permutation (plaquette.py:63): a legacy MT19937 state, drawn natively
    from supervillain_amd._abi import SvMT19937
    legacy_key = np.random.RandomState(rank + 1).get_state()
    mt = SvMT19937()
    ctypes.memmove(mt.key, np.ascontiguousarray(legacy_key[1], dtype=np.uint32).ctypes.data, 624 * 4)
    mt.pos = int(legacy_key[2])

    def step(k):
        if not reference:
            st = _native.stats_array(2 * k)  # one call: Sequentially(Plaquette, Coexact) x k on the device
            ctx.check(Lib.sv_worldline_plaquette_coexact_run(h, args.kappa, Weff, 1, k, ctypes.byref(r), st),
                      'sv_worldline_plaquette_coexact_run')
            return sum(st[2 * i].accepted for i in range(k))  # Plaquette acceptances
        # the bit-exact reference order: Sequentially(PlaquetteUpdate in the visit order plaquette.py:63 draws from
        # the legacy global RandomState, CoexactUpdate) x k in one call; the library draws each step's permutation
        # natively from the MT19937 state (sv_mt19937_permutation), pipelined with the device's sweeps
        st = _native.stats_array(2 * k)
        ctx.check(Lib.sv_worldline_plaquette_reference_coexact_run(h, args.kappa, Weff, 1, k, ctypes.byref(mt),
                                                                   ctypes.byref(r), st),
                  'sv_worldline_plaquette_reference_coexact_run')
        return sum(st[2 * i].accepted for i in range(k))

    warm_up(step, args, dist)
    Lib.sv_ctx_set_timing(ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    acc = step(args.steps)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    ms = ctypes.c_double()
    launches = ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(launches))
    step_kernel_s = ms.value / 1e3 / args.steps  # both sweeps' kernels per step (checkerboard)

    def baseline():
        from oracle import oracle as O
        mm, vv = np.zeros((2, L, L), dtype=np.int64), np.zeros((L, L), dtype=np.int64)
        g = np.random.default_rng(0)
        k = 3 if not reference else 2
        lg = np.random.RandomState(1)
        t = time.perf_counter()
        for _ in range(k):
            if reference:
                o = lg.permutation(L * L).astype(np.int64)
                O.worldline_plaquette_seq(L, args.kappa, Weff, mm, vv, o, g)
            else:
                O.worldline_plaquette_cb(L, args.kappa, Weff, mm, vv, 1, g)
            O.worldline_coexact(L, args.kappa, Weff, mm, vv, 1, g)
        dt = time.perf_counter() - t
        return {'value': k * L * L / dt, 'unit': 'plaquette-steps/s', 'cores': 1, 'kind': 'port',
                'sample': f'{k} steps ({"reference-order" if reference else "checkerboard"} Plaquette + Coexact '
                          f'sweep) of L={L} Worldline, oracle/sv_oracle.c single-threaded'}

    if rank == 0:
        if reference:
            config = {'workload': f'L={L} Worldline: reference-order PlaquetteUpdate (the NumPy RandomState visit '
                                  'permutation, plaquette.py:35-104, bit-exact) + CoexactUpdate sweep per step, '
                                  f'W={args.W}, kappa={args.kappa}, PCG64 replay; level-scheduled launches',
                      'L': L, 'lattice': [L, L], 'path': 'worldline-reference-order', 'parallelism': 'single GPU',
                      'visit_order': 'native MT19937 permutation (sv_mt19937_permutation), drawn on host threads while '
                                     'the device runs the previous steps'}
            # no single dominant kernel: the roofline line prices the whole step (both sweeps, 168 B) by its wall time
            step_kernel_s = elapsed / args.steps
        else:
            config = {'workload': f'L={L} Worldline: checkerboard PlaquetteUpdate + CoexactUpdate sweep per step, '
                                  f'W={args.W}, kappa={args.kappa}, bit-exact PCG64 replay (one worldline_step_fused '
                                  'launch per step)',
                      'L': L, 'lattice': [L, L], 'path': 'worldline', 'parallelism': 'single GPU'}
        report(args, world, world * L * L, L * L, elapsed, acc / (args.steps * L * L), step_kernel_s, config, L,
               metric=f'plaquette-steps/sec (Plaquette + Coexact sweep), L={L} Worldline, W={args.W}',
               unit='plaquette-steps/s',
               kernel='plaquette_level+coexact (whole call)' if reference else 'worldline_step_fused',
               alg_bytes=WORLDLINE_BYTES, min_bytes=WORLDLINE_BYTES, baseline=baseline, ctx=ctx, scaling='strong')
    Lib.sv_worldline_destroy(h)


def run_local(args, world, rank, dist):
    """the Villain and Worldline Hammers' local updates on a device-resident L x L state,
    cold start (Worldline: m = 0, v = 0)."""
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy
    L, kind = args.L, args.workload
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    worldline = kind in WORLDLINE_KINDS
    if worldline:
        ctx.check(Lib.sv_worldline_create(ctx.handle, L, 0, ctypes.byref(h)), 'sv_worldline_create')
        m, v = np.zeros((2, L, L), dtype=np.int64), np.zeros((L, L), dtype=np.int64)
        ctx.check(Lib.sv_worldline_upload(h, _native.ptr(m), _native.ptr(v)), 'upload')
        kinds = ['vortex', 'coexact', 'wrapping'] if kind == 'wlhammer' else [kind]
    else:
        ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'sv_villain_create')
        phi, n = np.zeros((L, L)), np.zeros((2, L, L), dtype=np.int64)
        ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
        kinds = ['site', 'link', 'exact', 'cohomology'] if kind == 'hammer' else [kind]
    rngs = {k: rng_from_numpy(np.random.default_rng(100 * rank + i)) for i, k in enumerate(kinds)}
    kp, W = args.kappa, args.W
    calls = {
        'site': lambda k, st: Lib.sv_villain_site_run(h, kp, float(np.pi), k, ctypes.byref(rngs['site']), st),
        'link': lambda k, st: Lib.sv_villain_link_run(h, kp, W, 1, k, ctypes.byref(rngs['link']), st),
        'exact': lambda k, st: Lib.sv_villain_exact_run(h, kp, 1, k, ctypes.byref(rngs['exact']), st),
        'cohomology': lambda k, st: Lib.sv_villain_cohomology_run(h, kp, 1, k, ctypes.byref(rngs['cohomology']), st),
        'vortex': lambda k, st: Lib.sv_worldline_vortex_run(h, kp, float(W), 1, k, ctypes.byref(rngs['vortex']), st),
        'coexact': lambda k, st: Lib.sv_worldline_coexact_run(h, kp, float(W), 1, k, ctypes.byref(rngs['coexact']),
                                                              st),
        'wrapping': lambda k, st: Lib.sv_worldline_wrapping_run(h, kp, float(W), 1, k, ctypes.byref(rngs['wrapping']),
                                                                st),
    }

    def run(k):
        acc = 0
        if len(kinds) > 1:  # a Hammer: Sequentially, one step of each generator in turn, one deferred step
            for _ in range(k):  # (sv_ctx_set_deferred: one synchronization per Hammer step, as DeviceChain.advance)
                ctx.begin_deferred()
                sts = []
                for g in kinds:
                    sts.append(_native.stats_array(1))
                    ctx.check(calls[g](1, sts[-1]), g)
                ctx.end_deferred()
                acc += sts[0][0].accepted
        else:
            st = _native.stats_array(k)
            ctx.check(calls[kind](k, st), kind)
            acc = sum(st[i].accepted for i in range(k))
        return acc

    warm_up(run, args, dist)
    Lib.sv_ctx_set_timing(ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    acc = run(args.steps)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    ms = ctypes.c_double()
    launches = ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(launches))
    step_kernel_s = ms.value / 1e3 / args.steps  # all kernels of one step (sweep)

    def baseline():
        from oracle import oracle as O
        names = {'site': 'SiteUpdate', 'link': 'LinkUpdate', 'exact': 'ExactUpdate', 'cohomology': 'CohomologyUpdate',
                 'vortex': 'VortexUpdate', 'wrapping': 'WrappingUpdate'}
        k = 2 if kind != 'cohomology' else 2000
        t = time.perf_counter()
        if worldline:
            mm, vv = np.zeros((2, L, L), dtype=np.int64), np.zeros((L, L), dtype=np.int64)
            for _ in range(k):
                for g in kinds:
                    if g == 'coexact':
                        O.worldline_coexact(L, kp, float(W), mm, vv, 1, np.random.default_rng(1))
                    else:
                        O.worldline_generator(names[g], L, kp, float(W), mm, vv, 1, np.random.default_rng(1))
        else:
            pp, nn = np.zeros((L, L)), np.zeros((2, L, L), dtype=np.int64)
            for _ in range(k):
                for g in kinds:
                    O.villain_generator(names[g], L, kp, W, pp, nn, 1, np.random.default_rng(1))
        dt = time.perf_counter() - t
        unit = 'plaquette-updates/s' if worldline else 'lattice-site updates/s'
        return {'value': k * L * L / dt, 'unit': unit, 'cores': 1, 'kind': 'port',
                'sample': f'{k} steps of L={L} {kind}, oracle/sv_oracle.c single-threaded'}

    if rank == 0:
        what = {'site': 'SiteUpdate', 'link': 'LinkUpdate', 'exact': 'ExactUpdate', 'cohomology': 'CohomologyUpdate',
                'hammer': 'Villain Hammer minus worm: SiteUpdate, LinkUpdate, ExactUpdate, CohomologyUpdate',
                'vortex': 'VortexUpdate', 'wrapping': 'WrappingUpdate',
                'wlhammer': 'Worldline Hammer minus worm: VortexUpdate, CoexactUpdate, WrappingUpdate'}[kind]
        model = 'Worldline' if worldline else 'Villain'
        config = {'workload': f'L={L} {model} {what} sweep per step, kappa={kp}, W={W}, bit-exact reference chain '
                              '(PCG64 replay), device-resident fields',
                  'L': L, 'path': kind, 'parallelism': f'{world} independent chain(s)'}
        unit = 'plaquette-updates/s' if worldline else 'lattice-site updates/s'
        report(args, world, world * L * L, L * L, elapsed, acc / (args.steps * L * L), step_kernel_s, config, L,
               metric=f'{unit[:-2]}/sec ({what}), L={L} {model}', unit=unit,
               kernel=f'{kind} (all kernels of a step)', alg_bytes=LOCAL_BYTES.get(kind, 0),
               min_bytes=LOCAL_BYTES.get(kind, 0), baseline=baseline, ctx=ctx, scaling='weak')
    (Lib.sv_worldline_destroy if worldline else Lib.sv_villain_destroy)(h)


def timed_rate(run, sites, args, dist):
    """Sites per second of `run(k)` (k sweeps) after the main run's warm-up (warm_up: W steps, then --warmup-s
    seconds), over max(--steps, 100) sweeps (a NumPy rejection costs about one sweep: over 20 sweeps one of them moved
    R1 by ~5%, and E_N with it); returns (rate, run's result)."""
    warm_up(run, args, dist)
    k = max(args.steps, 100)
    t = time.perf_counter()
    out = run(k)
    return sites * k / (time.perf_counter() - t), out


def single_lattice_rate(L, args, dist):
    """The N = 1 headline path (sv_villain_run on one periodic L x L lattice, villain_sweep_hot) on this rank's
    GPU: (site-updates/s, NumPy Lemire rejections in the timed sweeps)."""
    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy
    Lib = _native.lib()
    ctx = _native.context(_native.default_device())
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'sv_villain_create')
    try:
        phi, n = np.zeros((L, L)), np.zeros((2, L, L), np.int64)  # (held: ptr() keeps no reference)
        ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
        r = rng_from_numpy(np.random.default_rng(1))

        def run(k):
            st = _native.stats_array(k)
            ctx.check(Lib.sv_villain_run(h, args.kappa, args.W, float(np.pi), 1, k, ctypes.byref(r), st, 2),
                      'sv_villain_run')
            return sum(st[i].rejections for i in range(k))

        return timed_rate(run, L * L, args, dist)
    finally:
        Lib.sv_villain_destroy(h)


E_N_FLAG = 1.02  # an efficiency above this is not physical: R1 was mismeasured


def scaling_reference(value, world, r1, tile, single, single_rej, unit='sweeps'):
    """config.scaling_reference of a domain line: R1 (this tile alone), E_N = R_N / (N R1), and the single-lattice
    headline rate beside it; flags an E_N above E_N_FLAG (also on stderr)."""
    e = value / (world * r1)
    out = {'tile': tile, 'R1': r1, 'E_N': e, 'E_N_suspect': e > E_N_FLAG,
           'definition': 'E_N = R_N / (N R1), R1 = one GPU running one periodic tile of this size alone (SURVEY.md '
                         f'8(d)), timed after the main run\'s warm-up over max(--steps, 100) {unit}, mean over ranks'}
    if world == 1:
        out['emulation_note'] = ('one GPU runs every tile in turn: E_N here compares the decomposed lattice per tile with '
                                 'one tile alone (the decomposition\'s own overhead), and one NumPy rejection in a short '
                                 'timed window (one process does not predict them) moves it by ~5-10%')
    if single is not None:
        out['single_lattice_rate'] = single
        out['single_lattice_rejections_in_timed_steps'] = single_rej
        out['E_N_vs_single_lattice'] = value / (world * single)
        out['single_lattice_definition'] = ('the N = 1 headline path (sv_villain_run, villain_sweep_hot) on one '
                                            'periodic L x L lattice per GPU, mean over ranks: for --weak the per-GPU R1 '
                                            'of the headline kernel, for strong scaling the one-GPU rate of the whole '
                                            'lattice')
    if e > E_N_FLAG:
        print(f'bench.py: E_N = {e:.3f} > {E_N_FLAG} (R1 = {r1:.4g}): the tile-alone reference is suspect',
              file=sys.stderr, flush=True)
    return out


def run_domain(args, world, rank, local, dist):
    """N > 1 (or --tiles on one GPU): BASELINE config 4, one lattice domain-decomposed, RCCL halos."""
    from supervillain_amd import _native
    from supervillain_amd.domain import VillainDomain, ghost_frame, tile_grid
    L = args.L
    if args.tiles:
        ty, tx = (int(v) for v in args.tiles.lower().split('x'))
    else:
        ty, tx = tile_grid(world)
    Nt, Nx = (L, L) if args.strong else (ty * L, tx * L)
    Ht, Wt = Nt // ty, Nx // tx
    kw = dict(kappa=args.kappa, W=args.W)  # device: $SV_DEVICE, else $LOCAL_RANK
    if world > 1:
        dom = VillainDomain.distributed(Nt, Nx, (ty, tx), transport=args.transport, **kw)
    else:
        dom = VillainDomain(Nt, Nx, (ty, tx), **kw)
    dom.cold()
    gen = np.random.default_rng(0)  # one chain: every rank holds the same stream
    Lib = _native.lib()
    warm_up(lambda k: dom.run(k, gen), args, dist)
    Lib.sv_ctx_set_timing(dom.ctx.handle, 1)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    st = dom.run(args.steps, gen)  # synchronous on return
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(dist, t1 - t0)
    avg_launch_s = kernel_time(Lib, dom.ctx)
    acc = sum(s.accepted for s in st) / (args.steps * Nt * Nx)
    rej = sum(s.rejections for s in st)
    ctx = dom.ctx
    dom.close()

    # R1: this rank's tile alone, as a periodic Ht x Wt lattice on its own GPU, no exchange, timed
    # after the same warm-up as the main run; then the single-lattice headline path on one L x L lattice
    one = VillainDomain(Ht, Wt, (1, 1), **kw)
    one.cold()
    g1 = np.random.default_rng(1)
    r1, _ = timed_rate(lambda k: one.run(k, g1), Ht * Wt, args, dist)
    one.close()
    r1_mean = r1 if dist is None else _mean_over_ranks(dist, r1)
    single, single_rej = single_lattice_rate(L, args, dist)
    single_mean = single if dist is None else _mean_over_ranks(dist, single)

    if rank == 0:
        value = args.steps * Nt * Nx / elapsed
        config = {'workload': f'{Nt}x{Nx} Villain NeighborhoodUpdate sweep, kappa={args.kappa}, W={args.W}, '
                              f'domain-decomposed into {ty}x{tx} tiles of {Ht}x{Wt} (one per GPU), RCCL halo '
                              'exchange, bit-exact reference chain (PCG64 replay)',
                  'L': L, 'lattice': [Nt, Nx], 'tiles': [ty, tx], 'path': 'domain',
                  'halo_transport': args.transport if world > 1 else 'none (one process)',
                  # deep halos: K sweeps per halo exchange, ghost frame 2K / 3K deep
                  'sweeps_per_halo_exchange': ghost_frame(Nt, Nx, (ty, tx))[0] // 2,
                  'parallelism': f'{ty}x{tx} domain decomposition over {world} GPU(s)' +
                                 ('' if world > 1 else ' (emulated: every tile on this GPU in turn)'),
                  'lemire_rejections_in_timed_steps': int(rej),
                  'scaling_reference': scaling_reference(value, world, r1_mean, [Ht, Wt], single_mean, int(single_rej))}
        report(args, world, Nt * Nx, Nt * Nx // world, elapsed, acc, avg_launch_s, config, Ht, ctx=ctx,
               metric=lattice_metric(Nt, Nx, weak_tile=None if args.strong else [Ht, Wt]),
               kernel='villain_sweep_hot (tile)')


def _mean_over_ranks(dist, x):
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item()) / dist.get_world_size()


def run_ranks(args, world, rank, dist):
    """--workload ranks: the launcher's rank / world plumbing alone, no GPU (a CPU test drives it)."""
    tot = _mean_over_ranks(dist, float(rank)) * world if dist else 0.0
    if rank == 0:
        print(json.dumps({'workload': 'ranks', 'world': world, 'rank_sum': tot,
                          'master_addr': os.environ.get('MASTER_ADDR'),
                          'local_ranks': world}), flush=True)


def launch_command(gpus, argv, port):
    """The torch.distributed.run command that re-runs this script with one rank per GPU (no exec: the parent
    waits for it; it has touched no GPU)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={gpus}',
            '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + list(argv)


def spawn(gpus, argv):
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    return subprocess.call(launch_command(gpus, argv, port))


def main():
    args = parse()
    if args.gpus is not None and args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn(args.gpus, sys.argv[1:]))  # one rank per GPU, before any HIP call in this process
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.gpus is not None and args.gpus != world:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}', file=sys.stderr)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        # gloo prints its connection messages on stdout ("[Gloo] Rank 0 is connected to ..."), interleaved across the
        # ranks: they go to stderr, so that stdout carries rank 0's one JSON line only
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group('gloo', rank=rank, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if args.workload != 'villain':
        fn = {'replicas': run_replicas, 'worldline': run_worldline, 'worms': run_worms,
              'ranks': run_ranks}.get(args.workload, run_local)
        fn(args, world, rank, dist)
        if dist:
            dist.destroy_process_group()
        return
    if world > 1 or args.tiles:
        run_domain(args, world, rank, local, dist)
        if dist:
            dist.destroy_process_group()
        return

    from supervillain_amd import _native
    from supervillain_amd._abi import rng_from_numpy

    Lib = _native.lib()
    ctx = _native.context(local)
    L = args.L
    h = ctypes.c_void_p()
    ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'sv_villain_create')
    phi = np.zeros((L, L))
    n = np.zeros((2, L, L), dtype=np.int64)
    ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
    r = rng_from_numpy(np.random.default_rng(0))
    from supervillain_amd._abi import SvPhilox
    ph = SvPhilox(0x5eed, 0, 0)

    def run(k):
        st = _native.stats_array(k)
        if args.rng == 'philox':
            ctx.check(Lib.sv_villain_run_philox(h, args.kappa, args.W, float(np.pi), 1, k, ctypes.byref(ph), st),
                      'sv_villain_run_philox')
        else:
            ctx.check(Lib.sv_villain_run(h, args.kappa, args.W, float(np.pi), 1, k, ctypes.byref(r), st, args.path),
                      'sv_villain_run')
        return st

    warm_up(run, args)
    Lib.sv_ctx_set_timing(ctx.handle, 2 if args.event_timing == 'launch' else 1)
    Lib.sv_ctx_block_counts(ctx.handle, None, None)  # (reset: count the timed sweeps' kernels only)
    Lib.sv_ctx_band_counts(ctx.handle, None, None)
    t0 = time.perf_counter()
    st = run(args.steps)  # synchronous on return (stream synchronized)
    t1 = time.perf_counter()
    # hipEvents around the hot kernel's launches in the timed region (replays of a sweep that met a NumPy Lemire
    # rejection run on the general kernel and are not counted); if the window held no countable launch (a
    # rejection in its last sweep), time the next `steps` sweeps the same way, after the timed region
    launches = ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, None, ctypes.byref(launches))
    if launches.value == 0:
        run(args.steps)
    avg_launch_s = kernel_time(Lib, ctx)
    acc = sum(st[i].accepted for i in range(args.steps)) / (args.steps * L * L)
    rej = sum(st[i].rejections for i in range(args.steps))
    chain = ('bit-exact reference chain (PCG64 replay), fused two-colour sweep kernel (villain_sweep_hot)'
             if args.rng == 'pcg64' else 'counter-based Philox4x32-10 mode (a different chain from the reference\'s), '
             'fused two-colour sweep kernel (villain_sweep_hot_ph)')
    # which kernel ran the timed sweeps: small lattices run K sweeps per launch (temporal blocks,
    # villain_sweep_block; or the XCD bands, villain_sweep_hot_band), the rest villain_sweep_hot
    blk, band = ctypes.c_int64(), ctypes.c_int64()
    Lib.sv_ctx_block_counts(ctx.handle, ctypes.byref(blk), None)
    Lib.sv_ctx_band_counts(ctx.handle, ctypes.byref(band), None)
    kernel = 'villain_sweep_hot'
    if args.rng == 'philox':
        kernel = 'villain_sweep_hot_ph'
    elif blk.value > 0:
        kernel = 'villain_sweep_block'
        chain = chain.replace('fused two-colour sweep kernel (villain_sweep_hot)',
                              'temporal blocks of K sweeps per launch (villain_sweep_block)')
    elif band.value > 0:
        kernel = 'villain_sweep_hot_band'
        chain = chain.replace('(villain_sweep_hot)', '(villain_sweep_hot_band: K sweeps per launch)')
    config = {'workload': f'L={L} Villain NeighborhoodUpdate sweep, kappa={args.kappa}, W={args.W}, ' + chain,
              'rng': args.rng,
              'L': L, 'lattice': [L, L], 'path': args.path, 'parallelism': 'single GPU',
              'lemire_rejections_in_timed_steps': int(rej)}
    report(args, 1, L * L, L * L, t1 - t0, acc, avg_launch_s, config, L, ctx=ctx, kernel=kernel,
           metric=lattice_metric(L, L))
    Lib.sv_villain_destroy(h)


if __name__ == '__main__':
    main()
