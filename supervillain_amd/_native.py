"""Loader for libsvhip.so, the HIP/gfx950 engine behind the generators (C-ABI: include/supervillain_amd.h).

There is no CPU fallback: if the library or a HIP device is missing, every generator step raises.
"""
import ctypes
import logging
import os
import threading

from supervillain_amd._abi import SvMT19937, SvPhilox, SvRng, SvStats

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libsvhip.so')
# Timing experiments (scripts/build_variant.sh) load an instrumented build of the same sources through
# SV_LIB_OVERRIDE; only builds under the repository's variants/ directories are accepted.
VARIANT_DIRS = (os.path.join(_HERE, 'variants'), os.path.join(os.path.dirname(_HERE), 'variants'))


def lib_path():
    """The library to load: libsvhip.so beside this file, or an experiment build named by SV_LIB_OVERRIDE that lies
    under one of VARIANT_DIRS (anything else raises NativeError)."""
    o = os.environ.get('SV_LIB_OVERRIDE')
    if not o:
        return LIB_PATH
    p = os.path.realpath(o)
    if not any(p.startswith(os.path.realpath(d) + os.sep) for d in VARIANT_DIRS):
        raise NativeError(f'SV_LIB_OVERRIDE={o!r}: only experiment builds under {VARIANT_DIRS} are loaded')
    return p
_LIB = None
_LOCK = threading.RLock()
# sv_domain_create_hosted's callbacks (include/supervillain_amd.h sv_xfer_fn, sv_gather_fn)
XFER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
                           ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p)
GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
_CONTEXTS = {}


class NativeError(RuntimeError):
    pass


def lib():
    """The loaded libsvhip.so (raises NativeError if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = lib_path()
        if not os.path.exists(path):
            raise NativeError(f'{path} is missing; build it with `python -c "import __graft_entry__ as g; g.build()"` '
                              '(or `make -C supervillain_amd/csrc`).  There is no CPU fallback.')
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        i32, i64, f64, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
        L.sv_ctx_create.argtypes = [ctypes.c_int, P(vp)]
        L.sv_ctx_destroy.argtypes = [vp]
        L.sv_last_error.argtypes = [vp]
        L.sv_last_error.restype = ctypes.c_char_p
        L.sv_device_count.argtypes = []
        L.sv_build_info.restype = ctypes.c_char_p
        L.sv_ctx_set_timing.argtypes = [vp, i32]
        L.sv_ctx_kernel_time.argtypes = [vp, P(f64), P(i64)]
        L.sv_ctx_sweep_counts.argtypes = [vp, P(i64), P(i64), P(i64)]
        L.sv_ctx_band_counts.argtypes = [vp, P(i64), P(i64)]
        L.sv_ctx_block_counts.argtypes = [vp, P(i64), P(i64)]
        L.sv_ctx_split_counts.argtypes = [vp, P(i64)]
        L.sv_ctx_set_multisweep.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.sv_ctx_set_table_cap.argtypes = [vp, ctypes.c_int32]
        L.sv_ctx_table_purges.argtypes = [vp, P(i64)]
        L.sv_hbm_copy.argtypes = [vp, i64, i32, i32, P(f64)]
        L.sv_rng_gather.argtypes = [vp, i32, vp]
        L.sv_rng_scatter.argtypes = [vp, i32, vp]
        L.sv_villain_neighborhood.argtypes = [vp, i32, f64, i64, f64, i64, vp, vp, i32, P(SvRng), P(SvStats)]
        L.sv_villain_create.argtypes = [vp, i32, P(vp)]
        L.sv_villain_destroy.argtypes = [vp]
        L.sv_villain_upload.argtypes = [vp, vp, vp]
        L.sv_villain_download.argtypes = [vp, vp, vp]
        L.sv_villain_run_philox.argtypes = [vp, f64, i64, f64, i64, i32, P(SvPhilox), P(SvStats)]
        L.sv_villain_emit.argtypes = [vp, vp, vp]
        L.sv_villain_emit_wait.argtypes = [vp]
        L.sv_worldline_emit.argtypes = [vp, vp, vp]
        L.sv_worldline_emit_wait.argtypes = [vp]
        L.sv_host_alloc.argtypes = [ctypes.c_size_t, P(vp)]
        L.sv_ctx_set_deferred.argtypes = [vp, i32]
        L.sv_ctx_sync.argtypes = [vp]
        L.sv_host_free.argtypes = [vp]
        L.sv_villain_run.argtypes = [vp, f64, i64, f64, i64, i32, P(SvRng), P(SvStats), i32]
        L.sv_villain_observables.argtypes = [vp, f64, vp]
        L.sv_villain_site_run.argtypes = [vp, f64, f64, i32, P(SvRng), P(SvStats)]
        L.sv_villain_link_run.argtypes = [vp, f64, i64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_villain_exact_run.argtypes = [vp, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_villain_cohomology_run.argtypes = [vp, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_create.argtypes = [vp, i32, i32, P(vp)]
        L.sv_worldline_destroy.argtypes = [vp]
        L.sv_worldline_upload.argtypes = [vp, vp, vp]
        L.sv_worldline_download.argtypes = [vp, vp, vp]
        L.sv_worldline_coexact_run.argtypes = [vp, f64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_coexact.argtypes = [vp, i32, f64, f64, i64, vp, vp, i32, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_plaquette_ordered_run.argtypes = [vp, f64, f64, vp, P(SvRng), P(SvStats)]
        L.sv_mt19937_permutation.argtypes = [P(SvMT19937), i64, vp]
        L.sv_worldline_plaquette_reference_run.argtypes = [vp, f64, f64, i32, P(SvMT19937), P(SvRng), P(SvStats)]
        L.sv_worldline_plaquette_reference_coexact_run.argtypes = [vp, f64, f64, i64, i32, P(SvMT19937), P(SvRng),
                                                                   P(SvStats)]
        L.sv_worldline_plaquette_checkerboard_run.argtypes = [vp, f64, f64, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_plaquette.argtypes = [vp, i32, f64, f64, vp, vp, i32, vp, P(SvRng), P(SvStats)]
        L.sv_worldline_plaquette_coexact_run.argtypes = [vp, f64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_vortex_run.argtypes = [vp, f64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_worldline_wrapping_run.argtypes = [vp, f64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_domain_unique_id.argtypes = [vp]
        L.sv_domain_create.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, P(vp)]
        L.sv_domain_destroy.argtypes = [vp]
        L.sv_domain_upload.argtypes = [vp, vp, vp]
        L.sv_domain_download.argtypes = [vp, vp, vp]
        L.sv_domain_run.argtypes = [vp, f64, i64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_domain_exchange_plan.argtypes = [i32, i32, i32, i32, i32, vp]
        L.sv_domain_message_layout.argtypes = [i32, i32, i32, i32, i32, vp]
        L.sv_domain_create_worldline.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, P(vp)]
        L.sv_domain_create_hosted.argtypes = [vp, i32, i32, i32, i32, i32, i32, i32, XFER_FN, GATHER_FN, vp, P(vp)]
        L.sv_domain_upload_worldline.argtypes = [vp, vp, vp]
        L.sv_domain_download_worldline.argtypes = [vp, vp, vp]
        L.sv_domain_run_worldline.argtypes = [vp, f64, f64, i64, i32, P(SvRng), P(SvStats)]
        L.sv_domain_exchange_plan_worldline.argtypes = [i32, i32, i32, i32, i32, vp]
        L.sv_domain_message_layout_worldline.argtypes = [i32, i32, i32, i32, i32, vp]
        L.sv_replicas_create.argtypes = [vp, i32, i32, P(vp)]
        L.sv_replicas_destroy.argtypes = [vp]
        L.sv_replicas_upload.argtypes = [vp, vp, vp]
        L.sv_replicas_download.argtypes = [vp, vp, vp]
        L.sv_replicas_run.argtypes = [vp, f64, i64, f64, i64, i32, vp, vp, vp]
        L.sv_replicas_run_measured.argtypes = [vp, f64, i64, f64, i64, i32, vp, vp, vp, vp, vp, vp, vp]
        L.sv_replicas_villain.argtypes = [vp, i32, i32, f64, i64, f64, i64, vp, vp, i32, vp, vp, vp]
        L.sv_villain_worm_run.argtypes = [vp, f64, i64, i32, i64, P(SvRng), vp, vp]
        L.sv_replicas_worm_run.argtypes = [vp, f64, i64, i32, i64, vp, vp, vp]
        L.sv_worldline_worm_run.argtypes = [vp, f64, f64, i32, i64, P(SvRng), vp, vp]
        L.sv_worldline_worm_batch.argtypes = [vp, i32, i32, f64, f64, vp, vp, i32, i32, i64, vp, vp, vp]
        _LIB = L
        return L


EXPORTED = ('sv_ctx_create', 'sv_ctx_destroy', 'sv_last_error', 'sv_device_count', 'sv_build_info',
            'sv_ctx_set_timing', 'sv_ctx_kernel_time', 'sv_ctx_sweep_counts', 'sv_ctx_band_counts', 'sv_ctx_block_counts', 'sv_ctx_split_counts', 'sv_ctx_set_multisweep', 'sv_ctx_set_table_cap', 'sv_ctx_table_purges', 'sv_hbm_copy', 'sv_rng_gather', 'sv_rng_scatter',
            'sv_villain_neighborhood', 'sv_villain_create', 'sv_villain_destroy', 'sv_villain_upload',
            'sv_villain_download', 'sv_villain_run', 'sv_villain_observables', 'sv_villain_emit', 'sv_villain_emit_wait', 'sv_villain_run_philox',
            'sv_worldline_emit', 'sv_worldline_emit_wait', 'sv_host_alloc', 'sv_host_free',
            'sv_ctx_set_deferred', 'sv_ctx_sync',
            'sv_villain_site_run', 'sv_villain_link_run', 'sv_villain_exact_run', 'sv_villain_cohomology_run', 'sv_worldline_create',
            'sv_worldline_destroy', 'sv_worldline_upload', 'sv_worldline_download', 'sv_worldline_coexact_run',
            'sv_worldline_coexact', 'sv_worldline_plaquette_ordered_run', 'sv_mt19937_permutation',
            'sv_worldline_plaquette_reference_run', 'sv_worldline_plaquette_reference_coexact_run',
            'sv_worldline_plaquette_checkerboard_run', 'sv_worldline_plaquette', 'sv_worldline_plaquette_coexact_run',
            'sv_worldline_vortex_run', 'sv_worldline_wrapping_run',
            'sv_domain_unique_id', 'sv_domain_create', 'sv_domain_destroy', 'sv_domain_upload', 'sv_domain_download',
            'sv_domain_run', 'sv_domain_exchange_plan', 'sv_domain_message_layout', 'sv_domain_create_worldline',
            'sv_domain_create_hosted',
            'sv_domain_upload_worldline', 'sv_domain_download_worldline', 'sv_domain_run_worldline',
            'sv_domain_exchange_plan_worldline', 'sv_domain_message_layout_worldline',
            'sv_replicas_create', 'sv_replicas_destroy', 'sv_replicas_upload', 'sv_replicas_download',
            'sv_replicas_run', 'sv_replicas_run_measured', 'sv_replicas_villain', 'sv_villain_worm_run', 'sv_replicas_worm_run', 'sv_worldline_worm_run',
            'sv_worldline_worm_batch')


def default_device():
    for var in ('SV_DEVICE', 'LOCAL_RANK'):
        if var in os.environ:
            return int(os.environ[var])
    return 0


class Context:
    """One HIP device + stream (sv_ctx).  Not thread-safe, like the reference's generators."""

    def __init__(self, device):
        self.device = device
        h = ctypes.c_void_p()
        rc = lib().sv_ctx_create(device, ctypes.byref(h))
        if rc != 0 or not h.value:
            raise NativeError(f'cannot open HIP device {device} (sv_ctx_create returned {rc}); '
                              'the supervillain_amd generators run only on an MI355X')
        self.handle = h
        self.folds = None  # open deferred step: counter folds waiting for sv_ctx_sync

    def begin_deferred(self):
        """Open a deferred step: runs that cannot meet a rejection return without synchronizing (sv_ctx_set_deferred)
        and their counter folds (fold_later) wait for end_deferred."""
        self.check(lib().sv_ctx_set_deferred(self.handle, 1), 'sv_ctx_set_deferred')
        self.folds = []

    def end_deferred(self):
        """One synchronization lands every deferred statistic; then the folds run in call order."""
        folds, self.folds = self.folds, None
        err = None
        try:
            self.check(lib().sv_ctx_set_deferred(self.handle, 0), 'sv_ctx_set_deferred')
        except NativeError as e:
            err = e
        # the statistics landed even when a member aborted: fold them, so that the counters match the device.  The
        # deferred-run error stays the one raised; a fold that fails after it is chained to it, not raised instead.
        try:
            for f in folds or ():
                f()
        except Exception as fold_error:
            if err is not None:
                raise err from fold_error
            raise
        if err is not None:
            raise err

    def fold_later(self, fold):
        """Run a counter fold that reads sv_stats now, or at end_deferred inside a deferred step."""
        if self.folds is None:
            fold()
        else:
            self.folds.append(fold)

    def sweep_counts(self):
        """Villain sweep launches by kernel since the last call: {'hot', 'fused', 'generic'} (sv_ctx_sweep_counts)."""
        c = [ctypes.c_int64() for _ in range(3)]
        self.check(lib().sv_ctx_sweep_counts(self.handle, *[ctypes.byref(x) for x in c]), 'sv_ctx_sweep_counts')
        return dict(zip(('hot', 'fused', 'generic'), (x.value for x in c)))

    def split_counts(self):
        """Sweeps replayed on the split replay kernel since the last call (sv_ctx_split_counts)."""
        c = ctypes.c_int64()
        self.check(lib().sv_ctx_split_counts(self.handle, ctypes.byref(c)), 'sv_ctx_split_counts')
        return c.value

    def band_counts(self):
        """Multi-sweep band launches since the last call: {'sweeps', 'launches'} (sv_ctx_band_counts)."""
        c = [ctypes.c_int64() for _ in range(2)]
        self.check(lib().sv_ctx_band_counts(self.handle, *[ctypes.byref(x) for x in c]), 'sv_ctx_band_counts')
        return dict(zip(('sweeps', 'launches'), (x.value for x in c)))

    def block_counts(self):
        """Temporal-blocking launches since the last call: {'sweeps', 'launches'} (sv_ctx_block_counts)."""
        c = [ctypes.c_int64() for _ in range(2)]
        self.check(lib().sv_ctx_block_counts(self.handle, *[ctypes.byref(x) for x in c]), 'sv_ctx_block_counts')
        return dict(zip(('sweeps', 'launches'), (x.value for x in c)))

    def set_multisweep(self, mode, K=0):
        """Multi-sweep launches of small lattices: 0 blocks or bands, 1 blocks, 2 bands, 3 none; K sweeps per
        temporal-blocking launch (0: the default) (sv_ctx_set_multisweep)."""
        self.check(lib().sv_ctx_set_multisweep(self.handle, int(mode), int(K)), 'sv_ctx_set_multisweep')

    def set_table_cap(self, cap):
        """Bound this context's jump-table cache to `cap` increments (0: the default; tests) (sv_ctx_set_table_cap)."""
        self.check(lib().sv_ctx_set_table_cap(self.handle, int(cap)), 'sv_ctx_set_table_cap')

    def table_purges(self):
        """How often this context dropped its jump-table cache (sv_ctx_table_purges)."""
        n = ctypes.c_int64()
        self.check(lib().sv_ctx_table_purges(self.handle, ctypes.byref(n)), 'sv_ctx_table_purges')
        return n.value

    def check(self, rc, what):
        if rc != 0:
            msg = lib().sv_last_error(self.handle)
            raise NativeError(f'{what} failed: {msg.decode() if msg else rc}')

    def __del__(self):
        try:
            if _LIB is not None and self.handle:
                _LIB.sv_ctx_destroy(self.handle)
        except Exception:
            pass


def destroy(fn, handle, what, ctx=None, in_del=False):
    """Run an sv_*_destroy.  A destroy first drains the work queued on the context stream; when that work failed
    the library records which object's destroy saw it (sv_last_error) and returns -2 after freeing everything.  An
    explicit close raises it as NativeError; a destroy from __del__ (garbage collection) logs it, since it cannot
    raise -- so a fault is named at the object whose queued work failed, not at the next unrelated call."""
    rc = fn(handle)
    if rc == 0:
        return
    msg = lib().sv_last_error(ctx.handle) if ctx is not None and ctx.handle else None
    text = f'{what} failed: {msg.decode() if msg else rc}'
    if in_del:
        logging.getLogger('supervillain_amd').error(text)
    else:
        raise NativeError(text)


def context(device=None):
    if device is None:
        device = default_device()
    with _LOCK:
        ctx = _CONTEXTS.get(device)
        if ctx is None:
            ctx = Context(device)
            _CONTEXTS[device] = ctx
        return ctx


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def stats_array(k):
    return (SvStats * max(k, 1))()
