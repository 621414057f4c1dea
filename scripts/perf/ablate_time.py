"""hipEvent time per hot sweep at L x L over calls of `k` sweeps until the first call that fails or meets a NumPy
rejection (timing-only ablation builds cannot replay one).  Usage: ablate_time.py L k calls"""
import ctypes
import sys

import numpy as np

sys.path.insert(0, '.')
from supervillain_amd import _native  # noqa: E402
from supervillain_amd._abi import rng_from_numpy  # noqa: E402

L, k, calls = (int(x) for x in sys.argv[1:4])
Lib = _native.lib()
ctx = _native.context(0)
h = ctypes.c_void_p()
ctx.check(Lib.sv_villain_create(ctx.handle, L, ctypes.byref(h)), 'create')
phi = np.zeros((L, L))
n = np.zeros((2, L, L), dtype=np.int64)
ctx.check(Lib.sv_villain_upload(h, _native.ptr(phi), _native.ptr(n)), 'upload')
r = rng_from_numpy(np.random.default_rng(5))
st = _native.stats_array(k)
tot, nl = 0.0, 0
for c in range(calls):
    Lib.sv_ctx_set_timing(ctx.handle, 1)
    rc = Lib.sv_villain_run(h, 0.5, 1, float(np.pi), 1, k, ctypes.byref(r), st, 2)
    ms, cnt = ctypes.c_double(), ctypes.c_int64()
    Lib.sv_ctx_kernel_time(ctx.handle, ctypes.byref(ms), ctypes.byref(cnt))
    Lib.sv_ctx_set_timing(ctx.handle, 0)
    if rc != 0 or any(st[i].rejections for i in range(k)):
        break
    tot += ms.value
    nl += cnt.value
print(f'L={L}: {nl} clean hot launches, {tot / max(nl, 1) * 1e3:.1f} us each', flush=True)
