"""HBM copy ceiling and PMC calibration (measurement only): sv_hbm_copy with 16-B and 8-B lanes over two 1 GiB
buffers.  Run plain for GB/s, or under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` to compare the
counters with the known 1 GiB read + 1 GiB write per launch (MI355X_MICROARCH.md: FETCH_SIZE is uncalibrated
for widths other than 16 B/lane)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from supervillain_amd import _native  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = _native.context(0)
out = {'bytes_per_buffer': 1 << 30, 'iters': iters}
for w in (16, 8):
    g = ctypes.c_double()
    ctx.check(_native.lib().sv_hbm_copy(ctx.handle, 1 << 30, w, iters, ctypes.byref(g)), 'sv_hbm_copy')
    out[f'GBps_w{w}'] = g.value
print(json.dumps(out), flush=True)
