"""A process that only initialises HIP, allocates, frees and exits: with AMD_LOG_LEVEL=1 it shows which runtime
error-level lines (e.g. "Unknown Event Type") a clean process prints, to tell them from a fault's."""
import ctypes
hip = ctypes.CDLL('libamdhip64.so')
p = ctypes.c_void_p()
assert hip.hipSetDevice(0) == 0
assert hip.hipMalloc(ctypes.byref(p), 1 << 20) == 0
assert hip.hipFree(p) == 0
assert hip.hipDeviceSynchronize() == 0
print('clean HIP process done', flush=True)
