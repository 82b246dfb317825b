"""Device buffers for GPU tests, on the HIP runtime the product library runs on.

PyTorch-ROCm wheels bundle their own libamdhip64 / libhsa-runtime64; a second HIP runtime cannot
open the device once the product library's runtime holds it in the same process ("No HIP GPUs are
available", hipErrorNoDevice).  Tests therefore allocate device memory through the exact
libamdhip64 that libimls_gpu.so loaded (its RUNPATH copy, found in /proc/self/maps), never through
torch — bench.py, a separate process that initialises torch first, is unaffected."""
import ctypes
import functools

import numpy as np


@functools.lru_cache(maxsize=1)
def product_hip():
    import plo_amd
    plo_amd.load()._abi.load_library()           # libimls_gpu.so (and its libamdhip64) mapped
    paths = []
    with open("/proc/self/maps") as f:
        for line in f:
            part = line.split()
            if len(part) >= 6 and "libamdhip64.so" in part[-1] and "/torch/" not in part[-1]:
                paths.append(part[-1])
    if not paths:
        raise RuntimeError("libamdhip64 of the product library not mapped")
    h = ctypes.CDLL(paths[0], mode=ctypes.RTLD_GLOBAL)
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipFree.argtypes = [ctypes.c_void_p]
    return h


class DevSoa:
    """A (6, n) float32 SoA cloud (or any float32 array) copied to device memory."""

    def __init__(self, a, hip=None):
        a = np.ascontiguousarray(a, np.float32)
        self.hip = hip or product_hip()
        self.n = a.shape[-1]
        self.nbytes = a.nbytes
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), a.nbytes) == 0
        assert self.hip.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1) == 0   # host → device
        self.ptr = p.value

    def data_ptr(self):
        return self.ptr

    def overwrite(self, a):
        a = np.ascontiguousarray(a, np.float32)
        assert a.nbytes <= self.nbytes
        assert self.hip.hipMemcpy(ctypes.c_void_p(self.ptr), a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1) == 0

    def free(self):
        if self.ptr:
            self.hip.hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = None
