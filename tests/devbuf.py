"""Device buffers for the kernel-level parity tests, through the C-ABI only
(mpg_malloc / mpg_memcpy_*), so the tests exercise exactly what a foreign
binding would call."""
import ctypes as C

import numpy as np


class Hip:
    def __init__(self, lib, device: int = 0):
        self.lib = lib
        self.ctx = C.c_void_p()
        self.check(lib.mpg_ctx_create(device, C.byref(self.ctx)), "mpg_ctx_create")
        self._live = []

    def check(self, st, what="call"):
        if st != 0:
            err = self.lib.mpg_ctx_last_error(self.ctx) if self.ctx else b""
            raise RuntimeError(f"{what}: {self.lib.mpg_error_string(st).decode()} {err.decode() if err else ''}")

    def call(self, name, *args):
        self.check(getattr(self.lib, name)(self.ctx, *args), name)

    def buf(self, arr_or_n, dtype=None):
        return DevBuf(self, arr_or_n, dtype)

    def sync(self):
        self.check(self.lib.mpg_ctx_sync(self.ctx), "sync")

    def close(self):
        for b in self._live:
            b.free()
        self._live.clear()
        if self.ctx:
            self.lib.mpg_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()


class DevBuf:
    def __init__(self, hip: Hip, arr_or_n, dtype=None):
        self.hip = hip
        if isinstance(arr_or_n, (int, np.integer)):
            self.dtype = np.dtype(dtype or np.float64)
            self.n = int(arr_or_n)
            host = None
        else:
            host = np.ascontiguousarray(arr_or_n, dtype=dtype)
            self.dtype = host.dtype
            self.n = host.size
        self.nbytes = max(self.n * self.dtype.itemsize, 1)
        self.ptr = C.c_void_p()
        hip.check(hip.lib.mpg_malloc(hip.ctx, self.nbytes, C.byref(self.ptr)), "mpg_malloc")
        hip._live.append(self)
        if host is not None and host.size:
            hip.check(hip.lib.mpg_memcpy_h2d(hip.ctx, self.ptr, host.ctypes.data, host.nbytes), "h2d")

    @property
    def p(self):
        return self.ptr

    def at(self, i):
        """Device pointer to element i."""
        return C.c_void_p(self.ptr.value + i * self.dtype.itemsize)

    def get(self):
        out = np.empty(self.n, self.dtype)
        if self.n:
            self.hip.check(self.hip.lib.mpg_memcpy_d2h(self.hip.ctx, out.ctypes.data, self.ptr, out.nbytes), "d2h")
        return out

    def free(self):
        if self.ptr:
            self.hip.lib.mpg_free(self.hip.ctx, self.ptr)
            self.ptr = C.c_void_p()
