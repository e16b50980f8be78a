"""FFT plan objects over the C-ABI (neo_hip_fft_plan_*), cached per shape."""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from .. import _native


class FFTPlan:
    """A batched c2c / r2c / c2r plan on one GPU (replaces fft_plan / rfft_plan,
    src/neo/fft/fft.hpp:36-52, src/neo/fft/rfft.hpp:15-23)."""

    def __init__(self, kind: int, order: int, batch: int = 1, device: int = 0):
        lib = _native.load()
        h = ctypes.c_void_p()
        _native.check(lib.neo_hip_fft_plan_create(int(order), int(batch), int(kind), int(device), ctypes.byref(h)))
        self._h = h
        self.kind, self.order, self.batch, self.device = kind, order, batch, device

    @property
    def size(self) -> int:
        return 1 << self.order

    def execute_device(self, in_ptr: int, out_ptr: int, direction: int, stream: int = 0) -> None:
        _native.check(_native.load().neo_hip_fft_execute(self._h, ctypes.c_void_p(in_ptr), ctypes.c_void_p(out_ptr),
                                                         int(direction), ctypes.c_void_p(stream)))

    def execute_host(self, a: np.ndarray, out: np.ndarray, direction: int) -> None:
        assert a.flags.c_contiguous and out.flags.c_contiguous
        _native.check(_native.load().neo_hip_fft_execute_host(self._h, a.ctypes.data_as(ctypes.c_void_p),
                                                              out.ctypes.data_as(ctypes.c_void_p), int(direction)))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().neo_hip_fft_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_cache: dict = {}
_cache_lock = threading.Lock()


def get_plan(kind: int, order: int, batch: int, device: int = 0) -> FFTPlan:
    key = (kind, order, batch, device)
    with _cache_lock:
        p = _cache.get(key)
        if p is None:
            if len(_cache) > 64:
                _cache.clear()
            p = _cache[key] = FFTPlan(kind, order, batch, device)
        return p
