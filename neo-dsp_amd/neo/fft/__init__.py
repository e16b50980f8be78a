"""neo.fft on MI355X — mirrors the reference's Python facade.

Reference: extra/python/src/neo/fft/__init__.py:22-31 (fft/ifft) over
extra/python/src/main.cpp:129-167 (power-of-two sizes only, RuntimeError
otherwise; unnormalized transforms scaled per `norm`). Here every transform runs
on the GPU through libneo_hip.so (include/neo_hip.h); there is no CPU path.

Extensions over the reference (documented in INTEGRATION.md): arrays of rank > 1
are transformed along the last axis as one batched launch; torch CUDA tensors are
transformed in device memory on torch's current stream; rfft/irfft are exposed.
Plans are cached per (kind, order, batch, device) instead of rebuilt per call
(main.cpp:147).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _native
from ._plan import FFTPlan, get_plan

__all__ = ["fft", "ifft", "rfft", "irfft", "rfftfreq", "stft", "stft_num_frames", "FFTPlan", "get_plan", "next_order",
           "size", "max_order"]

_NORMS = ("backward", "ortho", "forward")


def max_order() -> int:
    return int(_native.load().neo_hip_fft_max_order())


def size(order: int) -> int:
    """neo::fft::size (src/neo/fft/order.hpp:26-30)."""
    return 1 << order


def next_order(n: int) -> int:
    """neo::fft::next_order = log2(bit_ceil(n)) (src/neo/fft/order.hpp:32-37)."""
    n = int(n)
    return 0 if n <= 1 else (n - 1).bit_length()


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "is_cuda")


def _check_size(n: int) -> int:
    if n < 1 or (n & (n - 1)) != 0:
        raise RuntimeError(f"unsupported size: {n}")  # main.cpp:137-139
    return n.bit_length() - 1


def _fit(x: np.ndarray, n: int) -> np.ndarray:
    if x.shape[-1] == n:
        return x
    if x.shape[-1] > n:
        return x[..., :n]
    pad = [(0, 0)] * (x.ndim - 1) + [(0, n - x.shape[-1])]
    return np.pad(x, pad)


def _scale(norm: str, n: int, inverse: bool) -> float:
    if norm not in _NORMS:
        raise ValueError(f"invalid norm {norm!r}")
    if norm == "ortho":
        return 1.0 / np.sqrt(n)
    if (norm == "backward") == inverse:
        return 1.0 / n
    return 1.0


def _c2c(x, n, norm, direction):
    inverse = direction > 0
    if _is_torch(x):
        import torch

        if x.dtype not in (torch.complex64, torch.complex128):
            raise TypeError("device tensors: complex64 or complex128")
        if n is not None and n != x.shape[-1]:
            raise ValueError("device tensors: n must equal the last dimension")
        n = x.shape[-1]
        order = _check_size(n)
        xc = x.resolve_conj().contiguous()
        out = torch.empty_like(xc)
        batch = xc.numel() // n if n else 0
        kind = _native.C2C | (_native.F64 if x.dtype == torch.complex128 else 0)
        plan = get_plan(kind, order, batch, xc.device.index or 0)
        plan.execute_device(xc.data_ptr(), out.data_ptr(), direction,
                            torch.cuda.current_stream(xc.device).cuda_stream)
        s = _scale(norm, n, inverse)
        return out if s == 1.0 else out.mul_(s)
    a = np.asarray(x)
    # the reference binds complex<float> then complex<double> (main.cpp:248-252): an exact
    # complex64 / complex128 array picks its own overload, anything else is converted to
    # the first one (pybind11's second, converting pass), i.e. complex64
    if a.dtype != np.complex128 and a.dtype != np.complex64:
        if a.dtype.kind not in "fciub":
            raise TypeError(f"unsupported dtype {a.dtype}")
        a = a.astype(np.complex64)
    if a.ndim == 0:
        raise ValueError("input must have at least one dimension")
    f64 = a.dtype == np.complex128
    n = a.shape[-1] if n is None else int(n)
    order = _check_size(n)
    a = np.ascontiguousarray(_fit(a, n))
    batch = a.size // n
    out = np.empty_like(a)
    plan = get_plan(_native.C2C | (_native.F64 if f64 else 0), order, batch, 0)
    plan.execute_host(a, out, direction)
    s = _scale(norm, n, inverse)
    if s != 1.0:
        out *= (np.float64 if f64 else np.float32)(s)
    return out


def fft(x, n=None, norm="backward"):
    """1-D forward DFT along the last axis (e^{-2 pi i nk/N})."""
    return _c2c(x, n, norm, -1)


def ifft(x, n=None, norm="backward"):
    """1-D inverse DFT along the last axis; `backward` norm scales by 1/N."""
    return _c2c(x, n, norm, +1)


def rfft(x, n=None, norm="backward"):
    """Real-input forward DFT: N/2+1 bins (fallback_rfft_plan semantics, packed on the GPU).
    float64 input runs the double plan and returns complex128; anything else float32."""
    a = np.asarray(x)
    f64 = a.dtype == np.float64
    a = np.ascontiguousarray(a, dtype=np.float64 if f64 else np.float32)
    n = a.shape[-1] if n is None else int(n)
    order = _check_size(n)
    a = np.ascontiguousarray(_fit(a, n))
    batch = a.size // n
    out = np.empty(a.shape[:-1] + (n // 2 + 1,), dtype=np.complex128 if f64 else np.complex64)
    get_plan(_native.R2C | (_native.F64 if f64 else 0), order, batch, 0).execute_host(a, out, -1)
    s = _scale(norm, n, False)
    if s != 1.0:
        out *= (np.float64 if f64 else np.float32)(s)
    return out


def irfft(x, n=None, norm="backward"):
    """Inverse of rfft: reads N/2+1 bins (Im of DC/Nyquist ignored), returns N reals
    (float64 for complex128 input)."""
    a = np.asarray(x)
    f64 = a.dtype == np.complex128
    a = np.asarray(a, dtype=np.complex128 if f64 else np.complex64)
    n = 2 * (a.shape[-1] - 1) if n is None else int(n)
    order = _check_size(n)
    need = n // 2 + 1
    a = np.ascontiguousarray(_fit(a, need))
    batch = a.size // need
    out = np.empty(a.shape[:-1] + (n,), dtype=np.float64 if f64 else np.float32)
    get_plan(_native.C2R | (_native.F64 if f64 else 0), order, batch, 0).execute_host(a, out, +1)
    s = _scale(norm, n, True)
    if s != 1.0:
        out *= (np.float64 if f64 else np.float32)(s)
    return out


def rfftfreq(n: int, d: float = 1.0) -> np.ndarray:
    """Bin frequencies, the reference's definition (src/neo/fft/rfftfreq.hpp:12-30,
    main.cpp:211-222): n values i * (1/d) * (1/n), i < n. Index arithmetic on the host,
    not a transform (nothing here runs on the GPU)."""
    n = int(n)
    fs = 1.0 / float(d)
    inv = 1.0 / float(n) if n else 0.0
    return np.arange(n, dtype=np.float64) * fs * inv


def stft_num_frames(length: int, frame_size: int, overlap_size: int) -> int:
    """detail::num_sftf_frames (src/neo/fft/stft.hpp:21-25)."""
    f = ctypes.c_int64()
    _native.check(_native.load().neo_hip_stft_num_frames(int(length), int(frame_size), int(overlap_size),
                                                         ctypes.byref(f)))
    return f.value


def stft(x, frame_size: int, transform_size=None, overlap_size=None, window="hann", device: int = 0):
    """stft_plan / stft (src/neo/fft/stft.hpp:40-125) on the GPU: x [C][L] (or [L]) ->
    [C][F][N/2+1], N = 2^next_order(transform_size). `stft(x, n)` is the reference's
    stft(x, window_size): frame = transform = n, overlap n/2, hann window. `window`:
    "hann", "rectangular", an array of N values or a callable window(index, size) (the
    stft_options::window signature, evaluated over N like fill_window)."""
    a = np.asarray(x)
    f64 = a.dtype == np.float64
    rt = np.float64 if f64 else np.float32
    a = np.ascontiguousarray(np.atleast_2d(a), dtype=rt)
    C, L = a.shape
    frame = int(frame_size)
    transform = frame if transform_size is None else int(transform_size)
    overlap = frame // 2 if overlap_size is None else int(overlap_size)
    N = 1 << next_order(transform)
    if isinstance(window, str):
        if window == "hann":
            w = None  # computed by the library in the transform's precision
        elif window == "rectangular":
            w = np.ones(N, rt)
        else:
            raise ValueError(f"unknown window {window!r}")
    elif callable(window):
        w = np.array([window(i, N) for i in range(N)], dtype=rt)
    else:
        w = np.ascontiguousarray(window, dtype=rt)
        if w.shape != (N,):
            raise ValueError(f"window must have {N} values (the transform size)")
    F = stft_num_frames(L, frame, overlap)
    out = np.empty((C, F, N // 2 + 1), np.complex128 if f64 else np.complex64)
    fn = _native.load().neo_hip_stft_f64 if f64 else _native.load().neo_hip_stft
    wp = None if w is None else w.ctypes.data_as(ctypes.c_void_p)
    _native.check(fn(a.ctypes.data_as(ctypes.c_void_p), C, L, frame, transform, overlap, wp,
                     out.ctypes.data_as(ctypes.c_void_p), 0, int(device)))
    return out
