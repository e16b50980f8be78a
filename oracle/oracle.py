"""ctypes front-end for the CPU restatement in neo_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline. The product
(neo-dsp_amd/, include/) never imports or links it.

Parity status: pinned by the reference's own known-answer, round-trip and
identity tests (tests/test_oracle.py) plus float64 numpy truth; the reference
itself is unbuildable here (FetchContent-only deps), so there is no oracle/_ref.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_sz = ctypes.c_size_t


def build(force: bool = False) -> str:
    srcs = [os.path.join(_HERE, f) for f in ("neo_oracle.c", "neo_oracle_f64.c")]
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        L.oracle_fft_c2c.argtypes = [ctypes.c_int, ctypes.c_int, _f32p]
        L.oracle_fft_c2c_batch.argtypes = [ctypes.c_int, ctypes.c_int, _f32p, _sz]
        L.oracle_twiddle_lut.argtypes = [ctypes.c_int, ctypes.c_int, _f32p]
        L.oracle_rfft.argtypes = [ctypes.c_int, _f32p, _f32p]
        L.oracle_irfft.argtypes = [ctypes.c_int, _f32p, _f32p]
        L.oracle_rfft_deinterleave.argtypes = [_sz, _f32p, _f32p, _f32p]
        L.oracle_multiply_add.argtypes = [_f32p, _f32p, _f32p, _f32p, _sz]
        L.oracle_split_multiply_add.argtypes = [_f32p] * 8 + [_sz]
        L.oracle_normalize_impulse.argtypes = [_f32p, _sz, _sz]
        L.oracle_num_partitions.argtypes = [_sz, _sz]
        L.oracle_num_partitions.restype = _sz
        L.oracle_uniform_partition.argtypes = [_f32p, _sz, _sz, _sz, _f32p]
        L.oracle_upols_create.argtypes = [_sz, _sz, _f32p, ctypes.c_int]
        L.oracle_upols_create.restype = ctypes.c_void_p
        L.oracle_upols_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_upols_process.argtypes = [ctypes.c_void_p, _f32p]
        L.oracle_upols_run.argtypes = [ctypes.c_void_p, _f32p, _sz]
        L.oracle_overlap_save_identity.argtypes = [_sz, _f32p, _sz]
        L.oracle_dense_convolve.argtypes = [_f32p, _f32p, _f32p, _sz, _sz, _sz, _sz, ctypes.c_int]
        L.oracle_noise.argtypes = [ctypes.c_uint64, _f32p, _sz]
        L.oracle_upola2_create.argtypes = [_sz, _sz, _f32p]
        L.oracle_upola2_create.restype = ctypes.c_void_p
        L.oracle_upola2_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_upola2_process.argtypes = [ctypes.c_void_p, _f32p, _sz]
        L.oracle_hann.argtypes = [_sz, _f32p]
        L.oracle_stft_frames.argtypes = [_sz, _sz, _sz]
        L.oracle_stft_frames.restype = _sz
        L.oracle_stft.argtypes = [_f32p, _sz, _sz, _sz, _sz, _sz, _f32p, _f32p]
        L.oracle_fft_c2c_f64.argtypes = [ctypes.c_int, ctypes.c_int, _f64p]
        L.oracle_rfft_f64.argtypes = [ctypes.c_int, _f64p, _f64p]
        L.oracle_irfft_f64.argtypes = [ctypes.c_int, _f64p, _f64p]
        L.oracle_fft_convolve_f64.argtypes = [_f64p, _sz, _f64p, _sz, _f64p]
        L.oracle_direct_convolve_f64.argtypes = [_f64p, _sz, _f64p, _sz, _f64p]
        L.oracle_upola_create.argtypes = [_sz, _sz, _f32p, ctypes.c_int]
        L.oracle_upola_create.restype = ctypes.c_void_p
        L.oracle_dense_convolve_method.argtypes = [_f32p, _f32p, _f32p, _sz, _sz, _sz, _sz, ctypes.c_int, ctypes.c_int]
        L.oracle_overlap_add_identity.argtypes = [_sz, _f32p, _sz]
        L.oracle_overlap_stage.argtypes = [ctypes.c_int, _sz, _sz, ctypes.c_void_p, _f32p, _sz]
        L.oracle_fft_convolve.argtypes = [_f32p, _sz, _f32p, _sz, _f32p]
        L.oracle_direct_convolve.argtypes = [_f32p, _sz, _f32p, _sz, _f32p]
        _lib = L
    return _lib


def _cf(x: np.ndarray) -> np.ndarray:
    """complex64 array -> contiguous float32 view (interleaved re,im)."""
    return np.ascontiguousarray(x, dtype=np.complex64).view(np.float32)


def noise(seed: int, n: int) -> np.ndarray:
    """splitmix64 -> U[-1,1) float32 (SURVEY §8c generator)."""
    out = np.empty(n, dtype=np.float32)
    lib().oracle_noise(seed, out, n)
    return out


def noise_np(seed: int, n: int) -> np.ndarray:
    """numpy restatement of noise() (same bits), for host-side input generation."""
    gamma = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        s = np.uint64(seed) + gamma * np.arange(1, n + 1, dtype=np.uint64)
        z = s
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    r = (z >> np.uint64(40)).astype(np.float32)
    return r * np.float32(2.0 / 16777216.0) - np.float32(1.0)


def fft(x: np.ndarray, direction: int = -1) -> np.ndarray:
    """c2c_dit2_plan (unnormalized); x is [..., N] complex64, transforms along the last axis."""
    x = np.array(x, dtype=np.complex64, copy=True)
    n = x.shape[-1]
    order = n.bit_length() - 1
    if 1 << order != n:
        raise ValueError("power-of-two sizes only")
    flat = np.ascontiguousarray(x.reshape(-1, n))
    buf = flat.view(np.float32).reshape(-1)
    rc = lib().oracle_fft_c2c_batch(order, direction, buf, flat.shape[0])
    if rc:
        raise RuntimeError(f"oracle fft failed rc={rc}")
    return buf.view(np.complex64).reshape(x.shape)


def ifft(x: np.ndarray) -> np.ndarray:
    return fft(x, +1)


def twiddle_lut(order: int, direction: int) -> np.ndarray:
    out = np.empty(1 << order, dtype=np.float32)
    lib().oracle_twiddle_lut(order, direction, out)
    return out.view(np.complex64)


def rfft(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = x.shape[-1]
    order = n.bit_length() - 1
    flat = x.reshape(-1, n)
    out = np.empty((flat.shape[0], n // 2 + 1), dtype=np.complex64)
    for i in range(flat.shape[0]):
        o = np.empty(2 * (n // 2 + 1), dtype=np.float32)
        lib().oracle_rfft(order, np.ascontiguousarray(flat[i]), o)
        out[i] = o.view(np.complex64)
    return out.reshape(x.shape[:-1] + (n // 2 + 1,))


def irfft(X: np.ndarray, n: int) -> np.ndarray:
    X = np.ascontiguousarray(X, dtype=np.complex64)
    order = n.bit_length() - 1
    flat = X.reshape(-1, X.shape[-1])
    out = np.empty((flat.shape[0], n), dtype=np.float32)
    for i in range(flat.shape[0]):
        o = np.empty(n, dtype=np.float32)
        lib().oracle_irfft(order, _cf(flat[i, : n // 2 + 1]), o)
        out[i] = o
    return out.reshape(X.shape[:-1] + (n,))


def rfft_deinterleave(dft: np.ndarray):
    n = dft.shape[0]
    x = np.empty(2 * (n // 2 + 1), dtype=np.float32)
    y = np.empty(2 * (n // 2 + 1), dtype=np.float32)
    lib().oracle_rfft_deinterleave(n, _cf(dft), x, y)
    return x.view(np.complex64), y.view(np.complex64)


def multiply_add(x, y, z) -> np.ndarray:
    out = np.empty(2 * len(x), dtype=np.float32)
    lib().oracle_multiply_add(_cf(x), _cf(y), _cf(z), out, len(x))
    return out.view(np.complex64)


def split_multiply_add(xr, xi, yr, yi, zr, zi):
    n = len(xr)
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    outr = np.empty(n, np.float32)
    outi = np.empty(n, np.float32)
    lib().oracle_split_multiply_add(f(xr), f(xi), f(yr), f(yi), f(zr), f(zi), outr, outi, n)
    return outr, outi


def normalize_impulse(ir: np.ndarray) -> np.ndarray:
    a = np.array(ir, dtype=np.float32, copy=True)
    if a.ndim == 1:
        lib().oracle_normalize_impulse(a, 1, a.shape[0])
    else:
        lib().oracle_normalize_impulse(a, a.shape[0], a.shape[1])
    return a


def num_partitions(length: int, block: int) -> int:
    return int(lib().oracle_num_partitions(length, block))


def uniform_partition(ir: np.ndarray, block: int) -> np.ndarray:
    ir = np.ascontiguousarray(np.atleast_2d(ir), dtype=np.float32)
    C, L = ir.shape
    P = num_partitions(L, block)
    out = np.empty(C * P * (block + 1) * 2, dtype=np.float32)
    rc = lib().oracle_uniform_partition(ir, C, L, block, out)
    if rc:
        raise RuntimeError("oracle uniform_partition failed")
    return out.view(np.complex64).reshape(C, P, block + 1)


class Upols:
    """upols_convolver<complex<float>> (split_upols_convolver with split=True; upola_convolver
    with ola=True), one channel."""

    def __init__(self, filt: np.ndarray, split: bool = False, ola: bool = False):
        filt = np.ascontiguousarray(filt, dtype=np.complex64)
        self.P, self.bins = filt.shape
        self.B = self.bins - 1
        create = lib().oracle_upola_create if ola else lib().oracle_upols_create
        self._h = create(self.P, self.bins, _cf(filt).reshape(-1), int(split))

    def __call__(self, block: np.ndarray) -> np.ndarray:
        b = np.array(block, dtype=np.float32, copy=True)
        lib().oracle_upols_process(self._h, b)
        return b

    def run(self, signal: np.ndarray) -> np.ndarray:
        s = np.array(signal, dtype=np.float32, copy=True)
        assert s.shape[0] % self.B == 0
        lib().oracle_upols_run(self._h, s, s.shape[0] // self.B)
        return s

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_upols_destroy(self._h)
            self._h = None


class Upola2:
    """upola_convolver_v2<complex<float>> (overlap_add_convolver.hpp:20-136), one channel:
    __call__ takes any number of samples (sub-block input), in place on a copy."""

    def __init__(self, filt: np.ndarray):
        filt = np.ascontiguousarray(filt, dtype=np.complex64)
        self.P, self.bins = filt.shape
        self.B = self.bins - 1
        self._h = lib().oracle_upola2_create(self.P, self.bins, _cf(filt).reshape(-1))

    def __call__(self, samples: np.ndarray) -> np.ndarray:
        b = np.array(samples, dtype=np.float32, copy=True)
        if lib().oracle_upola2_process(self._h, b, b.shape[0]):
            raise RuntimeError("oracle upola_convolver_v2 failed")
        return b

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_upola2_destroy(self._h)
            self._h = None


def overlap_save_identity(signal: np.ndarray, block: int) -> np.ndarray:
    s = np.array(signal, dtype=np.float32, copy=True)
    lib().oracle_overlap_save_identity(block, s, s.shape[0] // block)
    return s


def dense_convolve(signal: np.ndarray, partitions: np.ndarray, threads: int = 1, method: str = "upols") -> np.ndarray:
    """dense_convolve<upols_convolver | upola_convolver> on already-partitioned filters [C][P][B+1]."""
    signal = np.ascontiguousarray(signal, dtype=np.float32)
    C, N = signal.shape
    _, P, bins = partitions.shape
    out = np.empty_like(signal)
    rc = lib().oracle_dense_convolve_method(signal, out, _cf(partitions).reshape(-1), C, N, P, bins - 1, threads,
                                            int(method == "upola"))
    if rc:
        raise RuntimeError("oracle dense_convolve failed")
    return out


def overlap_transform_size(block: int, filter_size: int) -> int:
    """2^next_order(B + F - 1) (overlap_save.hpp:53, overlap_add.hpp:43-46)."""
    n = 1
    while n < block + filter_size - 1:
        n *= 2
    return n


def overlap_stage(kind: str, signal: np.ndarray, block: int, filter_size: int, G=None) -> np.ndarray:
    """The standalone overlap_save / overlap_add stage (kind "save" / "add") over consecutive
    blocks of a 1-D signal, transform size overlap_transform_size(B, F), callback = multiply the
    n/2 + 1 bins by G (None: no-op)."""
    s = np.array(signal, dtype=np.float32, copy=True)
    g = None
    if G is not None:
        g = np.ascontiguousarray(G, dtype=np.complex64)
        assert g.shape == (overlap_transform_size(block, filter_size) // 2 + 1,)
    rc = lib().oracle_overlap_stage(0 if kind == "save" else 1, block, filter_size,
                                    None if g is None else g.ctypes.data_as(ctypes.c_void_p), s, s.shape[0] // block)
    if rc:
        raise RuntimeError("oracle overlap stage failed")
    return s


def overlap_add_identity(signal: np.ndarray, block: int) -> np.ndarray:
    s = np.array(signal, dtype=np.float32, copy=True)
    lib().oracle_overlap_add_identity(block, s, s.shape[0] // block)
    return s


def fft_convolve(signal: np.ndarray, patch: np.ndarray) -> np.ndarray:
    """fft_convolve (fft_convolver.hpp:19-93), full mode."""
    a = np.ascontiguousarray(signal, dtype=np.float32)
    b = np.ascontiguousarray(patch, dtype=np.float32)
    if a.size == 0 or b.size == 0:
        return np.zeros(0, np.float32)
    out = np.empty(a.size + b.size - 1, np.float32)
    if lib().oracle_fft_convolve(a, a.size, b, b.size, out):
        raise RuntimeError("oracle fft_convolve failed")
    return out


def direct_convolve(signal: np.ndarray, patch: np.ndarray) -> np.ndarray:
    """direct_convolve (direct_convolve.hpp:14-56), full mode."""
    a = np.ascontiguousarray(signal, dtype=np.float32)
    b = np.ascontiguousarray(patch, dtype=np.float32)
    out = np.empty(a.size + b.size - 1, np.float32)
    lib().oracle_direct_convolve(a, a.size, b, b.size, out)
    return out


# ---------------------------------------------------------------- double precision
def fft_f64(x: np.ndarray, direction: int = -1) -> np.ndarray:
    """fft_plan<complex<double>> over the last axis (unnormalized; direction -1 / +1)."""
    a = np.array(x, dtype=np.complex128, copy=True)
    n = a.shape[-1]
    order = n.bit_length() - 1
    flat = a.reshape(-1, n)
    for i in range(flat.shape[0]):
        row = np.ascontiguousarray(flat[i]).view(np.float64)
        if lib().oracle_fft_c2c_f64(order, direction, row):
            raise RuntimeError("oracle fft_f64 failed")
        flat[i] = row.view(np.complex128)
    return flat.reshape(a.shape)


def rfft_f64(x: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(x, dtype=np.float64)
    n = a.shape[-1]
    out = np.empty(n // 2 + 1, np.complex128)
    o = out.view(np.float64)
    lib().oracle_rfft_f64(n.bit_length() - 1, a, o)
    return out


def irfft_f64(X: np.ndarray, n: int) -> np.ndarray:
    a = np.ascontiguousarray(X, dtype=np.complex128).view(np.float64)
    out = np.empty(n, np.float64)
    lib().oracle_irfft_f64(n.bit_length() - 1, a, out)
    return out


def fft_convolve_f64(signal: np.ndarray, patch: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(signal, dtype=np.float64)
    b = np.ascontiguousarray(patch, dtype=np.float64)
    if a.size == 0 or b.size == 0:
        return np.zeros(0, np.float64)
    out = np.empty(a.size + b.size - 1, np.float64)
    if lib().oracle_fft_convolve_f64(a, a.size, b, b.size, out):
        raise RuntimeError("oracle fft_convolve_f64 failed")
    return out


def direct_convolve_f64(signal: np.ndarray, patch: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(signal, dtype=np.float64)
    b = np.ascontiguousarray(patch, dtype=np.float64)
    out = np.empty(a.size + b.size - 1, np.float64)
    lib().oracle_direct_convolve_f64(a, a.size, b, b.size, out)
    return out


# ---------------------------------------------------------------- STFT
def hann(size: int) -> np.ndarray:
    """hann_window (math/windowing.hpp:29-41) in float over `size` points."""
    w = np.empty(size, np.float32)
    lib().oracle_hann(size, w)
    return w


def stft_frames(length: int, frame: int, overlap: int) -> int:
    return int(lib().oracle_stft_frames(length, frame, overlap))


def stft(x: np.ndarray, frame: int, transform: int, overlap: int, window: np.ndarray) -> np.ndarray:
    """stft_plan::operator() (stft.hpp:56-99): [C][L] -> [C][F][N/2+1] complex64."""
    x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
    C, L = x.shape
    N = 1 << (int(transform) - 1).bit_length()
    F = stft_frames(L, frame, overlap)
    out = np.empty(C * F * (N // 2 + 1) * 2, np.float32)
    w = np.ascontiguousarray(window, dtype=np.float32)
    if lib().oracle_stft(x, C, L, frame, transform, overlap, w, out):
        raise RuntimeError("oracle stft failed")
    return out.view(np.complex64).reshape(C, F, N // 2 + 1)


# ---------------------------------------------------------------------------------------
# cpu_baseline only (bench.py): the reference's SIMD MAC restated (neo_baseline.c), a separate
# library so that liboracle.so stays the exact scalar oracle
_BLIB = os.path.join(_HERE, "liboracle_simd.so")
_blib = None
SIMD_NAMES = {2: "avx512f (xsimd batch<complex<float>>, 16 complex per op, restated)",
              1: "avx2+fma (xsimd batch<complex<float>>, 8 complex per op, restated)", 0: "scalar"}


def baseline_lib():
    global _blib
    if _blib is None:
        srcs = [os.path.join(_HERE, f) for f in ("neo_baseline.c", "neo_oracle.c", "neo_oracle_f64.c")]
        if not os.path.exists(_BLIB) or os.path.getmtime(_BLIB) < max(os.path.getmtime(f) for f in srcs):
            subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle_simd.so"])
        L = ctypes.CDLL(_BLIB)
        L.baseline_dense_convolve.argtypes = [_f32p, _f32p, _f32p, _sz, _sz, _sz, _sz, ctypes.c_int, ctypes.c_int]
        L.baseline_simd_level.restype = ctypes.c_int
        _blib = L
    return _blib


def simd_level() -> int:
    """2 = AVX-512F, 1 = AVX2 + FMA, 0 = scalar: what the baseline's MAC uses on this host."""
    return int(baseline_lib().baseline_simd_level())


def dense_convolve_simd(signal: np.ndarray, partitions: np.ndarray, threads: int = 1, level: int = -1) -> np.ndarray:
    """dense_convolve<upols_convolver> with the reference's SIMD interleaved MAC (timing
    baseline; matches dense_convolve within float rounding, not bit for bit)."""
    signal = np.ascontiguousarray(signal, dtype=np.float32)
    C, N = signal.shape
    _, P, bins = partitions.shape
    out = np.empty_like(signal)
    rc = baseline_lib().baseline_dense_convolve(signal, out, _cf(partitions).reshape(-1), C, N, P, bins - 1,
                                                threads, level)
    if rc:
        raise RuntimeError("baseline dense_convolve failed")
    return out
