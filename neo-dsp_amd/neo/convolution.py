"""neo.convolution on MI355X: UPOLS convolvers, uniform_partition, normalize_impulse.

Mirrors the reference's C++ convolution API (the reference binds no UPOLS in
Python; extra/python/src/main.cpp:227-234 only lists the `upols` method enum):
  - uniform_partition      src/neo/convolution/uniform_partition.hpp:12-26
  - normalize_impulse      src/neo/convolution/normalize_impulse.hpp:11-33
  - upols_convolver        src/neo/convolution/dense_convolver.hpp:19-20 +
                           uniform_partitioned_convolver.hpp:13-65
  - split_upols_convolver  dense_convolver.hpp:38-42 (same math, SoA on the CPU;
                           one device layout here)
  - upola_convolver        dense_convolver.hpp:23-24 (overlap_add.hpp:76-106 stage)
  - upola_convolver_v2     dense_convolver.hpp:28 (overlap_add_convolver.hpp:20-136,
                           sub-block input)
  - dense_convolve         extra/plugin/src/dsp/DenseConvolution.hpp:39-70
Everything runs on the GPU through libneo_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native

__all__ = [
    "num_partitions",
    "host_register",
    "host_unregister",
    "uniform_partition",
    "normalize_impulse",
    "UpolsConvolver",
    "upols_convolver",
    "split_upols_convolver",
    "OverlapStage",
    "UpolsGroup",
    "overlap_save",
    "overlap_add",
    "upola_convolver",
    "split_upola_convolver",
    "upola_convolver_v2",
    "dense_convolve",
    "fft_convolve",
    "direct_convolve",
    "convolve",
]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "is_cuda")


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return a.ctypes.data_as(ctypes.c_void_p)


def _producer_join(t) -> None:
    """A device tensor handed to a synchronous setup call (filter, impulse, normalize, partition)
    is complete first: torch's current stream is its producer. The library orders such an input
    after the null stream (torch's default stream) itself, with a marker event, never after the
    whole device (a resident latency-mode kernel on another handle); a side stream
    (`with torch.cuda.stream(s)`) is synchronized here, that stream alone."""
    import torch

    s = torch.cuda.current_stream(t.device)
    if s.cuda_stream != 0:
        s.synchronize()


def num_partitions(length: int, block: int) -> int:
    """P = ceil(L / B) (stft.hpp:21-25 with overlap 0; clamped to 1 for L < B)."""
    p = ctypes.c_int64()
    _native.check(_native.load().neo_hip_num_partitions(int(length), int(block), ctypes.byref(p)))
    return p.value


def level_plan(partitions: int) -> dict:
    """The streaming level plan of a convolver with `partitions` partitions
    (neo_hip_upols_level_plan; no device needed): the block step takes [0, a0), Toeplitz
    level l a window of T[l] blocks over the band [a[l], b[l]), and nseg far segments of
    128 partitions from 256."""
    L = _native.load()
    a0, nl, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    T, a, b = (ctypes.c_int * 8)(), (ctypes.c_int * 8)(), (ctypes.c_int * 8)()
    _native.check(L.neo_hip_upols_level_plan(int(partitions), ctypes.byref(a0), ctypes.byref(nl), T, a, b,
                                             ctypes.byref(ns)))
    n = nl.value
    return {"a0": a0.value, "T": list(T[:n]), "a": list(a[:n]), "b": list(b[:n]), "nseg": ns.value}


def part_plan(channels: int, block: int, partitions: int, step_group: int, uniform: bool = False) -> dict:
    """The background plan of step groups of `step_group` blocks (neo_hip_upols_part_plan; no
    device needed): per Toeplitz level the window offset phi, the cycle length in step groups,
    per background level (T >= 2 step_group) the unit cuts of each window of the cycle
    ({level: [[T / G cuts of window k], ...]}) and the predicted background bytes per step group
    of the cycle; uniform: equal parts, no offsets."""
    if step_group < 2:
        raise ValueError("part_plan: step groups of >= 2 blocks")
    L = _native.load()
    lp = level_plan(partitions)
    phi, cyc, nc = (ctypes.c_int * 8)(), ctypes.c_int(), ctypes.c_int()
    loads = (ctypes.c_double * 512)()
    args = (int(channels), int(block), int(partitions), int(step_group), int(uniform), phi, ctypes.byref(cyc))
    _native.check(L.neo_hip_upols_part_plan(*args, None, 0, ctypes.byref(nc), loads, 512))
    cuts = (ctypes.c_int * max(1, nc.value))()
    _native.check(L.neo_hip_upols_part_plan(*args, cuts, nc.value, ctypes.byref(nc), loads, 512))
    flat, out, i = list(cuts[:nc.value]), {}, 0
    for l, T in enumerate(lp["T"]):
        if T < 2 * step_group:
            continue  # in the block launches
        Tg = T // step_group
        out[l] = [flat[i + k:i + k + Tg] for k in range(0, cyc.value, Tg)]
        i += cyc.value
    return {"phi": list(phi[:len(lp["T"])]), "cycle": cyc.value, "cuts": out, "loads": list(loads[:cyc.value])}


def host_register(array: np.ndarray) -> np.ndarray:
    """Page-lock a host array in place (neo_hip_host_register) so that host-buffer calls
    (UpolsConvolver.__call__) read and write it over PCIe without staging; call
    host_unregister before the array is freed."""
    if not (isinstance(array, np.ndarray) and array.flags.c_contiguous):
        raise TypeError("host_register takes a C-contiguous ndarray")
    _native.check(_native.load().neo_hip_host_register(_ptr(array), array.nbytes))
    return array


def host_unregister(array: np.ndarray) -> None:
    _native.check(_native.load().neo_hip_host_unregister(_ptr(array)))


def memory_info(device: int = 0) -> dict:
    """Device memory the library holds for convolver handles on `device` (neo_hip_memory_info):
    bytes reserved in its cached chunks and bytes in use by live handles."""
    r, u = ctypes.c_int64(), ctypes.c_int64()
    _native.check(_native.load().neo_hip_memory_info(device, ctypes.byref(r), ctypes.byref(u)))
    return {"reserved": r.value, "in_use": u.value}


def memory_trim(device: int = 0) -> None:
    """Return every cached chunk no handle uses to the driver (neo_hip_memory_trim)."""
    _native.check(_native.load().neo_hip_memory_trim(device))


def uniform_partition(impulse_response, block_size: int, device: int = 0):
    """[C][L] float32 -> [C][P][B+1] complex64: rfft_2B of each zero-padded B-sample partition.
    A CUDA tensor gives a CUDA tensor on its device (no host copies)."""
    if _is_torch(impulse_response) and impulse_response.is_cuda:
        import torch

        t = impulse_response
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise TypeError("uniform_partition takes a contiguous float32 tensor")
        C, L = (1, t.shape[0]) if t.dim() == 1 else tuple(t.shape)
        P = num_partitions(L, block_size)
        out = torch.empty((C, P, block_size + 1), dtype=torch.complex64, device=t.device)
        _producer_join(t)
        _native.check(_native.load().neo_hip_uniform_partition(ctypes.c_void_p(t.data_ptr()), C, L, int(block_size),
                                                               ctypes.c_void_p(out.data_ptr()), 1, t.device.index or 0))
        return out
    ir = np.ascontiguousarray(np.atleast_2d(np.asarray(impulse_response, dtype=np.float32)))
    C, L = ir.shape
    P = num_partitions(L, block_size)
    out = np.empty((C, P, block_size + 1), dtype=np.complex64)
    _native.check(_native.load().neo_hip_uniform_partition(_ptr(ir), C, L, int(block_size), _ptr(out), 0, int(device)))
    return out


def normalize_impulse(impulse_response, device: int = 0):
    """In place: scale every channel by min_c 1/sqrt(sum(ir[c]^2)), rounded exactly like the
    reference's sequential float sum. Accepts a float32 ndarray (rank 1 or 2) or CUDA tensor."""
    if _is_torch(impulse_response):
        t = impulse_response
        C, L = (1, t.shape[0]) if t.dim() == 1 else tuple(t.shape)
        _producer_join(t)
        _native.check(_native.load().neo_hip_normalize_impulse(ctypes.c_void_p(t.data_ptr()), C, L, 1,
                                                               t.device.index or 0))
        return t
    a = impulse_response
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
        raise TypeError("normalize_impulse works in place on a C-contiguous float32 array")
    C, L = (1, a.shape[0]) if a.ndim == 1 else a.shape
    _native.check(_native.load().neo_hip_normalize_impulse(_ptr(a), C, L, 0, int(device)))
    return a


class UpolsConvolver:
    """C independent UPOLS convolvers stepped together (one launch pair per block).

    State lives in HBM: filter [C][P][B] and FDL [C][P][B] (packed bins),
    previous block [C][B]. Blocks are processed in place, zero latency
    (output block t corresponds to input block t, overlap_save.hpp:84-112).
    """

    OPTION_DEFAULTS = {"fused": -1, "split_workgroups": 0, "batch_blocks": 0, "batch_bins": 0, "levels": -1,
                       "far_level": -1, "far_group": 0, "toep_split": 0, "step_group": 0,
                       "far_phase2": 0}

    def __init__(self, channels: int, block_size: int, partitions: int, device: int = 0, method: str = "upols",
                 options: dict | None = None):
        """`options` (neo_hip_upols_create_ex): explicit code-path choices instead of the
        shape-based defaults — fused (-1 auto / 0 / 1), split_workgroups (0 auto),
        batch_blocks (0 auto / 2..32), batch_bins (0 auto / 1 / 2), levels (-1 auto / 0 / 1),
        far_level (-1 auto / 0 Toeplitz window of 128 blocks / 1 partition-axis transform with stored spectra /
        2 the transform recomputed every window, for p >= 256),
        far_group (0 auto / 1..4 windows per far phase-1 pass over the stored segment spectra),
        toep_split (0 auto / 1 / 2 window parts per unit of the 32-block Toeplitz level),
        step_group (0 auto / 1 one launch per block / 2 or 4: the block of every call alone on the
        caller's stream, the level slices of G calls as one launch on a background stream),
        far_phase2 (G = 1: 0 auto / 1 one workgroup per unit / 2 the fresh transform one step
        before the products). Every choice gives the same results up to float summation order."""
        lib = _native.load()
        h = ctypes.c_void_p()
        methods = {"upols": 0, "upola": 1, "upola_v2": 2}
        if method not in methods:
            raise ValueError(f"method must be 'upols', 'upola' or 'upola_v2', got {method!r}")
        opts = dict(self.OPTION_DEFAULTS)
        for k, v in (options or {}).items():
            if k not in opts:
                raise ValueError(f"unknown convolver option {k!r}")
            opts[k] = int(v)
        o = _native.UpolsOpts(**opts)
        _native.check(lib.neo_hip_upols_create_ex(int(channels), int(block_size), int(partitions), int(device),
                                                  methods[method], ctypes.byref(o), ctypes.byref(h)))
        self._h = h
        self.channels, self.block_size, self.partitions, self.device = channels, block_size, partitions, device
        self.method = method

    # -- setup ------------------------------------------------------------
    def filter(self, partitions) -> None:
        """uniform_partitioned_convolver::filter(): [C][P][B+1] complex64 (host array or
        CUDA tensor); resets FDL, window and write position."""
        if _is_torch(partitions):
            _producer_join(partitions)
            _native.check(_native.load().neo_hip_upols_set_filter(self._h, ctypes.c_void_p(partitions.data_ptr()), 1))
            return
        H = np.ascontiguousarray(partitions, dtype=np.complex64)
        if H.ndim == 2:
            H = H[None]
        if H.shape != (self.channels, self.partitions, self.block_size + 1):
            raise ValueError(f"filter shape {H.shape} != {(self.channels, self.partitions, self.block_size + 1)}")
        _native.check(_native.load().neo_hip_upols_set_filter(self._h, _ptr(H), 0))

    def set_impulse(self, impulse_response, normalize: bool = True) -> None:
        """normalize_impulse (optional) + uniform_partition straight into the device filter."""
        if _is_torch(impulse_response):
            t = impulse_response
            _producer_join(t)
            _native.check(_native.load().neo_hip_upols_set_impulse(self._h, ctypes.c_void_p(t.data_ptr()),
                                                                   t.shape[-1], int(normalize), 1))
            return
        ir = np.ascontiguousarray(np.atleast_2d(np.asarray(impulse_response, dtype=np.float32)))
        if ir.shape[0] != self.channels:
            raise ValueError("impulse channel count mismatch")
        _native.check(_native.load().neo_hip_upols_set_impulse(self._h, _ptr(ir), ir.shape[1], int(normalize), 0))

    def reset(self) -> None:
        _native.check(_native.load().neo_hip_upols_reset(self._h))

    # -- processing ---------------------------------------------------------
    def __call__(self, block, stream: int = 0):
        """Process one block [C][B] in place (float32 ndarray or CUDA tensor)."""
        if _is_torch(block):
            import torch

            assert block.dtype == torch.float32 and block.is_contiguous()
            if block.numel() != self.channels * self.block_size:
                raise ValueError("block must hold channels * block_size samples")
            if not block.is_cuda:  # host tensor (pinned ones are read and written in place)
                _native.check(_native.load().neo_hip_upols_process(self._h, ctypes.c_void_p(block.data_ptr()), 0,
                                                                   None))
                return block
            s = stream or torch.cuda.current_stream(block.device).cuda_stream
            _native.check(_native.load().neo_hip_upols_process(self._h, ctypes.c_void_p(block.data_ptr()), 1,
                                                               ctypes.c_void_p(s)))
            return block
        if not (isinstance(block, np.ndarray) and block.dtype == np.float32 and block.flags.c_contiguous):
            raise TypeError("block must be a C-contiguous float32 array")
        if block.size != self.channels * self.block_size:
            raise ValueError("block must hold channels * block_size samples")
        _native.check(_native.load().neo_hip_upols_process(self._h, _ptr(block), 0, None))
        return block

    def process(self, samples, stream: int = 0):
        """Any number of samples per channel, in place: [C][n] float32 ndarray or CUDA
        tensor. upola_v2 splits at block boundaries like overlap_add_convolver::operator()
        (overlap_add_convolver.hpp:80-134); upols/upola need n % block_size == 0."""
        lib = _native.load()
        if _is_torch(samples):
            import torch

            assert samples.dtype == torch.float32 and samples.is_contiguous()
            n = samples.shape[-1]
            s = stream or torch.cuda.current_stream(samples.device).cuda_stream
            p = ctypes.c_void_p(samples.data_ptr())
            _native.check(lib.neo_hip_upols_process_samples(self._h, p, n, p, n, n, 1, ctypes.c_void_p(s)))
            return samples
        if not (isinstance(samples, np.ndarray) and samples.dtype == np.float32 and samples.flags.c_contiguous):
            raise TypeError("samples must be a C-contiguous float32 array")
        n = samples.shape[-1] if samples.ndim else 0
        if samples.size != self.channels * n:
            raise ValueError("samples must be [channels][n]")
        _native.check(lib.neo_hip_upols_process_samples(self._h, _ptr(samples), n, _ptr(samples), n, n, 0, None))
        return samples

    def process_device(self, in_ptr: int, ld_in: int, out_ptr: int, ld_out: int, stream: int = 0) -> None:
        _native.check(_native.load().neo_hip_upols_process_device(self._h, ctypes.c_void_p(in_ptr), int(ld_in),
                                                                  ctypes.c_void_p(out_ptr), int(ld_out),
                                                                  ctypes.c_void_p(stream)))

    def process_blocks(self, signal, out=None, stream: int = 0):
        """Run consecutive blocks of a CUDA tensor [C][nblocks*B] (out may alias signal)."""
        import torch

        out = signal if out is None else out
        nb = signal.shape[-1] // self.block_size
        s = stream or torch.cuda.current_stream(signal.device).cuda_stream
        _native.check(_native.load().neo_hip_upols_process_blocks(self._h, ctypes.c_void_p(signal.data_ptr()),
                                                                  ctypes.c_void_p(out.data_ptr()), signal.shape[-1],
                                                                  nb, ctypes.c_void_p(s)))
        return out

    def process_blocks_ptr(self, in_ptr: int, out_ptr: int, ld: int, nblocks: int, stream: int = 0) -> None:
        """nblocks consecutive blocks through the C-ABI loop: channel c of block t at
        in_ptr + 4*(c*ld + t*B) (device pointers)."""
        _native.check(_native.load().neo_hip_upols_process_blocks(self._h, ctypes.c_void_p(in_ptr),
                                                                  ctypes.c_void_p(out_ptr), int(ld), int(nblocks),
                                                                  ctypes.c_void_p(stream)))

    def set_batch(self, enable: bool) -> None:
        """process_blocks: T blocks per MAC pass (default) or one block per pass."""
        _native.check(_native.load().neo_hip_upols_set_batch(self._h, int(enable)))

    def batch_info(self):
        """(blocks per process_blocks pass, splits per channel of that pass)."""
        t, s = ctypes.c_int(), ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_batch_info(self._h, ctypes.byref(t), ctypes.byref(s)))
        return t.value, s.value

    def set_offline(self, enable: bool) -> None:
        """Offline windows for batched calls of >= 128 blocks (neo_hip_upols_set_offline; on by
        default from 128 partitions): 128-block windows through partition-axis transforms."""
        _native.check(_native.load().neo_hip_upols_set_offline(self._h, int(bool(enable))))

    def offline_info(self):
        """(offline windows on, 128-partition segments they transform)"""
        e, n = ctypes.c_int(), ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_get_offline(self._h, ctypes.byref(e), ctypes.byref(n)))
        return bool(e.value), n.value

    def set_ahead(self, enable: bool) -> None:
        """Streaming levels for single-block steps (neo_hip_upols_set_ahead)."""
        _native.check(_native.load().neo_hip_upols_set_ahead(self._h, int(bool(enable))))

    def ahead_info(self):
        """(streaming levels enabled, block position in the current far window, longest
        window, number of levels)."""
        v = [ctypes.c_int() for _ in range(4)]
        _native.check(_native.load().neo_hip_upols_get_ahead(self._h, *[ctypes.byref(x) for x in v]))
        return bool(v[0].value), v[1].value, v[2].value, v[3].value

    def far_group(self) -> int:
        """Windows per far phase-1 pass this handle runs (0: no far transform level)."""
        k = ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_get_far_group(self._h, ctypes.byref(k)))
        return k.value

    def step_group(self) -> int:
        """Steps per background launch of the streaming levels' slices (1: one launch per step)."""
        k = ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_get_step_group(self._h, ctypes.byref(k)))
        return k.value

    def far_form(self) -> int:
        """The p >= 256 band's form: 0 none, 1 transform with stored spectra, 2 transform recomputed
        every window, 3 the 128-block Toeplitz level (neo_hip_upols_get_far_form)."""
        k = ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_get_far_form(self._h, ctypes.byref(k)))
        return k.value

    def join_background(self, stream=None) -> None:
        """Make `stream` (a raw hipStream_t, None = the null stream) wait for the background
        slice launches of the step groups issued so far (device-side; no host wait)."""
        _native.check(_native.load().neo_hip_upols_join_background(self._h, ctypes.c_void_p(stream)))

    def set_paced(self, enable) -> None:
        """Step groups: issue the group's background launch in pieces, each block after the
        piece before it (neo_hip_upols_set_paced): an even host round trip per block. True / 1:
        a piece per call; 2: two pieces per group; False / 0: off."""
        _native.check(_native.load().neo_hip_upols_set_paced(self._h, int(enable)))

    def set_persistent(self, enable: bool, idle_ms: float = 50.0) -> None:
        """Latency mode (neo_hip_upols_set_persistent): one persistent kernel steps every block;
        every process call is then synchronous (complete on return, the stream is not used).
        With the streaming levels it runs their block and slice roles (blocks up to 512); without
        them (fewer than 64 partitions) the plain fused step, blocks up to 4096. Raises for shapes
        it does not take (more than 16 channels, sub-block v2, B > 512 with the levels)."""
        _native.check(_native.load().neo_hip_upols_set_persistent(self._h, int(bool(enable)), float(idle_ms)))

    def persistent_info(self) -> dict:
        e, r, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        _native.check(_native.load().neo_hip_upols_get_persistent(self._h, ctypes.byref(e), ctypes.byref(r),
                                                                   ctypes.byref(n)))
        return {"enabled": bool(e.value), "running": bool(r.value), "launches": n.value}

    def persist_step_times(self, cap: int = 63):
        """GPU time (us) of the last latency-mode steps, oldest first: record read -> done signal."""
        buf, n = (ctypes.c_double * cap)(), ctypes.c_int64()
        _native.check(_native.load().neo_hip_upols_persist_step_times(self._h, buf, cap, ctypes.byref(n)))
        return list(buf[: n.value])

    # -- instrumentation ------------------------------------------------------
    def set_timing(self, enable, every: int = 1) -> None:
        """HIP events around every `every`-th MAC launch while enabled (bench instrumentation)."""
        if every < 1:
            raise ValueError("every must be >= 1")
        _native.check(_native.load().neo_hip_upols_set_timing(self._h, int(every) if enable else 0))

    def timing(self):
        """(accumulated ms, timed launch groups) since the last call: the MAC kernel of
        plain / batched steps, the whole step of streaming-level steps."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _native.check(_native.load().neo_hip_upols_timing(self._h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def timing_detail(self):
        """Per part [(ms, count)] * 4 since the last call (neo_hip_upols_timing_detail):
        streaming-level steps 0 = the step kernel (k_lvl_step: block and level slices);
        plain / batched steps 0 = MAC kernel."""
        ms, n = (ctypes.c_double * 4)(), (ctypes.c_int64 * 4)()
        _native.check(_native.load().neo_hip_upols_timing_detail(self._h, ms, n))
        return [(ms[k], n[k]) for k in range(4)]

    def step_times(self, cap: int = 1 << 16):
        """Duration (ms) of every timed launch group since the last drain, in order (a
        streaming step: first to last event of the step)."""
        buf, n = (ctypes.c_double * cap)(), ctypes.c_int64()
        _native.check(_native.load().neo_hip_upols_step_times(self._h, buf, cap, ctypes.byref(n)))
        return list(buf[: min(n.value, cap)])

    @property
    def splits(self) -> int:
        s = ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_info(self._h, None, None, None, ctypes.byref(s)))
        return s.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().neo_hip_upols_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class UpolsMultiConvolver:
    """C channels sharded over several devices of one node (neo_hip_upols_multi_*): shard i
    = channels [C i / n, C (i + 1) / n) on devices[i] (a device may repeat), one handle and
    stream each, no collective (the reference steps all channels in one loop,
    DenseConvolution.hpp:35,50-67). Host I/O; every call runs the shards concurrently and
    returns when all are done. Results equal one UpolsConvolver over all channels bit for
    bit."""

    def __init__(self, channels: int, block_size: int, partitions: int, devices, method: str = "upols",
                 options: dict | None = None):
        lib = _native.load()
        methods = {"upols": 0, "upola": 1, "upola_v2": 2}
        if method not in methods:
            raise ValueError(f"method must be 'upols', 'upola' or 'upola_v2', got {method!r}")
        opts = dict(UpolsConvolver.OPTION_DEFAULTS)
        for k, v in (options or {}).items():
            if k not in opts:
                raise ValueError(f"unknown convolver option {k!r}")
            opts[k] = int(v)
        o = _native.UpolsOpts(**opts)
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        h = ctypes.c_void_p()
        _native.check(lib.neo_hip_upols_multi_create(int(channels), int(block_size), int(partitions), devs,
                                                     len(devices), methods[method], ctypes.byref(o), ctypes.byref(h)))
        self._h = h
        self.channels, self.block_size, self.partitions = channels, block_size, partitions
        self.devices = list(devices)

    def shards(self):
        """[(device, first_channel, channels)] per shard"""
        lib = _native.load()
        n = ctypes.c_int()
        _native.check(lib.neo_hip_upols_multi_shards(self._h, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            d, c0, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            _native.check(lib.neo_hip_upols_multi_shard(self._h, i, None, ctypes.byref(d), ctypes.byref(c0),
                                                        ctypes.byref(nc)))
            out.append((d.value, c0.value, nc.value))
        return out

    def filter(self, partitions) -> None:
        H = np.ascontiguousarray(partitions, dtype=np.complex64)
        if H.shape != (self.channels, self.partitions, self.block_size + 1):
            raise ValueError(f"filter shape {H.shape} != {(self.channels, self.partitions, self.block_size + 1)}")
        _native.check(_native.load().neo_hip_upols_multi_set_filter(self._h, _ptr(H)))

    def set_impulse(self, impulse_response, normalize: bool = True) -> None:
        ir = np.ascontiguousarray(np.atleast_2d(np.asarray(impulse_response, dtype=np.float32)))
        if ir.shape[0] != self.channels:
            raise ValueError("impulse channel count mismatch")
        _native.check(_native.load().neo_hip_upols_multi_set_impulse(self._h, _ptr(ir), ir.shape[1], int(normalize)))

    def process(self, samples) -> np.ndarray:
        """[C][n] float32 host samples (n a multiple of the block except for upola_v2) ->
        [C][n] output; the shards run concurrently."""
        x = np.ascontiguousarray(samples, dtype=np.float32)
        if x.ndim != 2 or x.shape[0] != self.channels:
            raise ValueError(f"samples must be [{self.channels}][n]")
        y = np.empty_like(x)
        n = x.shape[1]
        _native.check(_native.load().neo_hip_upols_multi_process_samples(self._h, _ptr(x), n, _ptr(y), n, n))
        return y

    def reset(self) -> None:
        _native.check(_native.load().neo_hip_upols_multi_reset(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().neo_hip_upols_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OverlapStage:
    """C independent overlap stages on the GPU (neo_hip_overlap_*): overlap_save
    (overlap_save.hpp:19-112) or overlap_add (overlap_add.hpp:23-107) of block B for F-tap
    filters, transform size 2^next_order(B + F - 1). forward(block) updates the window and
    returns the n/2 + 1 bins the reference's callback sees; inverse(spectrum, out) runs the
    irfft, 1/n and writes the output block. Host arrays (synchronous) or CUDA tensors."""

    KINDS = {"save": 0, "add": 1}

    def __init__(self, kind: str, channels: int, block_size: int, filter_size: int, device: int = 0):
        if kind not in self.KINDS:
            raise ValueError(f"kind must be 'save' or 'add', got {kind!r}")
        h = ctypes.c_void_p()
        _native.check(_native.load().neo_hip_overlap_create(self.KINDS[kind], int(channels), int(block_size),
                                                            int(filter_size), int(device), ctypes.byref(h)))
        self._h = h
        self.kind, self.channels, self.device = kind, channels, device
        b, f, n = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _native.check(_native.load().neo_hip_overlap_info(h, ctypes.byref(b), ctypes.byref(f), ctypes.byref(n)))
        self._block, self._filter, self._n = b.value, f.value, n.value

    def block_size(self) -> int:
        return self._block

    def filter_size(self) -> int:
        return self._filter

    def transform_size(self) -> int:
        return self._n

    def forward(self, block, spectrum=None, stream: int = 0):
        """block [C][B] float32 -> spectrum [C][n/2 + 1] complex64 (new array / tensor if None)."""
        lib = _native.load()
        bins = self._n // 2 + 1
        if _is_torch(block) and block.is_cuda:
            import torch

            spec = spectrum if spectrum is not None else torch.empty((self.channels, bins), dtype=torch.complex64,
                                                                     device=block.device)
            s = stream or torch.cuda.current_stream(block.device).cuda_stream
            ld = block.stride(0) if block.dim() == 2 else block.shape[-1]  # channel c at c * ld
            _native.check(lib.neo_hip_overlap_forward(self._h, ctypes.c_void_p(block.data_ptr()), ld,
                                                      ctypes.c_void_p(spec.data_ptr()), 1, ctypes.c_void_p(s)))
            return spec
        x = np.ascontiguousarray(np.asarray(block, dtype=np.float32).reshape(self.channels, -1))
        if x.shape[1] != self._block:
            raise ValueError(f"block must be [{self.channels}][{self._block}]")
        spec = np.empty((self.channels, bins), np.complex64) if spectrum is None else spectrum
        _native.check(lib.neo_hip_overlap_forward(self._h, _ptr(x), x.shape[1], _ptr(spec), 0, None))
        return spec

    def inverse(self, spectrum, out, stream: int = 0):
        """spectrum [C][n/2 + 1] complex64 -> out [C][B] float32 (in place)."""
        lib = _native.load()
        if _is_torch(out) and out.is_cuda:
            import torch

            s = stream or torch.cuda.current_stream(out.device).cuda_stream
            ld = out.stride(0) if out.dim() == 2 else out.shape[-1]
            _native.check(lib.neo_hip_overlap_inverse(self._h, ctypes.c_void_p(spectrum.data_ptr()),
                                                      ctypes.c_void_p(out.data_ptr()), ld, 1, ctypes.c_void_p(s)))
            return out
        spec = np.ascontiguousarray(spectrum, dtype=np.complex64)
        if not (isinstance(out, np.ndarray) and out.dtype == np.float32 and out.flags.c_contiguous):
            raise TypeError("out must be a C-contiguous float32 array")
        _native.check(lib.neo_hip_overlap_inverse(self._h, _ptr(spec), _ptr(out), out.shape[-1], 0, None))
        return out

    def reset(self) -> None:
        _native.check(_native.load().neo_hip_overlap_reset(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().neo_hip_overlap_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class overlap_save:
    """Drop-in for neo::convolution::overlap_save<complex<float>> (overlap_save.hpp:19-112):
    overlap_save(block_size, filter_size); __call__(block, callback) processes one block of a
    1-D float32 array in place, callback(bins) sees (and may modify in place) the
    transform_size() / 2 + 1 bins."""

    _kind = "save"

    def __init__(self, block_size: int, filter_size: int, device: int = 0):
        self._stage = OverlapStage(self._kind, 1, block_size, filter_size, device)

    def block_size(self) -> int:
        return self._stage.block_size()

    def filter_size(self) -> int:
        return self._stage.filter_size()

    def transform_size(self) -> int:
        return self._stage.transform_size()

    def __call__(self, block, callback):
        if not (isinstance(block, np.ndarray) and block.dtype == np.float32 and block.flags.c_contiguous):
            raise TypeError("block must be a C-contiguous float32 array")
        if block.size != self.block_size():
            raise ValueError(f"block must hold {self.block_size()} samples")
        spec = self._stage.forward(block.reshape(1, -1))
        callback(spec[0])
        self._stage.inverse(spec, block.reshape(1, -1))
        return block


class overlap_add(overlap_save):
    """Drop-in for neo::convolution::overlap_add<complex<float>> (overlap_add.hpp:23-107)."""

    _kind = "add"


class UpolsGroup:
    """Single-channel convolvers of one shape stepped together (neo_hip_upols_group_*): members
    join(), take a filter [P][B+1] each and process one host block [B] per call, in place; while
    the calls follow the plugin's frame pattern (DenseConvolution.cpp:62-74: every member once
    per frame, each on a buffer of its own) and every member's buffer is registered with the
    group (register(): the owner keeps it allocated until unregister()), a frame is ONE launch,
    else each member runs on a handle of its own; outputs are each member's own sequential
    convolver's either way (up to float summation order after a mode switch)."""

    def __init__(self, block_size: int, partitions: int, method: str = "upols", device: int = 0):
        methods = {"upols": 0, "upola": 1}
        if method not in methods:
            raise ValueError("groups take method 'upols' or 'upola'")
        h = ctypes.c_void_p()
        _native.check(_native.load().neo_hip_upols_group_create(int(block_size), int(partitions), methods[method],
                                                                int(device), ctypes.byref(h)))
        self._h = h
        self.block_size, self.partitions = block_size, partitions

    def join(self) -> int:
        i = ctypes.c_int()
        _native.check(_native.load().neo_hip_upols_group_join(self._h, ctypes.byref(i)))
        return i.value

    def leave(self, member: int) -> None:
        _native.check(_native.load().neo_hip_upols_group_leave(self._h, int(member)))

    def filter(self, member: int, partitions) -> None:
        H = np.ascontiguousarray(partitions, dtype=np.complex64)
        if H.shape != (self.partitions, self.block_size + 1):
            raise ValueError(f"filter shape {H.shape} != {(self.partitions, self.block_size + 1)}")
        _native.check(_native.load().neo_hip_upols_group_set_filter(self._h, int(member), _ptr(H), 0))

    def __call__(self, member: int, block: np.ndarray) -> np.ndarray:
        if not (isinstance(block, np.ndarray) and block.dtype == np.float32 and block.flags.c_contiguous
                and block.size == self.block_size):
            raise TypeError("block must be a C-contiguous float32 array of block_size samples")
        _native.check(_native.load().neo_hip_upols_group_process(self._h, int(member), _ptr(block)))
        return block

    def reset(self, member: int) -> None:
        _native.check(_native.load().neo_hip_upols_group_reset(self._h, int(member)))

    def register(self, buffer: np.ndarray, frame_stable: bool = False, in_place: bool = False) -> None:
        """the group may read `buffer` (host memory the caller keeps alive until unregister).
        frame_stable: the caller also promises that during a frame nothing but the members' own
        calls writes it (neo_hip_upols_group_register_ex, NEO_HIP_GROUP_FRAME_STABLE): members then
        commit without comparing their blocks with a snapshot. in_place (NEO_HIP_GROUP_FRAME_INPLACE,
        implies frame_stable): it also reads each member's block only through that member's call,
        each member on the same block every frame: the frame's first call writes every output in place."""
        if not isinstance(buffer, np.ndarray) or not buffer.flags.c_contiguous:
            raise TypeError("register takes a C-contiguous numpy array")
        self._keep = getattr(self, "_keep", {})
        self._keep[buffer.ctypes.data] = buffer  # keeps the registered array alive on the Python side too
        _native.check(_native.load().neo_hip_upols_group_register_ex(self._h, ctypes.c_void_p(buffer.ctypes.data),
                                                                     int(buffer.nbytes),
                                                                     3 if in_place else (1 if frame_stable else 0)))

    def unregister(self, buffer=None) -> None:
        """stop reading `buffer` (None: every registered range)"""
        ptr = None if buffer is None else buffer.ctypes.data
        _native.check(_native.load().neo_hip_upols_group_unregister(self._h, ctypes.c_void_p(ptr)))
        keep = getattr(self, "_keep", {})
        if ptr is None:
            keep.clear()
        else:
            keep.pop(ptr, None)

    def stats(self) -> dict:
        c = ctypes.c_int()
        v = [ctypes.c_int64() for _ in range(4)]
        _native.check(_native.load().neo_hip_upols_group_stats(self._h, ctypes.byref(c), *[ctypes.byref(x) for x in v]))
        return {"coalesced": bool(c.value), "frame_steps": v[0].value, "calls": v[1].value, "redos": v[2].value,
                "switches": v[3].value}

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _native.load().neo_hip_upols_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class upols_convolver:
    """Single-channel drop-in for upols_convolver<complex<float>>: default-constructible,
    filter([P][B+1]) then __call__(block[B]) in place."""

    _method = "upols"

    def __init__(self, device: int = 0):
        self._impl = None
        self._device = device

    def filter(self, filt) -> None:
        H = np.ascontiguousarray(filt, dtype=np.complex64)
        if H.ndim != 2:
            raise ValueError("filter must be [P][B+1]")
        P, bins = H.shape
        impl = self._impl
        if impl is None or (impl.partitions, impl.block_size) != (P, bins - 1):
            impl = UpolsConvolver(1, bins - 1, P, self._device, method=self._method)
        impl.filter(H[None])
        self._impl = impl

    def __call__(self, block):
        if self._impl is None:
            raise RuntimeError("filter() must be called first")
        return self._impl(block)


split_upols_convolver = upols_convolver


class upola_convolver(upols_convolver):
    """Single-channel drop-in for upola_convolver<complex<float>> (overlap-add stage)."""

    _method = "upola"


split_upola_convolver = upola_convolver


class upola_convolver_v2(upols_convolver):
    """Single-channel drop-in for upola_convolver_v2<complex<float>> (overlap_add_convolver.hpp:
    20-136): __call__ takes any number of samples, in place."""

    _method = "upola_v2"

    def __call__(self, samples):
        if self._impl is None:
            raise RuntimeError("filter() must be called first")
        if _is_torch(samples):
            return self._impl.process(samples.view(1, -1))
        if not (isinstance(samples, np.ndarray) and samples.dtype == np.float32 and samples.flags.c_contiguous):
            raise TypeError("samples must be a C-contiguous float32 array")
        self._impl.process(samples.reshape(1, -1))  # a view: processed in place
        return samples


def dense_convolve(signal, impulse_response, block_size: int, device: int = 0, method: str = "upols",
                   options: dict | None = None) -> np.ndarray:
    """dense_convolve<upols_convolver | upola_convolver> (DenseConvolution.hpp:39-70): normalize
    the IR matrix, partition it, run every block (tail zero-padded), output truncated to N.
    `options`: UpolsConvolver code-path choices (same results)."""
    sig = np.ascontiguousarray(np.atleast_2d(np.asarray(signal, dtype=np.float32)))
    ir = np.ascontiguousarray(np.atleast_2d(np.asarray(impulse_response, dtype=np.float32)))
    C, N = sig.shape
    if ir.shape[0] != C:
        raise ValueError("signal and impulse response channel counts differ")
    P = num_partitions(ir.shape[1], block_size)
    conv = UpolsConvolver(C, block_size, P, device, method=method, options=options)
    conv.set_impulse(ir, normalize=True)
    nb = -(-N // block_size)
    # whole signal in chunks of <= 2^26 samples: one upload, batched passes (T blocks per
    # pass over filter + FDL), one download per chunk; the tail block is zero-padded
    chunk = max(1, (1 << 26) // (C * block_size))
    chunk = max(256, chunk // 256 * 256)  # whole offline passes (256 blocks: two windows of 128)
    out = np.empty_like(sig)
    for t0 in range(0, nb, chunk):
        t1 = min(nb, t0 + chunk)
        lo, hi = t0 * block_size, min(N, t1 * block_size)
        buf = np.zeros((C, (t1 - t0) * block_size), dtype=np.float32)
        buf[:, : hi - lo] = sig[:, lo:hi]
        conv.process(buf)
        out[:, lo:hi] = buf[:, : hi - lo]
    conv.close()
    return out


def _one_shot(name, signal, patch, device):
    """The reference binds float then double (main.cpp:255-258): a float64 pair picks the
    double overload, anything else converts to float32 (pybind11's converting pass)."""
    a = np.asarray(signal)
    b = np.asarray(patch)
    if a.ndim != 1 or b.ndim != 1:
        raise RuntimeError("unsupported dimension: in1 and in2 must be 1-D")  # main.cpp:173-175
    f64 = a.dtype == np.float64 and b.dtype == np.float64
    dt = np.float64 if f64 else np.float32
    a = np.ascontiguousarray(a, dtype=dt)
    b = np.ascontiguousarray(b, dtype=dt)
    if a.size == 0 or b.size == 0:
        return np.zeros(0, dt)
    out = np.empty(a.size + b.size - 1, dt)
    fn = getattr(_native.load(), name + ("_f64" if f64 else ""))
    _native.check(fn(_ptr(a), a.size, _ptr(b), b.size, _ptr(out), 0, int(device)))
    return out


def fft_convolve(signal, patch, device: int = 0) -> np.ndarray:
    """Full linear convolution through one r2c/c2r pair (fft_convolver.hpp:19-93)."""
    return _one_shot("neo_hip_fft_convolve", signal, patch, device)


def direct_convolve(signal, patch, device: int = 0) -> np.ndarray:
    """Full linear convolution, direct sum (direct_convolve.hpp:14-56), bit-identical loop order."""
    return _one_shot("neo_hip_direct_convolve", signal, patch, device)


def convolve(in1, in2, mode: str = "full", method: str = "auto", device: int = 0) -> np.ndarray:
    """neo.convolve (extra/python/src/neo/__init__.py:43-48): method "fft" -> fft_convolve,
    anything else -> direct_convolve; only mode "full" (others raise RuntimeError, main.cpp:197)."""
    if mode not in ("full", "valid", "same"):
        raise KeyError(mode)
    if mode != "full":
        raise RuntimeError("unsupported convolution mode")
    if method == "fft":
        return fft_convolve(in1, in2, device)
    return direct_convolve(in1, in2, device)
