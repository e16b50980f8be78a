"""Setup calls beside real-time work.

1. The first call after filter() is an ordinary block step. The reference's filter() rebuilds the
   convolver's state (uniform_partitioned_convolver.hpp:37-45) and its next call is the plain
   per-block step (:47-65); the plugin changes the IR beside its audio thread
   (extra/plugin/src/dsp/DenseConvolution.cpp:78-108). Here set_filter / set_impulse / reset
   prepare the streaming levels themselves (buffers, far segment spectra, window 0 of every
   level, which after a reset is all zero), so the blocks after them are checked against the
   oracle at far-level shapes, in one-launch and step-group form, OLS and OLA, and after a
   batched pass (a non-zero delay line: the full prime runs at the next streaming step).
2. Setup calls never wait for the whole device: with another handle's latency-mode kernel
   resident, normalize_impulse / uniform_partition on device tensors and a filter change on a
   handle that stepped on many streams each return in milliseconds.
3. A device impulse written on a torch side stream right before set_impulse is complete when the
   filter is built (the Python layer joins torch's current stream)."""
import time

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _parts(oracle, C, B, P, seed):
    L = B * (P - 1) + B // 2 + 1
    ir = np.stack([oracle.noise(seed + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    assert parts.shape[1] == P
    return ir, parts


def _blocks(conv, sig, B, torch, per_call=1):
    t = torch.from_numpy(np.ascontiguousarray(sig)).cuda()
    cur = torch.cuda.current_stream()
    nb = sig.shape[1] // B
    for i in range(0, nb, per_call):
        k = min(per_call, nb - i)
        conv.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, sig.shape[1], k, cur.cuda_stream)
    cur.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("method", ["upols", "upola"])
@pytest.mark.parametrize("C,B,P,opts", [
    (2, 64, 300, {}),                      # G = 1: one launch per step, far level
    (128, 256, 300, {}),                   # 2048 units: step groups of 4, far level
    (1, 32, 700, {"far_group": 3}),        # several far segments, window group 3
    (2, 128, 600, {"far_level": 0}),       # the 128-block Toeplitz level
    (2, 64, 420, {"far_level": 2, "step_group": 4}),  # the recomputed far level
])
def test_blocks_after_filter_change_and_reset(neo_gpu, oracle, method, C, B, P, opts):
    """A handle streams 40 blocks with one filter, then set_filter(another) and 8 + 140 blocks
    (the first eight one call each, as the plugin's audio thread), then reset and 8 more: every
    output against the oracle's fresh convolver over the same blocks."""
    torch = pytest.importorskip("torch")
    _, p0 = _parts(oracle, C, B, P, 3100 + P)
    _, p1 = _parts(oracle, C, B, P, 3200 + P)
    conv = neo_gpu.UpolsConvolver(C, B, P, method=method, options=opts)
    conv.filter(p0)
    conv.set_batch(False)
    assert conv.ahead_info()[0]
    s0 = np.stack([oracle.noise(3300 + c, B * 40) for c in range(C)])
    assert peak_err(_blocks(conv, s0, B, torch), oracle.dense_convolve(s0, p0, method=method)) <= TOL
    conv.filter(p1)
    s1 = np.stack([oracle.noise(3400 + c, B * 148) for c in range(C)])
    got = np.concatenate([_blocks(conv, s1[:, : 8 * B], B, torch), _blocks(conv, s1[:, 8 * B:], B, torch, 16)], axis=1)
    ref = oracle.dense_convolve(s1, p1, method=method)
    assert peak_err(got[:, : 8 * B], ref[:, : 8 * B]) <= TOL
    assert peak_err(got, ref) <= TOL
    conv.reset()
    s2 = np.stack([oracle.noise(3500 + c, B * 8) for c in range(C)])
    assert peak_err(_blocks(conv, s2, B, torch), oracle.dense_convolve(s2, p1, method=method)) <= TOL
    conv.close()


def test_reset_after_batched_pass_and_impulse_change(neo_gpu, oracle):
    """Batched passes leave a non-zero delay line (full prime at the next streaming step); a
    reset zeroes it (zero prime at the reset); set_impulse on a device IR does the same after
    normalizing and partitioning: blocks after each against the oracle."""
    torch = pytest.importorskip("torch")
    C, B, P = 2, 64, 300
    ir, parts = _parts(oracle, C, B, P, 3600)
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.filter(parts)
    sig = np.stack([oracle.noise(3610 + c, B * 96) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts)
    t = torch.from_numpy(sig[:, : 64 * B].copy()).cuda()
    conv.process_blocks(t)  # two batched passes of 32
    got = [t.cpu().numpy(), _blocks(conv, sig[:, 64 * B:], B, torch)]  # streaming: full prime
    assert peak_err(np.concatenate(got, axis=1), ref) <= TOL
    conv.reset()
    s2 = np.stack([oracle.noise(3620 + c, B * 8) for c in range(C)])
    assert peak_err(_blocks(conv, s2, B, torch), oracle.dense_convolve(s2, parts)) <= TOL
    ir2 = np.stack([oracle.noise(3630 + c, ir.shape[1]) for c in range(C)])
    conv.set_impulse(torch.from_numpy(ir2).cuda())
    p2 = oracle.uniform_partition(oracle.normalize_impulse(ir2), B)
    s3 = np.stack([oracle.noise(3640 + c, B * 300) for c in range(C)])
    assert peak_err(_blocks(conv, s3, B, torch), oracle.dense_convolve(s3, p2)) <= TOL
    conv.close()


def test_latency_mode_after_filter_change(neo_gpu, oracle):
    """The latency mode continues from the levels a filter change prepared (no prime in the
    persistent kernel's launch): one channel with a far level, filter change, reset, against
    the oracle."""
    torch = pytest.importorskip("torch")
    C, B, P = 1, 64, 300
    _, p0 = _parts(oracle, C, B, P, 3700)
    _, p1 = _parts(oracle, C, B, P, 3710)
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.filter(p0)
    conv.set_batch(False)
    conv.set_persistent(True, idle_ms=200.0)
    s0 = np.stack([oracle.noise(3720, B * 100)])
    assert peak_err(_blocks(conv, s0, B, torch), oracle.dense_convolve(s0, p0)) <= TOL
    conv.filter(p1)
    s1 = np.stack([oracle.noise(3730, B * 300)])
    assert peak_err(_blocks(conv, s1, B, torch), oracle.dense_convolve(s1, p1)) <= TOL
    conv.reset()
    s2 = np.stack([oracle.noise(3740, B * 20)])
    assert peak_err(_blocks(conv, s2, B, torch), oracle.dense_convolve(s2, p1)) <= TOL
    conv.set_persistent(False)
    conv.close()


def test_setup_calls_do_not_wait_for_the_device(neo_gpu, oracle):
    """Handle A's latency-mode kernel stays resident (idle limit 3 s) between its calls. Meanwhile
    normalize_impulse and uniform_partition on device tensors, and set_impulse (device IR) on a
    handle B that stepped on six streams (more than it remembers individually would once have
    made it wait for the device), each return within 5 ms, with correct results; A steps on."""
    torch = pytest.importorskip("torch")
    B, P = 256, 100
    _, pa_parts = _parts(oracle, 1, B, P, 3800)
    a = neo_gpu.UpolsConvolver(1, B, P)
    a.filter(pa_parts)
    a.set_batch(False)
    a.set_persistent(True, idle_ms=3000.0)
    xa = np.stack([oracle.noise(3810, B * 8)])
    first = _blocks(a, xa[:, : 4 * B], B, torch)
    assert a.persistent_info()["running"]

    Cb, Pb = 2, 40
    ir, _ = _parts(oracle, Cb, 128, Pb, 3820)
    b = neo_gpu.UpolsConvolver(Cb, 128, Pb)
    b.set_batch(False)
    streams = [torch.cuda.Stream() for _ in range(6)]
    xb = torch.zeros((Cb, 128), device="cuda")
    torch.cuda.current_stream().synchronize()
    for s in streams:
        b.process_blocks_ptr(xb.data_ptr(), xb.data_ptr(), 128, 1, s.cuda_stream)
    for s in streams:
        s.synchronize()
    dev_ir = torch.from_numpy(ir).cuda()
    torch.cuda.current_stream().synchronize()
    times = {}
    for rep in range(2):  # the first round allocates pooled memory; the second is timed
        t = dev_ir.clone()
        torch.cuda.current_stream().synchronize()
        t0 = time.perf_counter()
        neo_gpu.normalize_impulse(t)
        t1 = time.perf_counter()
        parts = neo_gpu.uniform_partition(t, 128)
        t2 = time.perf_counter()
        for s in streams:
            b.process_blocks_ptr(xb.data_ptr(), xb.data_ptr(), 128, 1, s.cuda_stream)
            s.synchronize()
        t3 = time.perf_counter()
        b.set_impulse(dev_ir)
        t4 = time.perf_counter()
        times = {"normalize": t1 - t0, "partition": t2 - t1, "set_impulse": t4 - t3}
    assert a.persistent_info()["running"], "the latency-mode kernel left: the timing proves nothing"
    assert all(v < 5e-3 for v in times.values()), times
    ref_parts = oracle.uniform_partition(oracle.normalize_impulse(ir.copy()), 128)
    assert peak_err(parts.cpu().numpy(), ref_parts) <= TOL
    second = _blocks(a, xa[:, 4 * B:], B, torch)
    assert peak_err(np.concatenate([first, second], axis=1), oracle.dense_convolve(xa, pa_parts)) <= TOL
    a.set_persistent(False)
    a.close()
    b.close()


def test_device_impulse_from_a_side_stream(neo_gpu, oracle):
    """An IR produced on a torch side stream (a long chain of kernels) right before set_impulse
    inside `with torch.cuda.stream(s)`: the filter is built from the finished IR."""
    torch = pytest.importorskip("torch")
    C, B, P = 2, 128, 60
    ir, _ = _parts(oracle, C, B, P, 3900)
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.set_batch(False)
    src = torch.from_numpy(ir).cuda()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        big = torch.rand((4096, 4096), device="cuda")
        for _ in range(20):  # keep the side stream busy
            big = big @ big
            big = big / big.abs().max()
        dev_ir = torch.zeros_like(src)
        dev_ir.add_(src)
        conv.set_impulse(dev_ir)
        normed = dev_ir.clone()
        neo_gpu.normalize_impulse(normed)
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir.copy()), B)
    sig = np.stack([oracle.noise(3910 + c, B * 40) for c in range(C)])
    assert peak_err(_blocks(conv, sig, B, torch), oracle.dense_convolve(sig, parts)) <= TOL
    s.synchronize()
    assert peak_err(normed.cpu().numpy(), oracle.normalize_impulse(ir.copy())) <= TOL
    conv.close()
