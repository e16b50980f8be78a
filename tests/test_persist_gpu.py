"""Latency mode (neo_hip_upols_set_persistent, upols_levels.hip k_lvl_persist; upols.hip
k_plain_persist for handles without streaming levels): one persistent kernel per handle steps
every block of a latency-bound shape (the reference's benchmark shape,
extra/benchmark/src/convolution.cpp:34-44: one channel, one call per block). Outputs must equal
the oracle's dense_convolve (uniform_partitioned_convolver.hpp:47-65) and the normal streaming
step's bit for bit: the same sums in the same order, and its block role, a separate code
instantiation (write-through output, system-scope input loads), rounds the same way because the
library is built with -ffp-contract=on (a*b+c fused per source expression, never across
statements after inlining; with the HIP default =fast the two differed by up to 2.4e-7 at C3,
tools/dbg_bitexact.py). The mode survives idle timeouts (relaunch) and hands back to the normal
schedule (re-prime) when switched off."""
import os
import time

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
TOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def same_sums(a, b):
    """the same sums in the same order: bit-equal"""
    return np.array_equal(a, b)


def _pair(neo_gpu, oracle, C, B, P, seed, method="upols"):
    ir = np.stack([oracle.noise(seed + c, B * P) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    convs = []
    for _ in range(2):
        c = neo_gpu.UpolsConvolver(C, B, P, method=method)
        c.filter(parts)
        c.set_batch(False)
        convs.append(c)
    return convs, parts


def _run(conv, x, B, torch, per_call=1):
    """x [C][N] through conv, per_call blocks per process call, device-resident, in place"""
    t = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    cur = torch.cuda.current_stream()
    cur.synchronize()  # not a device-wide sync: that would wait for a resident persistent kernel to leave
    nb = x.shape[1] // B
    for i in range(0, nb, per_call):
        k = min(per_call, nb - i)
        conv.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, x.shape[1], k, cur.cuda_stream)
    cur.synchronize()
    return t.cpu().numpy()


def test_c3_latency_mode_golden_and_oracle(neo_gpu, oracle):
    """configs[2] at its exact shape (B = 512, L = 96000, P = 188, 1 channel): the golden
    fixture's 200 blocks one call per block, then 640 blocks of fresh noise against the oracle
    and against the normal streaming step."""
    torch = pytest.importorskip("torch")
    g = np.load(os.path.join(GOLD, "upols_b512_l96000_seed7.npz"))
    B = 512
    P = neo_gpu.num_partitions(g["ir"].shape[-1], B)
    conv = neo_gpu.UpolsConvolver(1, B, P)
    conv.set_impulse(np.atleast_2d(g["ir"]), normalize=True)
    conv.set_batch(False)
    conv.set_persistent(True)
    assert conv.persistent_info()["enabled"]
    sig = np.atleast_2d(g["signal"]).astype(np.float32)
    nb = sig.shape[1] // B
    got = _run(conv, sig[:, : nb * B], B, torch)
    out = np.atleast_2d(g["out"])[:, : nb * B]
    assert peak_err(got, out) <= TOL
    assert np.abs(got - out).max() <= 1e-5
    info = conv.persistent_info()
    assert info["enabled"] and info["launches"] >= 1, info
    st = conv.persist_step_times()
    assert len(st) == 63 and all(0 < s < 1000 for s in st), st[:4]
    # fresh noise vs the oracle and vs the normal step
    conv.reset()
    conv.set_persistent(True)
    nb2 = 640
    x = np.stack([oracle.noise(4243, B * nb2)])
    irn = oracle.normalize_impulse(np.atleast_2d(g["ir"]).astype(np.float32))
    ref = oracle.dense_convolve(x, oracle.uniform_partition(irn, B))
    got = _run(conv, x, B, torch, per_call=4)
    assert peak_err(got, ref) <= TOL
    normal = neo_gpu.UpolsConvolver(1, B, P)
    normal.set_impulse(np.atleast_2d(g["ir"]), normalize=True)
    normal.set_batch(False)
    assert same_sums(got, _run(normal, x, B, torch))
    conv.close()
    normal.close()


@pytest.mark.parametrize("method,C,B,P", [("upols", 4, 256, 100), ("upola", 3, 128, 240), ("upols", 16, 64, 200)])
def test_latency_mode_channels_methods(neo_gpu, oracle, method, C, B, P):
    """several channels (one block workgroup each, the last to finish signals), OLA, small
    blocks: oracle (the OLS restatement for upols; for upola the same bit-equality with the
    normal step, which the streaming tests pin to the oracle) and the normal step (bit-equal)."""
    torch = pytest.importorskip("torch")
    (pc, nc), parts = _pair(neo_gpu, oracle, C, B, P, 5000 + C, method)
    pc.set_persistent(True)
    nb = 3 * P // 2 + 37
    x = np.stack([oracle.noise(5100 + c, B * nb) for c in range(C)])
    got = _run(pc, x, B, torch, per_call=3)
    assert same_sums(got, _run(nc, x, B, torch))
    if method == "upols":
        assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL


def test_latency_mode_idle_relaunch_and_handback(neo_gpu, oracle):
    """idle_ms = 5: the kernel leaves between bursts and the next call relaunches it (state
    kept); switched off mid-stream, the normal schedule re-primes and continues; both equal a
    handle that never left the normal step (bit for bit) and the oracle."""
    torch = pytest.importorskip("torch")
    C, B, P = 2, 256, 150
    (pc, nc), parts = _pair(neo_gpu, oracle, C, B, P, 5300)
    pc.set_persistent(True, idle_ms=5.0)
    nb = 400
    x = np.stack([oracle.noise(5400 + c, B * nb) for c in range(C)])
    t = torch.from_numpy(x.copy()).cuda()
    torch.cuda.current_stream().synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    for i in range(nb):
        if i in (100, 101, 250):
            time.sleep(0.03)  # past the idle limit
        if i == 300:
            pc.set_persistent(False)  # hand back: the normal step re-primes
        pc.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, x.shape[1], 1, stream)
    torch.cuda.current_stream().synchronize()
    got = t.cpu().numpy()
    assert pc.persistent_info()["launches"] >= 4
    assert same_sums(got, _run(nc, x, B, torch))
    assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL


def test_latency_mode_host_buffers(neo_gpu, oracle):
    """the plugin's call (neo_hip_upols_process on a host block, in place) in latency mode:
    page-locked (read and written in place by the kernel) and pageable (the handle's staging)."""
    torch = pytest.importorskip("torch")
    C, B, P = 1, 512, 188
    (pc, nc), parts = _pair(neo_gpu, oracle, C, B, P, 5500)
    pc.set_persistent(True)
    nb = 300
    x = np.stack([oracle.noise(5600, B * nb)])
    pinned = torch.empty((C, B), dtype=torch.float32).pin_memory().numpy()
    y = np.empty_like(x)
    for i in range(nb):
        blk = x[:, i * B:(i + 1) * B]
        if i % 2:
            pinned[:] = blk
            pc(pinned)
            y[:, i * B:(i + 1) * B] = pinned
        else:
            b = blk.copy()
            pc(b)
            y[:, i * B:(i + 1) * B] = b
    assert same_sums(y, _run(nc, x, B, torch))


def test_latency_mode_rejects_other_shapes(neo_gpu):
    """more than 16 channels, B > 512 with the streaming levels, sub-block v2, the far band as a 128-block Toeplitz level or
    recomputed every window: EINVAL"""
    for args, kw in (((32, 128, 100), {}), ((1, 1024, 100), {}), ((1, 256, 100), {"method": "upola_v2"}),
                     ((1, 512, 300), {"options": {"far_level": 0}}), ((1, 512, 300), {"options": {"far_level": 2}})):
        c = neo_gpu.UpolsConvolver(*args, **kw)
        with pytest.raises(RuntimeError, match="latency mode"):
            c.set_persistent(True)
        c.close()


@pytest.mark.parametrize("how", ["reset", "filter", "paced"])
def test_latency_mode_restart_after_short_run(neo_gpu, oracle, how):
    """A schedule that restarts before its first lap of the mailbox (10 one-block calls, then
    reset / set_filter / a set_paced toggle, then 10 more): no record of the first run may be
    taken for a step of the second (every step below 64 carries the same lap tag). The kernel
    stays resident across the setup call (idle limit 3 s), so only the cleared mailbox keeps
    the second run's steps apart. After reset / set_filter the second run equals the oracle on
    its blocks alone; after the paced toggle (state kept) the whole 20 blocks do."""
    torch = pytest.importorskip("torch")
    C, B, P = 1, 256, 100
    (pc, _), parts = _pair(neo_gpu, oracle, C, B, P, 5700)
    pc.set_persistent(True, idle_ms=3000.0)
    x = np.stack([oracle.noise(5800, B * 20)])
    first = _run(pc, x[:, : 10 * B], B, torch)
    assert peak_err(first, oracle.dense_convolve(x[:, : 10 * B], parts)) <= TOL
    if how == "reset":
        pc.reset()
    elif how == "filter":
        pc.filter(parts)
    else:
        pc.set_paced(True)
    pc.set_persistent(True, idle_ms=3000.0)
    second = _run(pc, x[:, 10 * B:], B, torch)
    if how == "paced":
        ref = oracle.dense_convolve(x, parts)[:, 10 * B:]
    else:
        ref = oracle.dense_convolve(x[:, 10 * B:], parts)
    assert peak_err(second, ref) <= TOL
    pc.set_persistent(False)
    pc.close()


def test_setup_call_does_not_wait_for_another_latency_kernel(neo_gpu, oracle):
    """Two handles: A in latency mode with its kernel resident (idle limit 3 s); a filter change
    and a reset on B return in well under that (setup calls join B's own streams, not the
    device), and A keeps stepping correctly afterwards."""
    torch = pytest.importorskip("torch")
    C, B, P = 1, 256, 100
    (pa, pb), parts = _pair(neo_gpu, oracle, C, B, P, 5900)
    pa.set_persistent(True, idle_ms=3000.0)
    x = np.stack([oracle.noise(6000, B * 8)])
    first = _run(pa, x[:, : 4 * B], B, torch)
    assert pa.persistent_info()["running"]
    t0 = time.perf_counter()
    pb.filter(parts)
    pb.reset()
    dt = time.perf_counter() - t0
    assert dt < 1.0, f"setup on another handle waited {dt:.2f} s for the resident kernel"
    second = _run(pa, x[:, 4 * B:], B, torch)
    got = np.concatenate([first, second], axis=1)
    assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL
    pa.set_persistent(False)
    pa.close()
    pb.close()


def _far_pair(neo_gpu, oracle, C, B, L, seed):
    """a latency-mode handle and a normal one whose far phase 2 is the same one-workgroup-per-unit
    form (far2c_role) the persistent kernel runs: the same sums in the same order"""
    P = neo_gpu.num_partitions(L, B)
    ir = np.stack([oracle.noise(seed + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    pc = neo_gpu.UpolsConvolver(C, B, P)
    nc = neo_gpu.UpolsConvolver(C, B, P, options={"far_phase2": 1})
    for c in (pc, nc):
        c.filter(parts)
        c.set_batch(False)
    assert pc.far_form() == 1
    return pc, nc, parts


def test_latency_mode_far_level_10s_ir(neo_gpu, oracle):
    """The plugin's real-time case at the headline's IR (one channel, B = 512, L = 480000: P = 938,
    six far segments): 640 one-block calls (five far windows: every segment meets real FDL rows,
    the ring of 969 rows wraps) through the persistent kernel's far workgroups, against the oracle
    (uniform_partitioned_convolver.hpp:47-65) and the normal step bit for bit."""
    torch = pytest.importorskip("torch")
    C, B, L, nb = 1, 512, 480000, 640
    pc, nc, parts = _far_pair(neo_gpu, oracle, C, B, L, 6400)
    pc.set_persistent(True)
    x = np.stack([oracle.noise(6500, B * nb)])
    got = _run(pc, x, B, torch)
    assert pc.persistent_info()["launches"] >= 1
    assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL
    assert same_sums(got, _run(nc, x, B, torch))
    pc.set_persistent(False)


def test_latency_mode_far_level_channels_relaunch(neo_gpu, oracle):
    """4 channels, B = 256, P = 600 (three far segments), idle limit 5 ms with pauses (relaunches
    mid-window and at a far window's first block) and calls of 1 and 3 blocks: the oracle and the
    normal step bit for bit."""
    torch = pytest.importorskip("torch")
    C, B, L = 4, 256, 600 * 256
    pc, nc, parts = _far_pair(neo_gpu, oracle, C, B, L, 6600)
    pc.set_persistent(True, idle_ms=5.0)
    nb = 700
    x = np.stack([oracle.noise(6700 + c, B * nb) for c in range(C)])
    t = torch.from_numpy(x.copy()).cuda()
    torch.cuda.current_stream().synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    i = 0
    while i < nb:
        if i in (130, 256, 257, 400):
            time.sleep(0.03)  # past the idle limit: the next call relaunches
        k = 3 if 300 <= i < 360 and i + 3 <= nb else 1
        pc.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, x.shape[1], k, stream)
        i += k
    torch.cuda.current_stream().synchronize()
    got = t.cpu().numpy()
    assert pc.persistent_info()["launches"] >= 4
    chans = [0, 3]
    assert peak_err(got[chans], oracle.dense_convolve(x[chans], parts[chans])) <= TOL
    assert same_sums(got, _run(nc, x, B, torch))
    pc.set_persistent(False)


@pytest.mark.parametrize("C,B,L,nb", [(16, 128, 128 * 700, 420), (16, 512, 480000, 300)])
def test_latency_mode_far_level_16_channels(neo_gpu, oracle, C, B, L, nb):
    """The latency mode's largest channel count with the far level: 16 channels (B = 128 with six
    far segments; the headline's B = 512 and 10 s IR), one call per block through two far windows,
    against the oracle on four channels and the normal step bit for bit on all 16."""
    torch = pytest.importorskip("torch")
    pc, nc, parts = _far_pair(neo_gpu, oracle, C, B, L, 6800 + B)
    pc.set_persistent(True, idle_ms=200.0)
    x = np.stack([oracle.noise(6900 + c, B * nb) for c in range(C)])
    got = _run(pc, x, B, torch)
    assert pc.persistent_info()["running"]
    chans = [0, 5, 10, 15]
    assert peak_err(got[chans], oracle.dense_convolve(x[chans], parts[chans])) <= TOL
    assert same_sums(got, _run(nc, x, B, torch))
    pc.set_persistent(False)


@pytest.mark.parametrize("L", [2 ** 11, 2 ** 14, 2 ** 17])
def test_latency_mode_plain_step_b4096(neo_gpu, oracle, L):
    """The reference benchmark's shape (extra/benchmark/src/convolution.cpp:47-55: one channel,
    B = 4096, IR 2^11..2^17, one call per block): P = 1..32 partitions, no streaming levels, so the
    plain fused step runs as the persistent kernel (k_plain_persist). Against the oracle and the
    normal one-launch step bit for bit (the same workgroup body, upols_step_wg)."""
    torch = pytest.importorskip("torch")
    B = 4096
    P = neo_gpu.num_partitions(L, B)
    ir = np.stack([oracle.noise(7000 + L % 97, L)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    pc = neo_gpu.UpolsConvolver(1, B, P)
    nc = neo_gpu.UpolsConvolver(1, B, P)
    for c in (pc, nc):
        c.filter(parts)
        c.set_batch(False)
    assert not pc.ahead_info()[0]
    pc.set_persistent(True)
    nb = P + 40
    x = np.stack([oracle.noise(7100, B * nb)])
    got = _run(pc, x, B, torch)
    info = pc.persistent_info()
    assert info["launches"] >= 1 and info["running"], info
    st = pc.persist_step_times()
    assert len(st) == min(63, nb) and all(0 < s < 1000 for s in st), st[:4]
    assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL
    assert same_sums(got, _run(nc, x, B, torch))
    pc.set_persistent(False)
    pc.close()
    nc.close()


@pytest.mark.parametrize("method,C,B,P", [("upols", 4, 512, 40), ("upola", 3, 256, 63), ("upols", 16, 64, 20),
                                          ("upols", 2, 2048, 12)])
def test_latency_mode_plain_step_channels_relaunch(neo_gpu, oracle, method, C, B, P):
    """k_plain_persist with several channels (the last channel's tail signals), OLA, small and
    large blocks; idle limit 5 ms with pauses (relaunches keep the FDL ring and write position),
    calls of 1 and 3 blocks, switched off mid-stream (the normal step continues from the same
    state): the normal step bit for bit, and the oracle for upols."""
    torch = pytest.importorskip("torch")
    (pc, nc), parts = _pair(neo_gpu, oracle, C, B, P, 7200 + C, method)
    assert not pc.ahead_info()[0]
    pc.set_persistent(True, idle_ms=5.0)
    nb = 2 * P + 50
    x = np.stack([oracle.noise(7300 + c, B * nb) for c in range(C)])
    t = torch.from_numpy(x.copy()).cuda()
    torch.cuda.current_stream().synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    i = 0
    while i < nb:
        if i in (P // 2, P + 33):
            time.sleep(0.03)  # past the idle limit: the next call relaunches
        if i == nb - 20:
            pc.set_persistent(False)  # hand back to the normal step
        k = 3 if P <= i < P + 30 and i + 3 <= nb else 1
        pc.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, x.shape[1], k, stream)
        i += k
    torch.cuda.current_stream().synchronize()
    got = t.cpu().numpy()
    assert pc.persistent_info()["launches"] >= 3
    assert same_sums(got, _run(nc, x, B, torch))
    if method == "upols":
        assert peak_err(got, oracle.dense_convolve(x, parts)) <= TOL


def test_latency_mode_plain_step_host_buffers(neo_gpu, oracle):
    """the plugin's call (neo_hip_upols_process on a host block, in place) at B = 4096, P = 32:
    page-locked and pageable blocks through the plain persistent kernel, against the oracle."""
    pytest.importorskip("torch")
    import torch
    C, B, P = 1, 4096, 32
    (pc, nc), parts = _pair(neo_gpu, oracle, C, B, P, 7500)
    pc.set_persistent(True)
    nb = 60
    x = np.stack([oracle.noise(7600, B * nb)])
    pinned = torch.empty((C, B), dtype=torch.float32).pin_memory().numpy()
    y = np.empty_like(x)
    for i in range(nb):
        blk = x[:, i * B:(i + 1) * B]
        if i % 2:
            pinned[:] = blk
            pc(pinned)
            y[:, i * B:(i + 1) * B] = pinned
        else:
            b = blk.copy()
            pc(b)
            y[:, i * B:(i + 1) * B] = b
    assert peak_err(y, oracle.dense_convolve(x, parts)) <= TOL
    assert same_sums(y, _run(nc, x, B, torch))
