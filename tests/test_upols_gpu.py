"""GPU parity of the UPOLS path (libneo_hip.so via the C-ABI) against the CPU
restatement of upols_convolver / dense_convolve and the golden fixtures.

Tolerance (BASELINE.json north_star: <= 1e-5 rel, float32) read as SURVEY §8(a):
max|y - y_ref| / max|y_ref| <= 1e-5 (peak-normalized), plus the reference's
per-sample abs 1e-5 on the identity tests (uniform_partitioned_convolver_test.cpp:74)."""
import os

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
TOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def identity_impulse(B, n):
    """generate_identity_impulse (src/neo/testing/testing.hpp:74-82)."""
    h = np.zeros((n, B + 1), np.complex64)
    h[0] = 1
    return h


@pytest.mark.parametrize("B", [128, 256, 512, 1024])
def test_identity_ir(neo_gpu, oracle, B):
    """uniform_partitioned_convolver_test.cpp:35-75: identity IR, 20 noise blocks, out == in."""
    sig = oracle.noise(11, B * 20)
    conv = neo_gpu.upols_convolver()
    conv.filter(identity_impulse(B, 3))
    out = sig.copy()
    for i in range(0, len(out), B):
        blk = np.ascontiguousarray(out[i:i + B])
        conv(blk)
        out[i:i + B] = blk
    assert np.abs(out - sig).max() <= 1e-5


@pytest.mark.parametrize("B,L,C,nb", [(512, 4096, 1, 40), (256, 2560, 2, 40), (128, 1000, 3, 30),
                                      (16, 100, 2, 20), (64, 64, 1, 10), (1024, 5000, 2, 12),
                                      (2048, 9000, 1, 6), (4096, 12000, 1, 5), (32, 7, 1, 8)])
@pytest.mark.parametrize("fused", [0, 1])
def test_random_ir_vs_oracle(neo_gpu, oracle, B, L, C, nb, fused):
    """Both plain step forms for the single blocks after the batched passes: MAC + finish
    launches, and one launch with the last-arriver tail (the default below 64 MiB of
    filter + FDL)."""
    ir = np.stack([oracle.noise(20 + c, L) for c in range(C)])
    irn = oracle.normalize_impulse(ir)
    parts = oracle.uniform_partition(irn, B)
    sig = np.stack([oracle.noise(30 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts)
    got = neo_gpu.dense_convolve(sig, ir, B, options={"fused": fused, "levels": 0})
    assert peak_err(got, ref) <= TOL
    assert np.abs(got - ref).max() <= 1e-5


@pytest.mark.parametrize("name", ["upols_b512_l4096_seed5", "upols_b256_l2560_2ch_seed6",
                                  "upols_b512_l96000_seed7"])
def test_golden_upols(neo_gpu, name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    B = 256 if "b256" in name else 512
    got = neo_gpu.dense_convolve(g["signal"], g["ir"], B)
    assert peak_err(got, g["out"]) <= TOL
    assert np.abs(got - g["out"]).max() <= 1e-5


def test_uniform_partition_vs_oracle(neo_gpu, oracle):
    g = np.load(os.path.join(GOLD, "partition_seed4.npz"))
    H = neo_gpu.uniform_partition(g["ir"][None], 256)
    assert H.shape == (1, 12, 257)
    assert peak_err(H, g["H"]) <= TOL
    H2 = neo_gpu.uniform_partition(g["ir2_norm"], 128)
    assert peak_err(H2, g["H2"]) <= TOL
    # uniform_partition_test.cpp:8-37 shapes
    for C, L in [(1, 4096), (2, 4096), (2, 4095)]:
        assert neo_gpu.uniform_partition(np.zeros((C, L), np.float32), 128).shape == (C, 32, 129)


def test_normalize_impulse_bit_exact(neo_gpu, oracle):
    """Sequential float energy (normalize_energy.hpp:21-33): the GPU rounds identically."""
    # up to 10 s @ 48 kHz, where rounding order matters most; ragged C (not a multiple of
    # the 16-channel group) and L (not a multiple of the 256-sample tile)
    for C, L in [(4, 48000), (2, 480000), (17, 48001), (3, 255), (1, 1), (20, 256)]:
        ir = np.stack([oracle.noise(50 + c, L) * (c + 1) for c in range(C)]).astype(np.float32)
        ref = oracle.normalize_impulse(ir)
        got = ir.copy()
        neo_gpu.normalize_impulse(got)
        assert np.array_equal(got, ref), (C, L)
    # normalize_impulse_test.cpp:13-56 known answers
    v = np.zeros(33, np.float32)
    v[0] = 2
    neo_gpu.normalize_impulse(v)
    assert v[0] == pytest.approx(1.0)
    v[0] = v[1] = 2
    neo_gpu.normalize_impulse(v)
    assert v[0] == pytest.approx(0.707106782) and v[1] == pytest.approx(0.707106782)
    m = np.zeros((33, 66), np.float32)
    m[0, 0] = 2
    neo_gpu.normalize_impulse(m)
    assert m[0, 0] == pytest.approx(1.0)


def test_ring_order_delay(neo_gpu, oracle):
    """fdl_index ring (fdl_index.hpp:23-36): a filter whose only nonzero partition is p
    delays the input by exactly p blocks."""
    B, P = 128, 5
    sig = oracle.noise(60, B * 16)
    for p in range(P):
        H = np.zeros((P, B + 1), np.complex64)
        H[p] = 1
        c = neo_gpu.UpolsConvolver(1, B, P)
        c.filter(H[None])
        out = np.empty_like(sig)
        for t in range(16):
            blk = sig[t * B:(t + 1) * B][None].copy()  # a view would be processed in place
            c(blk)
            out[t * B:(t + 1) * B] = blk[0]
        expect = np.concatenate([np.zeros(p * B, np.float32), sig[: len(sig) - p * B]])
        assert np.abs(out - expect).max() <= 1e-5, p


def test_set_filter_equals_set_impulse_and_reset(neo_gpu, oracle):
    B, L, C = 256, 3000, 3
    ir = np.stack([oracle.noise(70 + c, L) for c in range(C)])
    P = neo_gpu.num_partitions(L, B)
    a = neo_gpu.UpolsConvolver(C, B, P)
    b = neo_gpu.UpolsConvolver(C, B, P)
    a.set_impulse(ir, normalize=True)
    b.filter(oracle.uniform_partition(oracle.normalize_impulse(ir), B))
    blocks = [np.ascontiguousarray(np.stack([oracle.noise(80 + 10 * t + c, B) for c in range(C)])) for t in range(12)]
    ya = [a(x.copy()) for x in blocks]
    yb = [b(x.copy()) for x in blocks]
    assert max(np.abs(p - q).max() for p, q in zip(ya, yb)) <= 1e-5
    a.reset()
    ya2 = [a(x.copy()) for x in blocks]
    assert max(np.abs(p - q).max() for p, q in zip(ya, ya2)) == 0.0  # deterministic after reset


@pytest.mark.parametrize("levels", [0, 1])
def test_host_buffers_zero_copy(neo_gpu, oracle, levels):
    """Host-buffer blocks (neo_hip_upols_process, the plugin's processFrame call,
    DenseConvolution.cpp:62-74): pageable memory through the mapped staging, page-locked
    memory (torch pinned tensors = hipHostMalloc; numpy arrays page-locked with
    neo.host_register) read and written in place by the step kernel. All three equal the
    device-resident step bit for bit; a misaligned registered view falls back to staging."""
    torch = pytest.importorskip("torch")
    B, L, C, nb = 256, 256 * 70, 3, 24
    ir = np.stack([oracle.noise(980 + c, L) for c in range(C)])
    P = neo_gpu.num_partitions(L, B)
    sig = np.stack([oracle.noise(990 + c, B * nb) for c in range(C)])
    opts = {"levels": levels}
    dev = neo_gpu.UpolsConvolver(C, B, P, options=opts)
    dev.set_impulse(ir)
    dev.set_batch(False)
    t = torch.from_numpy(sig).cuda()
    dev.process_blocks(t)
    torch.cuda.synchronize()
    ref = t.cpu().numpy()
    convs = [neo_gpu.UpolsConvolver(C, B, P, options=opts) for _ in range(4)]
    for c in convs:
        c.set_impulse(ir)
    pinned = torch.empty((C, B), dtype=torch.float32).pin_memory()
    reg = np.empty((C, B + 4), np.float32)  # registered; rows B apart at an offset: a copy lands in it
    neo_gpu.host_register(reg)
    try:
        regv = np.ndarray((C, B), np.float32, buffer=reg, offset=0, strides=(4 * B, 4))
        odd = np.ndarray((C, B), np.float32, buffer=reg, offset=4, strides=(4 * B, 4))  # 4-byte aligned
        outs = [np.empty_like(sig) for _ in convs]
        for i in range(nb):
            blk = sig[:, i * B:(i + 1) * B]
            a = np.ascontiguousarray(blk)
            convs[0](a)
            outs[0][:, i * B:(i + 1) * B] = a
            pinned.numpy()[:] = blk
            convs[1](pinned)
            outs[1][:, i * B:(i + 1) * B] = pinned.numpy()
            regv[:] = blk
            convs[2](regv)
            outs[2][:, i * B:(i + 1) * B] = regv
            odd[:] = blk
            convs[3](odd)
            outs[3][:, i * B:(i + 1) * B] = odd
    finally:
        neo_gpu.host_unregister(reg)
    for k, o in enumerate(outs):
        assert np.array_equal(o, ref), k


def test_errors(neo_gpu):
    with pytest.raises(RuntimeError):
        neo_gpu.UpolsConvolver(1, 500, 4)  # not a power of two
    with pytest.raises(RuntimeError):
        neo_gpu.UpolsConvolver(0, 512, 4)
    c = neo_gpu.UpolsConvolver(2, 128, 3)
    with pytest.raises(ValueError):
        c.filter(np.zeros((2, 4, 129), np.complex64))
    with pytest.raises(RuntimeError):
        c.set_impulse(np.zeros((2, 1000), np.float32))  # 8 partitions != 3


def test_device_blocks_match_host_blocks(neo_gpu, oracle):
    torch = pytest.importorskip("torch")
    B, L, C, nb = 512, 20000, 4, 72
    ir = np.stack([oracle.noise(90 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(95 + c, B * nb) for c in range(C)])
    P = neo_gpu.num_partitions(L, B)
    # host blocks one at a time: the streaming step
    host = neo_gpu.UpolsConvolver(C, B, P)
    host.set_impulse(ir)
    ref = sig.copy()
    for i in range(nb):
        blk = np.ascontiguousarray(ref[:, i * B:(i + 1) * B])
        host(blk)
        ref[:, i * B:(i + 1) * B] = blk
    assert peak_err(neo_gpu.dense_convolve(sig, ir, B), ref) <= TOL  # batched passes
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.set_impulse(torch.from_numpy(ir).cuda(), normalize=True)
    t = torch.from_numpy(sig).cuda()
    out = torch.empty_like(t)
    conv.process_blocks(t, out)  # batched passes: same math, another summation order
    torch.cuda.synchronize()
    assert peak_err(out.cpu().numpy(), ref) <= TOL
    conv.reset()
    conv.process_blocks(t)  # in place
    torch.cuda.synchronize()
    assert peak_err(t.cpu().numpy(), ref) <= TOL
    # one block per pass through the same entry point is the streaming step, bit for bit
    conv1 = neo_gpu.UpolsConvolver(C, B, P)
    conv1.set_batch(False)
    conv1.set_impulse(torch.from_numpy(ir).cuda(), normalize=True)
    t = torch.from_numpy(sig).cuda()
    conv1.process_blocks(t)
    torch.cuda.synchronize()
    assert np.abs(t.cpu().numpy() - ref).max() == 0.0


@pytest.mark.parametrize("C,B,L", [(256, 256, 480000), (256, 512, 480000)])
def test_full_size_properties(neo_gpu, oracle, C, B, L):
    """C4 / C5-per-GPU shapes at full size: (a) three channels spot-checked against the
    oracle over the first blocks, (b) linearity over the whole multichannel state."""
    torch = pytest.importorskip("torch")
    nb = 6
    g = torch.Generator(device="cuda").manual_seed(C + B)
    ir = (torch.rand((C, L), generator=g, device="cuda") * 2 - 1).contiguous()
    x = (torch.rand((C, B * nb), generator=g, device="cuda") * 2 - 1).contiguous()
    y = (torch.rand((C, B * nb), generator=g, device="cuda") * 2 - 1).contiguous()
    P = neo_gpu.num_partitions(L, B)
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.set_impulse(ir, normalize=True)
    ox = conv.process_blocks(x.clone())
    conv.reset()
    oy = conv.process_blocks(y.clone())
    conv.reset()
    oxy = conv.process_blocks((0.5 * x + y).contiguous())
    torch.cuda.synchronize()
    lin = 0.5 * ox + oy
    assert (torch.max(torch.abs(oxy - lin)) / torch.max(torch.abs(lin))).item() <= 1e-5
    irh = oracle.normalize_impulse(ir.cpu().numpy())
    xh = x.cpu().numpy()
    for c in (0, C // 2, C - 1):
        parts = oracle.uniform_partition(irh[c:c + 1], B)
        ref = oracle.dense_convolve(xh[c:c + 1], parts)
        assert peak_err(ox[c].cpu().numpy(), ref[0]) <= TOL


def _full_size_streaming(neo_gpu, oracle, C, B, L, nb, seed, chans, far_group=None, far_level=-1, far_form=None):
    """Default options (streaming levels on, far level on), device input, one block per
    call as a real-time caller steps it, nb blocks: every level's windows repeat many times,
    every far segment meets real FDL rows and the ring wraps. Channels `chans` against the
    oracle's dense_convolve over the whole stream."""
    torch = pytest.importorskip("torch")
    g = torch.Generator(device="cuda").manual_seed(seed)
    ir = (torch.rand((C, L), generator=g, device="cuda") * 2 - 1).contiguous()
    x = (torch.rand((C, B * nb), generator=g, device="cuda") * 2 - 1).contiguous()
    P = neo_gpu.num_partitions(L, B)
    conv = neo_gpu.UpolsConvolver(C, B, P, options={"far_level": far_level})
    assert conv.ahead_info()[0]  # streaming levels are the default here
    if far_group is not None:
        assert conv.far_group() == far_group  # the automatic choice at this shape
    if far_form is not None:
        assert conv.far_form() == far_form
    conv.set_impulse(ir, normalize=True)
    conv.set_batch(False)  # one block per pass
    xh = {c: x[c].cpu().numpy()[None] for c in chans}
    # one normalization factor over all channels (normalize_impulse.hpp:21-30)
    irh = oracle.normalize_impulse(ir.cpu().numpy())
    irc = {c: irh[c:c + 1].copy() for c in chans}
    del irh
    tail = 128 * B  # the last far window (steady state, the ring wrapped many times)
    x_in = x[:, -(P + 128) * B:].clone()  # the blocks the plain step needs for that window
    conv.process_blocks(x)
    torch.cuda.synchronize()
    conv.close()
    refs = {}
    for c in chans:
        ref = oracle.dense_convolve(xh[c], oracle.uniform_partition(irc[c], B))
        refs[c] = ref[0, -tail:]
        assert peak_err(x[c].cpu().numpy(), ref[0]) <= TOL, c
        assert peak_err(x[c, -tail:].cpu().numpy(), refs[c]) <= TOL, c
    # EVERY channel over the last far window against the plain step (k_upols_step: one pass over
    # all P partitions per block; test_random_ir_vs_oracle, and the sampled channels below), run on the same input: a
    # fault confined to channels the oracle does not sample cannot pass. The plain handle starts
    # from zero state P + 128 blocks before the end, so its last 128 blocks see exactly the
    # streaming run's FDL contents (every partition covered by real rows).
    plain = neo_gpu.UpolsConvolver(C, B, P, options={"levels": 0})
    assert not plain.ahead_info()[0]
    plain.set_impulse(ir, normalize=True)
    plain.set_batch(False)
    del ir
    plain.process_blocks(x_in)
    torch.cuda.synchronize()
    plain.close()
    for c in chans:
        assert peak_err(x_in[c, -tail:].cpu().numpy(), refs[c]) <= TOL, c
    a, b = x[:, -tail:], x_in[:, -tail:]
    err = (torch.amax(torch.abs(a - b), dim=1) / torch.amax(torch.abs(b), dim=1)).cpu().numpy()
    assert err.max() <= TOL, (int(err.argmax()), float(err.max()))


@pytest.mark.parametrize("far_level,form", [(-1, 1), (2, 2)])
def test_full_size_c5_shard_steady_state(neo_gpu, oracle, far_level, form):
    """The headline path at its own shape (configs[4] per-GPU shard: 256 ch, B = 512,
    L = 480000, P = 938, 6 far segments, ring 1194 / 969): 1152 blocks (9 far windows), channels
    0, 127, 255; the default far level (stored spectra) and the one recomputed every window."""
    _full_size_streaming(neo_gpu, oracle, 256, 512, 480000, 1152, 77, (0, 127, 255), far_level=far_level,
                         far_form=form)


@pytest.mark.parametrize("far_level,form,K", [(-1, 1, 3), (2, 2, 1)])
def test_full_size_c5full_steady_state(neo_gpu, oracle, far_level, form, K):
    """The headline workload itself (configs[4]'s 2048 channels on one GPU, B = 512,
    L = 480000, P = 938): the default far level (stored spectra), which at 32768 16-column units
    runs window groups of K = 3 (far1_mac<FPL, 3> and phase 2's extra segments), and the one
    recomputed every window: 1152 blocks (9 far windows, the ring wraps), channels 0, 1024 and
    2047."""
    _full_size_streaming(neo_gpu, oracle, 2048, 512, 480000, 1152, 79, (0, 1024, 2047), far_group=K,
                         far_level=far_level, far_form=form)


def test_c3_streaming_exact_shape(neo_gpu, oracle):
    """configs[2] at its exact shape as the bench steps it (B = 512, L = 96000 -> P = 188,
    1 channel, streaming levels: block step + Toeplitz 4..32 + no far level): the golden
    fixture's 200 blocks one block per call, then 640 single-block steps of fresh noise
    against the oracle's dense_convolve (uniform_partitioned_convolver.hpp:47-65)."""
    torch = pytest.importorskip("torch")
    g = np.load(os.path.join(GOLD, "upols_b512_l96000_seed7.npz"))
    B = 512
    P = neo_gpu.num_partitions(g["ir"].shape[-1], B)
    assert P == 188
    conv = neo_gpu.UpolsConvolver(1, B, P)
    assert conv.ahead_info()[0]  # the streaming form is the default at this shape
    conv.set_impulse(np.atleast_2d(g["ir"]), normalize=True)
    conv.set_batch(False)
    sig = np.atleast_2d(g["signal"]).astype(np.float32)
    nb = sig.shape[1] // B
    t = torch.from_numpy(sig[:, : nb * B].copy()).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    for i in range(nb):  # one call per block, in place
        p = t.data_ptr() + 4 * i * B
        conv.process_blocks_ptr(p, p, nb * B, 1, stream)
    torch.cuda.synchronize()
    out = np.atleast_2d(g["out"])[:, : nb * B]
    assert peak_err(t.cpu().numpy(), out) <= TOL
    assert np.abs(t.cpu().numpy() - out).max() <= 1e-5
    # fresh noise, 640 blocks (several windows of every level, the ring of 219 rows wraps)
    nb2 = 640
    x = np.stack([oracle.noise(4242, B * nb2)])
    irn = oracle.normalize_impulse(np.atleast_2d(g["ir"]).astype(np.float32))
    ref = oracle.dense_convolve(x, oracle.uniform_partition(irn, B))
    conv.reset()
    tx = torch.from_numpy(x.copy()).cuda()
    conv.process_blocks(tx)
    torch.cuda.synchronize()
    assert peak_err(tx.cpu().numpy(), ref) <= TOL


def test_full_size_c4_steady_state(neo_gpu, oracle):
    """configs[3] (256 ch, B = 256, L = 480000, P = 1875, 13 far segments): 2176 blocks
    (17 far windows, the ring of 1906 rows wraps), channels 0, 127 and 255."""
    _full_size_streaming(neo_gpu, oracle, 256, 256, 480000, 2176, 78, (0, 127, 255))


def test_multirow_splits_with_wraparound(neo_gpu, oracle):
    """More blocks than partitions and several partitions per split (every split carries
    nonzero FDL rows, ring wraps), plain MAC + finish steps with forced split targets."""
    B, L, C, nb = 128, 50 * 128, 2, 130  # P = 50
    ir = np.stack([oracle.noise(700 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(710 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, oracle.uniform_partition(oracle.normalize_impulse(ir), B))
    for target in (6, 1, 64):
        P = neo_gpu.num_partitions(L, B)
        conv = neo_gpu.UpolsConvolver(C, B, P, options={"split_workgroups": target, "fused": 0, "levels": 0})
        conv.set_impulse(ir)
        out = np.empty_like(sig)
        for t in range(nb):
            blk = np.ascontiguousarray(sig[:, t * B:(t + 1) * B])
            conv(blk)
            out[:, t * B:(t + 1) * B] = blk
        # S = ceil(P / ceil(P / min(ceil(t/C), P, 64))): an explicit target is taken as given
        assert conv.splits == {6: 3, 1: 1, 64: 25}[target]
        assert peak_err(out, ref) <= TOL, (target, conv.splits)


# ---------------------------------------------------------------- UPOLA (overlap-add stage)
@pytest.mark.parametrize("B", [128, 256, 512, 1024])
def test_upola_identity_ir(neo_gpu, oracle, B):
    """uniform_partitioned_convolver_test.cpp:35-75 with upola_convolver / split_upola_convolver."""
    for cls in (neo_gpu.upola_convolver, neo_gpu.split_upola_convolver):
        sig = oracle.noise(B + 3, B * 20)
        conv = cls()
        conv.filter(identity_impulse(B, 3))
        out = sig.copy()
        for i in range(0, len(out), B):
            blk = out[i:i + B].copy()
            conv(blk)
            out[i:i + B] = blk
        assert np.abs(out - sig).max() <= 1e-5


@pytest.mark.parametrize("B,L,C,nb", [(512, 4096, 1, 40), (256, 2560, 2, 40), (128, 1000, 3, 30), (16, 100, 2, 20),
                                      (2048, 9000, 1, 6), (4096, 12000, 1, 5), (64, 64 * 50, 2, 120)])
def test_upola_random_ir_vs_oracle(neo_gpu, oracle, B, L, C, nb):
    ir = np.stack([oracle.noise(120 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    sig = np.stack([oracle.noise(130 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts, method="upola")
    got = neo_gpu.dense_convolve(sig, ir, B, method="upola")
    assert peak_err(got, ref) <= TOL
    assert np.abs(got - ref).max() <= 1e-5


def test_golden_upola(neo_gpu):
    g = np.load(os.path.join(GOLD, "upola_b256_l2560_2ch_seed8.npz"))
    got = neo_gpu.dense_convolve(g["signal"], g["ir"], 256, method="upola")
    assert peak_err(got, g["out"]) <= TOL


def test_upola_equals_upols(neo_gpu, oracle):
    """Both stages compute the same linear convolution of the stream."""
    B, L, C, nb = 256, 4000, 2, 30
    ir = np.stack([oracle.noise(140 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(150 + c, B * nb) for c in range(C)])
    a = neo_gpu.dense_convolve(sig, ir, B, method="upols")
    b = neo_gpu.dense_convolve(sig, ir, B, method="upola")
    assert peak_err(b, a) <= TOL


def test_fused_step_matches_two_launch(neo_gpu, oracle):
    """The one-launch plain step (last-arriver tail) equals the two-launch step."""
    B, L, C, nb = 256, 60 * 256, 3, 70
    ir = np.stack([oracle.noise(160 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(170 + c, B * nb) for c in range(C)])
    outs = []
    for fused in (0, 1):
        for method in ("upols", "upola"):
            # 4 splits per channel; the single blocks after the batched passes take the plain step
            opts = {"fused": fused, "split_workgroups": 12, "levels": 0}
            outs.append((fused, method, neo_gpu.dense_convolve(sig, ir, B, method=method, options=opts)))
    ref = {m: oracle.dense_convolve(sig, oracle.uniform_partition(oracle.normalize_impulse(ir), B), method=m)
           for m in ("upols", "upola")}
    for fused, method, out in outs:
        assert peak_err(out, ref[method]) <= TOL, (fused, method)


# ------------------------------------------- UPOLA v2 (overlap_add_convolver, sub-block input)
def _v2_reference(oracle, parts, sig, cuts):
    """oracle.Upola2 per channel over the same piece boundaries."""
    out = np.empty_like(sig)
    for c in range(sig.shape[0]):
        o = oracle.Upola2(parts[c])
        for a, b in zip(cuts[:-1], cuts[1:]):
            out[c, a:b] = o(sig[c, a:b])
    return out


@pytest.mark.parametrize("B", [128, 256, 512, 1024])
def test_upola_v2_identity_ir(neo_gpu, oracle, B):
    """uniform_partitioned_convolver_test.cpp:35-75 with upola_convolver_v2 (whole blocks),
    then uneven pieces (the identity filter passes any piece pattern through)."""
    sig = oracle.noise(B + 5, B * 20)
    conv = neo_gpu.upola_convolver_v2()
    conv.filter(identity_impulse(B, 3))
    out = sig.copy()
    for i in range(0, len(out), B):
        blk = out[i:i + B].copy()
        conv(blk)
        out[i:i + B] = blk
    assert np.abs(out - sig).max() <= 1e-5
    conv.filter(identity_impulse(B, 3))
    cuts = [0, B // 3, B + 5, 3 * B, 3 * B + 1, 7 * B - 2, len(sig)]
    out = np.concatenate([conv(sig[a:b].copy()) for a, b in zip(cuts[:-1], cuts[1:])])
    assert np.abs(out - sig).max() <= 1e-5


@pytest.mark.parametrize("B,L,C", [(128, 1000, 3), (256, 2560, 2), (512, 4096, 1), (16, 100, 2), (64, 64, 2),
                                   (4096, 12000, 1)])
def test_upola_v2_pieces_vs_oracle(neo_gpu, oracle, B, L, C):
    """Sub-block calls (host I/O) against the restatement of overlap_add_convolver::operator(),
    window reuse after the irfft included; whole aligned blocks take the UPOLA launch pair."""
    ir = np.stack([oracle.noise(180 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    N = B * 9
    sig = np.stack([oracle.noise(190 + c, N) for c in range(C)])
    cuts = sorted({0, 1, B // 2 + 1, B + B // 2 + 1, 3 * B + 1, 4 * B + 1, 4 * B + 2, 6 * B, 8 * B, N})
    ref = _v2_reference(oracle, parts, sig, cuts)
    conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method="upola_v2")
    conv.filter(parts)
    got = np.concatenate([conv.process(np.ascontiguousarray(sig[:, a:b])) for a, b in zip(cuts[:-1], cuts[1:])],
                         axis=1)
    assert peak_err(got, ref) <= TOL


def test_upola_v2_device_pieces_and_blocks(neo_gpu, oracle):
    """CUDA-tensor pieces (device path) equal host pieces; whole blocks equal upola."""
    torch = pytest.importorskip("torch")
    B, L, C = 256, 5000, 4
    ir = np.stack([oracle.noise(200 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    N = B * 12
    sig = np.stack([oracle.noise(210 + c, N) for c in range(C)])
    cuts = [0, 3, B + 3, 2 * B + 3, 5 * B, 5 * B + 77, 9 * B, N]
    ref = _v2_reference(oracle, parts, sig, cuts)
    conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method="upola_v2")
    conv.filter(parts)
    outs = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        t = torch.from_numpy(np.ascontiguousarray(sig[:, a:b])).cuda()
        conv.process(t)
        outs.append(t.cpu().numpy())
    got = np.concatenate(outs, axis=1)
    assert peak_err(got, ref) <= TOL
    # whole blocks: v2 == upola (same math; the launch pair does the work)
    v2 = neo_gpu.dense_convolve(sig, ir, B, method="upola_v2")
    v1 = neo_gpu.dense_convolve(sig, ir, B, method="upola")
    assert peak_err(v2, v1) <= TOL
    # reset returns to the initial state
    conv.reset()
    t = torch.from_numpy(np.ascontiguousarray(sig[:, :cuts[1]])).cuda()
    conv.process(t)
    assert peak_err(t.cpu().numpy(), ref[:, :cuts[1]]) <= TOL


def test_process_samples_errors(neo_gpu):
    c = neo_gpu.UpolsConvolver(2, 128, 3)  # upols: whole blocks only
    with pytest.raises(RuntimeError):
        c.process(np.zeros((2, 100), np.float32))
    c.process(np.zeros((2, 256), np.float32))  # two whole blocks are fine
    with pytest.raises(ValueError):
        neo_gpu.UpolsConvolver(1, 128, 3, method="upola_v3")


# ------------------------------------------------ batched passes (process_blocks, T blocks/pass)
@pytest.mark.parametrize("method", ["upols", "upola", "upola_v2"])
@pytest.mark.parametrize("B,L,C,nb", [(512, 20000, 3, 37), (256, 2560, 2, 29), (16, 100, 2, 40), (64, 64, 1, 19),
                                      (1024, 30000, 2, 21), (2048, 9000, 1, 11), (4096, 12000, 1, 9),
                                      (128, 128 * 40, 2, 100)])
def test_batched_blocks_vs_oracle(neo_gpu, oracle, method, B, L, C, nb):
    """process_blocks runs batch_cfg<B>::T blocks per MAC pass (sliding FDL window, ring of
    P + 31 rows); leftover blocks and the FDL wraparound (nb > P) included."""
    torch = pytest.importorskip("torch")
    ir = np.stack([oracle.noise(230 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    sig = np.stack([oracle.noise(240 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts, method="upols" if method == "upols" else "upola")
    conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method)
    conv.filter(parts)
    t = torch.from_numpy(sig).cuda()
    out = torch.empty_like(t)
    conv.process_blocks(t, out)
    torch.cuda.synchronize()
    assert peak_err(out.cpu().numpy(), ref) <= TOL


def test_batched_mixed_with_single_blocks(neo_gpu, oracle):
    """Batched passes, single-block steps and host blocks share one state (ring position,
    previous block / overlap) in any interleaving."""
    torch = pytest.importorskip("torch")
    B, L, C = 256, 7000, 3
    ir = np.stack([oracle.noise(250 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    for method in ("upols", "upola"):
        sig = np.stack([oracle.noise(260 + c, B * 60) for c in range(C)])
        ref = oracle.dense_convolve(sig, parts, method=method)
        conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method)
        conv.filter(parts)
        t = torch.from_numpy(sig).cuda()
        pos = 0
        for kind, n in [("batch", 13), ("one", 1), ("batch", 8), ("host", 1), ("batch", 3), ("one", 2),
                        ("batch", 32)]:
            seg = t[:, pos * B:(pos + n) * B].contiguous()
            if kind == "batch":
                conv.process_blocks(seg)
            elif kind == "one":
                for i in range(n):
                    blk = seg[:, i * B:(i + 1) * B].contiguous()
                    conv(blk)
                    seg[:, i * B:(i + 1) * B] = blk
            else:
                torch.cuda.synchronize()
                h = seg.cpu().numpy().copy()
                conv(h)
                seg = torch.from_numpy(h).cuda()
            t[:, pos * B:(pos + n) * B] = seg
            pos += n
        torch.cuda.synchronize()
        assert peak_err(t.cpu().numpy(), ref) <= TOL, method


@pytest.mark.parametrize("T", [2, 4, 8, 16, 32])
@pytest.mark.parametrize("nbins", [1, 2])
def test_every_batch_size(neo_gpu, oracle, T, nbins):
    """Each compiled batch size (and the smaller ones used for leftovers) against the oracle,
    with 1 or 2 bins per lane-vector."""
    torch = pytest.importorskip("torch")
    B, L, C = 256, 9000, 2
    nb = 2 * T + 3
    ir = np.stack([oracle.noise(270 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    sig = np.stack([oracle.noise(280 + c, B * nb) for c in range(C)])
    for method in ("upols", "upola"):
        ref = oracle.dense_convolve(sig, parts, method=method)
        conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method,
                                      options={"batch_blocks": T, "batch_bins": nbins})
        conv.filter(parts)
        assert conv.batch_info()[0] == min(T, 32 // nbins)  # accumulator cap at B = 256
        t = torch.from_numpy(sig).cuda()
        conv.process_blocks(t)
        torch.cuda.synchronize()
        assert peak_err(t.cpu().numpy(), ref) <= TOL, method


def test_timing_stride(neo_gpu):
    """set_timing(every=n) brackets every n-th MAC launch with a HIP event pair."""
    torch = pytest.importorskip("torch")
    conv = neo_gpu.UpolsConvolver(2, 128, 5)
    conv.set_batch(False)
    x = torch.zeros((2, 128 * 10), device="cuda")
    conv.set_timing(True, every=4)
    conv.process_blocks(x)
    conv.set_timing(False)
    ms, n = conv.timing()
    assert n == 3 and ms > 0  # launches 0, 4, 8
    conv.set_timing(True)
    conv.process_blocks(x)
    conv.set_timing(False)
    assert conv.timing()[1] == 10
    with pytest.raises(ValueError):
        conv.set_timing(True, every=0)


def test_host_staging_growth_keeps_batch_buffers(neo_gpu, oracle):
    """Host process() with a growing staging buffer between batched device passes: the
    batched partial / tail buffers stay valid (regression: the staging growth path freed
    them)."""
    torch = pytest.importorskip("torch")
    B, L, C = 128, 3000, 2
    ir = np.stack([oracle.noise(300 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    for method in ("upols", "upola"):
        sig = np.stack([oracle.noise(310 + c, B * 120) for c in range(C)])
        ref = oracle.dense_convolve(sig, parts, method=method)
        conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method)
        conv.filter(parts)
        out = np.empty_like(sig)
        pos = 0
        for kind, n in [("dev", 32), ("host", 2), ("dev", 32), ("host", 16), ("dev", 32), ("host", 6)]:
            seg = np.ascontiguousarray(sig[:, pos * B:(pos + n) * B])
            if kind == "dev":
                t = torch.from_numpy(seg).cuda()
                conv.process_blocks(t)
                torch.cuda.synchronize()
                seg = t.cpu().numpy()
            else:
                conv.process(seg)  # staging grows 2 -> 16 blocks
            out[:, pos * B:(pos + n) * B] = seg
            pos += n
        assert peak_err(out, ref) <= TOL, method


# ------------------------------------------------ streaming levels (upols_levels.hip)
def _stream(neo_gpu, oracle, method, B, P, C, nb, seed, options=None):
    """Single-block steps with the streaming levels against the oracle's dense_convolve."""
    torch = pytest.importorskip("torch")
    L = B * (P - 1) + B // 2 + 1
    ir = np.stack([oracle.noise(seed + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    assert parts.shape[1] == P
    sig = np.stack([oracle.noise(seed + 10 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts, method=method)
    conv = neo_gpu.UpolsConvolver(C, B, P, method=method, options=options)
    conv.filter(parts)
    conv.set_batch(False)
    conv.set_ahead(True)
    assert conv.ahead_info()[:2] == (True, 0)
    t = torch.from_numpy(sig).cuda()
    conv.process_blocks(t)
    torch.cuda.synchronize()
    assert conv.ahead_info()[1] == nb % 128
    return peak_err(t.cpu().numpy(), ref)


@pytest.mark.parametrize("method", ["upols", "upola"])
@pytest.mark.parametrize("B,P,C,nb", [(512, 40, 3, 75), (256, 10, 2, 70), (16, 7, 2, 40), (64, 1, 1, 37),
                                      (1024, 30, 2, 33), (128, 40, 2, 100), (32, 2, 1, 20)])
def test_level_steps_small_filters(neo_gpu, oracle, method, B, P, C, nb):
    """P below the far level: the block step alone (P <= 16) and the Toeplitz levels, every
    block size the block step is built for, P = 1, ring wraparound; OLS and OLA."""
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 320) <= TOL


@pytest.mark.parametrize("P,far", [(p, -1) for p in (3, 8, 9, 16, 17, 32, 33, 64, 65, 255, 256, 257, 448, 449, 450)] +
                         [(p, 1) for p in (257, 384, 385, 513)])
def test_level_band_edges(neo_gpu, oracle, P, far):
    """Every band edge of the level plan (the block's own partitions / 4 / 8 / 16 / 32-block
    Toeplitz levels / the 128-block level and its 192-partition LDS chunks / far segments, a
    last far segment of one partition): B = 32, past the ring length."""
    assert _stream(neo_gpu, oracle, "upols", 32, P, 2, max(2 * P + 140, 300), 400 + P, {"far_level": far}) <= TOL


@pytest.mark.parametrize("far", [0, 1])
@pytest.mark.parametrize("method", ["upols", "upola"])
@pytest.mark.parametrize("B,P,C,nb", [(256, 300, 2, 420), (32, 700, 1, 900), (64, 400, 2, 700), (16, 1000, 1, 1200),
                                      (1024, 270, 1, 300), (128, 600, 3, 800)])
def test_far_level_steps_vs_oracle(neo_gpu, oracle, method, B, P, C, nb, far):
    """Partitions >= 256, both forms: the 128-block Toeplitz level (far = 0) and the far
    level (far = 1: 256-point transforms along the partition axis), each computing its next
    window during the current one: several windows, ring wraparound, the packed DC / Nyquist
    bin, several sub-units per 16-column unit; OLS and OLA."""
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 520, {"far_level": far}) <= TOL


@pytest.mark.parametrize("method", ["upols", "upola"])
@pytest.mark.parametrize("K", [1, 2, 3, 4])
@pytest.mark.parametrize("B,P,C", [(32, 700, 1), (32, 1100, 1), (64, 1000, 2)])
def test_far_window_groups_vs_oracle(neo_gpu, oracle, method, K, B, P, C):
    """The far level's phase 1 over groups of K windows (neo_hip_upols_opts.far_group forces
    K; by default only shapes of >= 16384 16-column units, the headline and its 2- and 4-GPU shards, run
    K = 3 / 4): far1_mac<FPL, K> for every K, phase 2's segments 1 .. j of window j of a
    group, the classes' staggered start after priming, and the two kernel builds (pairs
    only for K <= 2, any group for K > 2). nseg = 4 / 7 / 6 (FPL 4 / 2 / 2), >= 2P + 300
    single-block steps (many windows, ring wraparound); OLS and OLA. Ring semantics:
    fdl_index.hpp:23-36."""
    nb = 2 * P + 320
    conv_opts = {"far_level": 1, "far_group": K}
    probe = neo_gpu.UpolsConvolver(C, B, P, options=conv_opts)
    assert probe.far_group() == K
    probe.close()
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 900 + K, conv_opts) <= TOL


@pytest.mark.parametrize("f2", [1, 2])
@pytest.mark.parametrize("method,B,P,C,K", [("upols", 32, 700, 1, 3), ("upola", 64, 1000, 2, 4), ("upols", 32, 1100, 1, 2),
                                            ("upols", 256, 300, 2, 0), ("upola", 1024, 270, 1, 0), ("upols", 16, 1000, 1, 1)])
def test_far_phase2_forms_vs_oracle(neo_gpu, oracle, f2, method, B, P, C, K):
    """One launch per step (step_group 1) with far phase 2 in one workgroup per unit (far_phase2
    = 1, far2c_role one step after phase 1; the default from 32768 16-column units) or in two
    steps (2: 2a beside phase 1, 2b one step later): window groups K = 1..4, several windows,
    ring wraparound, OLS and OLA, against the oracle (fdl_index.hpp:23-36)."""
    nb = 2 * P + 320
    opts = {"far_level": 1, "far_group": K, "step_group": 1, "far_phase2": f2}
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 1700 + P, opts) <= TOL


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("method,B,P,C,nb,opts", [
    ("upols", 512, 40, 3, 75, {}), ("upola", 128, 40, 2, 100, {}), ("upols", 16, 7, 2, 40, {}),
    ("upols", 32, 700, 1, 1720, {"far_group": 3, "far_level": 1}),
    ("upola", 64, 1000, 2, 2320, {"far_group": 4, "far_level": 1}),
    ("upols", 32, 1100, 1, 2520, {"far_group": 2, "far_level": 1}), ("upols", 256, 300, 2, 420, {"far_level": 0}),
    ("upola", 1024, 270, 1, 300, {}), ("upols", 32, 257, 2, 654, {"far_level": 1})])
def test_step_groups_vs_oracle(neo_gpu, oracle, G, method, B, P, C, nb, opts):
    """Step groups (neo_hip_upols_opts.step_group = G): the block of every call alone on the
    caller's stream, the level slices of G calls as one launch on the background stream (the
    levels of 4 G <= T <= 32 with their windows offset by T / 2, every window's parts and the far
    level's kFarT / G - 2 slices cut where part_plan evens out the groups); every band, the far
    window groups K = 2..4, the
    128-block Toeplitz level, several windows and ring wraparound; OLS and OLA
    (uniform_partitioned_convolver.hpp:47-65, fdl_index.hpp:23-36)."""
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 1300 + P, dict(opts, step_group=G)) <= TOL


@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("method,B,P,C", [("upols", 32, 700, 1), ("upola", 64, 1000, 2), ("upols", 16, 1000, 1),
                                          ("upols", 1024, 270, 1), ("upols", 256, 300, 2), ("upola", 32, 257, 2),
                                          ("upols", 128, 600, 3)])
def test_far_recomputed_vs_oracle(neo_gpu, oracle, G, method, B, P, C):
    """The recomputed far level (neo_hip_upols_opts.far_level = 2, far2r_role): every segment
    from the filter's and the FDL's rows each window, one launch per step (G = 1) and step
    groups; one and several segments, a last segment of one partition, the packed bin 0,
    B = 16..1024, several windows and ring wraparound, OLS and OLA, against the oracle (uniform_partitioned_convolver.hpp:47-65, fdl_index.hpp:23-36)."""
    nb = 2 * P + 320
    opts = {"far_level": 2, "step_group": G}
    probe = neo_gpu.UpolsConvolver(C, B, P, options=opts)
    assert probe.far_form() == 2 and probe.step_group() == G
    probe.close()
    assert _stream(neo_gpu, oracle, method, B, P, C, nb, 1900 + P + G, opts) <= TOL


@pytest.mark.parametrize("G", [1, 4])
def test_join_background(neo_gpu, oracle, G):
    """neo_hip_upols_join_background: after it, an event on the caller's stream completes only
    when every background slice launch issued so far has (step groups); a no-op with G = 1. The
    outputs are complete in stream order either way, and the handle steps on afterwards."""
    torch = pytest.importorskip("torch")
    B, P, C, nb = 64, 420, 2, 300
    ir = np.stack([oracle.noise(1600 + c, B * P) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    sig = np.stack([oracle.noise(1610 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts)
    conv = neo_gpu.UpolsConvolver(C, B, P, options={"step_group": G})
    assert conv.step_group() == G
    conv.filter(parts)
    conv.set_batch(False)
    s = torch.cuda.Stream()
    t = torch.from_numpy(sig).cuda()
    torch.cuda.synchronize()
    half = nb // 2
    conv.process_blocks_ptr(t.data_ptr(), t.data_ptr(), B * nb, half, s.cuda_stream)
    conv.join_background(s.cuda_stream)
    e = torch.cuda.Event()
    e.record(s)
    e.synchronize()
    conv.process_blocks_ptr(t.data_ptr() + 4 * B * half, t.data_ptr() + 4 * B * half, B * nb, nb - half,
                            s.cuda_stream)
    conv.join_background(s.cuda_stream)
    s.synchronize()
    assert peak_err(t.cpu().numpy(), ref) <= TOL
    conv.close()


@pytest.mark.parametrize("G", [2, 4, 8])
def test_step_groups_equal_one_launch(neo_gpu, oracle, G):
    """The same sums in the same order as the one-launch step. Not bit-identical: the step
    groups' far phase 2 (far2c_role) runs the fresh transform in the workgroup that uses it, and
    the compiler may contract its butterflies' multiply-adds differently there than in far2a_role;
    equal to a few float32 roundings (measured 0 with 2a / 2b split in both)."""
    torch = pytest.importorskip("torch")
    B, P, C, nb = 64, 1000, 2, 700
    ir = np.stack([oracle.noise(1400 + c, B * P) for c in range(C)])
    sig = torch.from_numpy(np.stack([oracle.noise(1410 + c, B * nb) for c in range(C)])).cuda()
    outs = []
    for g in (1, G):
        conv = neo_gpu.UpolsConvolver(C, B, P, options={"step_group": g})
        conv.set_impulse(ir)
        conv.set_batch(False)
        t = sig.clone()
        conv.process_blocks(t)
        torch.cuda.synchronize()
        outs.append(t.cpu().numpy())
        conv.close()
    assert peak_err(outs[1], outs[0]) <= 1e-6


def test_step_groups_mixed_paths(neo_gpu, oracle):
    """Step groups across batched passes, plain steps, host blocks, level toggles, a reset and
    a filter change (each joins the background stream before it touches the FDL ring or the
    level buffers), one block per call and many per call, against the oracle."""
    torch = pytest.importorskip("torch")
    B, P, C = 64, 420, 2
    L = B * P
    irs = [np.stack([oracle.noise(1500 + 7 * k + c, L) for c in range(C)]) for k in range(2)]
    parts = [oracle.uniform_partition(oracle.normalize_impulse(ir), B) for ir in irs]
    conv = neo_gpu.UpolsConvolver(C, B, P, options={"step_group": 4})
    for k in range(2):
        nb = 1100
        sig = np.stack([oracle.noise(1520 + 3 * k + c, B * nb) for c in range(C)])
        ref = oracle.dense_convolve(sig, parts[k])
        conv.filter(parts[k])
        t = torch.from_numpy(sig).cuda()
        pos = 0
        for kind, n in [("stream", 301), ("batch", 64), ("one", 7), ("off", 5), ("stream", 3), ("host", 2),
                        ("stream", 290), ("batch", 33), ("one", 6), ("stream", 389)]:
            seg = t[:, pos * B:(pos + n) * B].contiguous()
            if kind == "host":
                torch.cuda.synchronize()
                h = seg.cpu().numpy().copy()
                for i in range(n):
                    blk = np.ascontiguousarray(h[:, i * B:(i + 1) * B])
                    conv(blk)  # the host-buffer call (zero-copy block)
                    h[:, i * B:(i + 1) * B] = blk
                seg = torch.from_numpy(h).cuda()
            elif kind == "one":
                for i in range(n):
                    blk = seg[:, i * B:(i + 1) * B].contiguous()
                    conv(blk)
                    seg[:, i * B:(i + 1) * B] = blk
            else:
                conv.set_ahead(kind != "off")
                conv.set_batch(kind == "batch")
                conv.process_blocks(seg)
                conv.set_ahead(True)
            t[:, pos * B:(pos + n) * B] = seg
            pos += n
        assert pos == nb
        torch.cuda.synchronize()
        assert peak_err(t.cpu().numpy(), ref) <= TOL, k
    conv.reset()
    x = torch.zeros((C, B * 40), device="cuda")
    conv.set_batch(False)
    conv.process_blocks(x)
    torch.cuda.synchronize()
    assert torch.count_nonzero(x).item() == 0  # silence after a reset


def test_step_group_timing_detail(neo_gpu):
    """timing_detail() with step groups: part 0 the block launches (every timed step), part 1
    the slice launches on the background stream (one per G steps)."""
    torch = pytest.importorskip("torch")
    conv = neo_gpu.UpolsConvolver(4, 256, 300, options={"step_group": 4})
    conv.set_batch(False)
    x = torch.zeros((4, 256 * 16), device="cuda")
    conv.set_timing(True)
    conv.process_blocks(x)
    torch.cuda.synchronize()
    conv.set_timing(False)
    parts = conv.timing_detail()
    # 16 block launches; background launches at steps 0, 4, 8, 12 that carry work (an empty one
    # is not launched, nor timed): from the plan (part_plan: window offsets and part cuts; slice_part)
    pp = neo_gpu.convolution.part_plan(4, 256, 300, 4)
    lp = neo_gpu.convolution.level_plan(300)
    busy = 0
    for g in range(4):
        work = g >= 1 and lp["nseg"] > 0  # far phase 1 of slice g - 1 (and phase 2 from g = 2)
        for l, wins in pp["cuts"].items():
            T, phi = lp["T"][l], pp["phi"][l]
            m0 = 4 * g + phi
            j, Tg = (m0 % T) // 4, T // 4
            gw = (m0 // T * T - phi) // 4  # the window's first group
            c = wins[(gw % pp["cycle"]) // Tg]
            work = work or (j >= 1 and c[j] > c[j - 1])
        busy += work
    assert [n for _, n in parts] == [16, busy, 0, 0]
    assert parts[0][0] > 0 and parts[1][0] > 0
    assert conv.step_group() == 4
    with pytest.raises(RuntimeError):
        neo_gpu.UpolsConvolver(1, 64, 300, options={"step_group": 3})


def test_far_group_defaults(neo_gpu):
    """The automatic window group: 2 below 16384 16-column units (the 256-channel shapes),
    round(sqrt(2 (nseg - 1))) from there (bench.far_group restates it)."""
    import bench

    for C, B, P in [(4, 512, 938), (256, 512, 938), (512, 512, 938), (256, 256, 1875), (1, 512, 188), (3, 64, 300)]:
        c = neo_gpu.UpolsConvolver(C, B, P, options={"far_level": 1})  # the stored form
        nseg = neo_gpu.convolution.level_plan(P)["nseg"]
        assert c.far_group() == (bench.far_group(nseg, C * B // 16) if nseg else 0), (C, B, P)
        c.close()
        # the automatic form: stored spectra; recomputed (one window per pass) on request
        c = neo_gpu.UpolsConvolver(C, B, P)
        assert c.far_form() == (1 if nseg else 0), (C, B, P)
        assert c.far_group() == (bench.far_group(nseg, C * B // 16) if nseg else 0), (C, B, P)
        c.close()
        if nseg:
            c = neo_gpu.UpolsConvolver(C, B, P, options={"far_level": 2})
            assert c.far_form() == 2 and c.far_group() == 1, (C, B, P)
            c.close()
    with pytest.raises(RuntimeError):
        neo_gpu.UpolsConvolver(1, 64, 300, options={"far_group": 5})


@pytest.mark.parametrize("far", [0, 1])
def test_far_field_mixed_and_refilter(neo_gpu, oracle, far):
    """Streaming levels across batched passes, toggles at arbitrary blocks and a filter
    change: the levels re-prime at the next streaming step."""
    torch = pytest.importorskip("torch")
    B, P, C = 256, 290, 2
    L = B * P
    irs = [np.stack([oracle.noise(540 + 7 * k + c, L) for c in range(C)]) for k in range(2)]
    parts = [oracle.uniform_partition(oracle.normalize_impulse(ir), B) for ir in irs]
    conv = neo_gpu.UpolsConvolver(C, B, P, options={"far_level": far})
    for k in range(2):
        nb = 480
        sig = np.stack([oracle.noise(560 + 3 * k + c, B * nb) for c in range(C)])
        ref = oracle.dense_convolve(sig, parts[k])
        conv.filter(parts[k])
        out = np.empty_like(sig)
        pos = 0
        for ahead, batch, n in [(True, False, 150), (False, True, 64), (True, False, 37), (True, True, 32),
                                (True, False, 197)]:
            conv.set_batch(batch)
            conv.set_ahead(ahead)
            seg = torch.from_numpy(np.ascontiguousarray(sig[:, pos * B:(pos + n) * B])).cuda()
            conv.process_blocks(seg)
            torch.cuda.synchronize()
            out[:, pos * B:(pos + n) * B] = seg.cpu().numpy()
            pos += n
        assert pos == nb
        assert peak_err(out, ref) <= TOL, k


def test_batched_calls_keep_levels_primed(neo_gpu, oracle):
    """process_blocks with batching on and a block count that is not a whole number of
    batches: only whole T-block batches run (they leave the levels to re-prime once), and
    once the levels are primed a call of fewer than 4 T blocks streams them all, so repeated
    33-block calls do not re-prime every call (ahead_info's window position keeps counting).
    filter() primes the levels itself (lvl_setup_prime), so the first call streams too; after a
    reset and one batched call of 128 blocks the next 33-block call runs one batch and primes."""
    torch = pytest.importorskip("torch")
    B, P, C = 64, 300, 2
    L = B * P
    ir = np.stack([oracle.noise(960 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    nb = 33 * 6
    sig = np.stack([oracle.noise(970 + c, B * nb) for c in range(C)])
    ref = oracle.dense_convolve(sig, parts)
    conv = neo_gpu.UpolsConvolver(C, B, P)
    conv.filter(parts)
    assert conv.ahead_info()[0] and conv.batch_info()[0] == 32
    t = torch.from_numpy(sig).cuda()
    phases = []
    for k in range(6):
        seg = t[:, k * 33 * B:(k + 1) * 33 * B].contiguous()
        conv.process_blocks(seg)
        t[:, k * 33 * B:(k + 1) * 33 * B] = seg
        phases.append(conv.ahead_info()[1])
    torch.cuda.synchronize()
    # primed by filter(): 33 streamed blocks per call from the first
    assert phases == [(33 * (k + 1)) % 128 for k in range(6)], phases
    assert peak_err(t.cpu().numpy(), ref) <= TOL
    conv.reset()
    t = torch.from_numpy(sig).cuda()
    conv.process_blocks(t[:, : 128 * B].contiguous())  # 4 T blocks: batched passes, the levels re-prime later
    phases = []
    for k in range(2):
        seg = t[:, 128 * B + k * 33 * B:128 * B + (k + 1) * 33 * B].contiguous()
        conv.process_blocks(seg)
        phases.append(conv.ahead_info()[1])
    # call 0: one batch of 32, one streamed block (primes); then 33 streamed blocks
    assert phases == [1, 34], phases


@pytest.mark.parametrize("far", [0, 1])
def test_levels_before_any_filter(neo_gpu, far):
    """Streaming steps on a fresh handle with a far level (or the 128-block level) and no
    filter set (H is zero): silence, no fault (the level buffers are allocated and primed on
    the first step)."""
    torch = pytest.importorskip("torch")
    conv = neo_gpu.UpolsConvolver(2, 128, 600, options={"far_level": far})
    conv.set_batch(False)
    assert conv.ahead_info()[0]
    x = torch.rand((2, 128 * 140), device="cuda")
    conv.process_blocks(x)
    torch.cuda.synchronize()
    assert torch.count_nonzero(x).item() == 0


def test_level_timing_detail(neo_gpu):
    """timing_detail(): one step kernel per timed step (part 0)."""
    torch = pytest.importorskip("torch")
    conv = neo_gpu.UpolsConvolver(4, 256, 300)
    conv.set_batch(False)
    x = torch.zeros((4, 256 * 12), device="cuda")
    conv.set_timing(True, every=3)
    conv.process_blocks(x)
    conv.set_timing(False)
    parts = conv.timing_detail()
    assert [n for _, n in parts] == [4, 0, 0, 0]  # steps 0, 3, 6, 9
    assert parts[0][0] > 0


def test_ahead_mixed_paths(neo_gpu, oracle):
    """Lookahead steps, batched passes, plain steps and host blocks share one state; the
    lookahead can be switched at any block boundary."""
    torch = pytest.importorskip("torch")
    B, L, C = 256, 9000, 3
    ir = np.stack([oracle.noise(340 + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    for method in ("upols", "upola"):
        sig = np.stack([oracle.noise(350 + c, B * 150) for c in range(C)])
        ref = oracle.dense_convolve(sig, parts, method=method)
        conv = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method)
        conv.filter(parts)
        conv.set_ahead(True)
        t = torch.from_numpy(sig).cuda()
        pos = 0
        for kind, n in [("one", 5), ("batch", 40), ("host", 3), ("off", 4), ("on", 0), ("one", 33), ("batch", 64),
                        ("one", 1)]:
            if kind == "on":
                conv.set_ahead(True)
                continue
            seg = t[:, pos * B:(pos + n) * B].contiguous()
            if kind == "off":
                conv.set_ahead(False)
                conv.set_batch(False)
                conv.process_blocks(seg)
                conv.set_batch(True)
            elif kind == "batch":
                conv.process_blocks(seg)  # lookahead steps up to the window end, then batches
            elif kind == "one":
                for i in range(n):
                    blk = seg[:, i * B:(i + 1) * B].contiguous()
                    conv(blk)
                    seg[:, i * B:(i + 1) * B] = blk
            else:
                torch.cuda.synchronize()
                h = seg.cpu().numpy().copy()
                conv.process(h)
                seg = torch.from_numpy(h).cuda()
            t[:, pos * B:(pos + n) * B] = seg
            pos += n
        torch.cuda.synchronize()
        assert peak_err(t[:, :pos * B].cpu().numpy(), ref[:, :pos * B]) <= TOL, method


def test_ahead_defaults_and_errors(neo_gpu):
    big = neo_gpu.UpolsConvolver(64, 512, 300)  # filter + FDL 157 MB: HBM-bound step
    assert big.ahead_info()[0]
    assert neo_gpu.UpolsConvolver(1, 512, 188).ahead_info()[0]  # C3
    small = neo_gpu.UpolsConvolver(1, 128, 20)  # P < 64: the plain step
    assert not small.ahead_info()[0]
    huge = neo_gpu.UpolsConvolver(1, 2048, 100)  # the block step is built for B <= 1024
    assert not huge.ahead_info()[0]
    with pytest.raises(RuntimeError):
        huge.set_ahead(True)
    with pytest.raises(ValueError):
        neo_gpu.UpolsConvolver(1, 128, 20, options={"nope": 1})
    with pytest.raises(RuntimeError):
        neo_gpu.UpolsConvolver(1, 128, 20, options={"batch_blocks": 3})
    v2 = neo_gpu.UpolsConvolver(2, 128, 4, method="upola_v2")
    assert not v2.ahead_info()[0]
    with pytest.raises(RuntimeError):
        v2.set_ahead(True)
    v2.set_ahead(False)


@pytest.mark.parametrize("devices,C,method", [([0, 0], 6, "upols"), ([0, 0, 0], 7, "upols"), ([0, 0], 5, "upola")])
def test_multi_device_shards(neo_gpu, oracle, devices, C, method):
    """neo_hip_upols_multi_*: C channels sharded over a device list (here the box's one
    device, repeated: shards of 3 / 2-2-3 / 2-3 channels on their own handles and streams).
    Bit for bit the unsharded handle on the same calls (set_impulse normalization over all
    channels, 90 blocks in one call, a reset, 5 more), and within tolerance of the oracle."""
    B, L, nb = 128, 128 * 70, 90
    P = neo_gpu.num_partitions(L, B)
    ir = np.stack([oracle.noise(500 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(600 + c, B * nb) for c in range(C)])
    multi = neo_gpu.UpolsMultiConvolver(C, B, P, devices, method=method)
    assert [s[1:] for s in multi.shards()] == [(C * i // len(devices), C * (i + 1) // len(devices) - C * i // len(devices))
                                               for i in range(len(devices))]
    one = neo_gpu.UpolsConvolver(C, B, P, method=method)
    multi.set_impulse(ir, normalize=True)
    one.set_impulse(ir, normalize=True)
    got = multi.process(sig)
    ref = one.process(sig.copy())
    assert np.array_equal(got, ref)
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    assert peak_err(got, oracle.dense_convolve(sig, parts, method=method)) < TOL
    multi.reset()
    one.reset()
    tail = sig[:, :5 * B].copy()
    assert np.array_equal(multi.process(tail), one.process(tail.copy()))


def test_multi_device_errors(neo_gpu):
    with pytest.raises(neo_gpu._native.NeoHipError):
        neo_gpu.UpolsMultiConvolver(2, 128, 10, [0, 0, 0])  # more shards than channels
    with pytest.raises(neo_gpu._native.NeoHipError):
        neo_gpu.UpolsMultiConvolver(4, 128, 10, [0, 1 << 20])  # no such device
