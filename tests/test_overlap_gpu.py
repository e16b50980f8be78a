"""GPU parity of the standalone overlap stages (neo_hip_overlap_*, overlap_save.hpp:19-112 and
overlap_add.hpp:23-107 for any filter size F) against the oracle's restatement
(oracle_overlap_stage) and the reference's own identity test (overlap_test.cpp:21-64)."""
import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
F_SIZES = [8, 9, 10, 17, 127, 128, 129, 130, 512, 999, 1024]


@pytest.mark.parametrize("kind", ["save", "add"])
@pytest.mark.parametrize("B", [128, 512])
@pytest.mark.parametrize("F", F_SIZES)
def test_overlap_identity(neo_gpu, oracle, kind, B, F):
    """overlap_test.cpp:21-64: block_size / filter_size kept, transform_size >= B + F - 1, the
    callback sees transform_size / 2 + 1 bins, a no-op callback gives output == input (per
    sample abs 1e-5 and RMSE 1e-5)."""
    stage = neo_gpu.overlap_save(B, F) if kind == "save" else neo_gpu.overlap_add(B, F)
    assert stage.block_size() == B and stage.filter_size() == F
    n = stage.transform_size()
    assert n == oracle.overlap_transform_size(B, F) and n >= B + F - 1
    sig = oracle.noise(F, B * 8)
    out = sig.copy()
    seen = []
    for i in range(0, out.size, B):
        blk = out[i:i + B]  # a view: processed in place
        stage(blk, lambda io: seen.append(io.shape[0]))
    assert seen == [n // 2 + 1] * 8
    assert np.abs(out - sig).max() <= 1e-5
    assert np.sqrt(np.mean((out - sig) ** 2)) <= 1e-5


@pytest.mark.parametrize("kind", ["save", "add"])
@pytest.mark.parametrize("B,F", [(128, 8), (128, 129), (64, 999), (512, 512), (16, 1)])
def test_overlap_filter_callback_vs_oracle(neo_gpu, oracle, kind, B, F):
    """A callback multiplying the bins by the spectrum of an F-tap filter, 12 blocks: the GPU
    stage against the restatement with the same callback (peak-normalized 1e-5); for
    overlap_save that is the linear convolution (n >= B + F - 1)."""
    n = oracle.overlap_transform_size(B, F)
    h = oracle.noise(300 + F, F)
    G = np.fft.rfft(np.concatenate([h, np.zeros(n - F, np.float32)]).astype(np.float64)).astype(np.complex64)
    x = oracle.noise(400 + B, B * 12)
    ref = oracle.overlap_stage(kind, x, B, F, G)
    stage = neo_gpu.overlap_save(B, F) if kind == "save" else neo_gpu.overlap_add(B, F)
    out = x.copy()

    def mul(io):
        io *= G  # complex64 product in place, as the restatement's callback

    for i in range(0, out.size, B):
        stage(out[i:i + B], mul)
    assert peak_err(out, ref) <= 1e-5
    if kind == "save":
        lin = np.convolve(x.astype(np.float64), h.astype(np.float64))[: x.size]
        assert peak_err(out, lin) <= 1e-5


@pytest.mark.parametrize("kind", ["save", "add"])
def test_overlap_stage_device_multichannel(neo_gpu, oracle, kind):
    """OverlapStage over 5 channels with CUDA tensors (asynchronous device path, ld > B) equals
    the host path channel by channel; reset() restarts the window."""
    torch = pytest.importorskip("torch")
    C, B, F, nb = 5, 256, 300, 6
    n = oracle.overlap_transform_size(B, F)
    G = (oracle.noise(77, 2 * (n // 2 + 1)).view(np.complex64)).copy()
    x = np.stack([oracle.noise(500 + c, B * nb) for c in range(C)])
    host = neo_gpu.OverlapStage(kind, C, B, F)
    dev = neo_gpu.OverlapStage(kind, C, B, F)
    ref = x.copy()
    for t in range(nb):
        blk = np.ascontiguousarray(ref[:, t * B:(t + 1) * B])
        spec = host.forward(blk)
        spec *= G
        host.inverse(spec, blk)
        ref[:, t * B:(t + 1) * B] = blk
    xt = torch.from_numpy(x).cuda()
    for t in range(nb):
        view = xt[:, t * B:]  # channel c at c * ld, ld = B * nb
        spec = dev.forward(view)
        torch.cuda.synchronize()
        sh = spec.cpu().numpy()
        sh *= G  # the same callback arithmetic as the host path (numpy complex64)
        spec.copy_(torch.from_numpy(sh))
        dev.inverse(spec, view)
    torch.cuda.synchronize()
    assert np.array_equal(xt.cpu().numpy(), ref)
    for c in range(C):  # each channel against the one-channel restatement
        assert peak_err(ref[c], oracle.overlap_stage(kind, x[c], B, F, G)) <= 1e-5
    dev.reset()
    spec = dev.forward(torch.from_numpy(np.ascontiguousarray(x[:, :B])).cuda())
    torch.cuda.synchronize()
    spec0 = host.__class__(kind, C, B, F).forward(np.ascontiguousarray(x[:, :B]))
    assert np.array_equal(spec.cpu().numpy(), spec0)


def test_overlap_errors(neo_gpu):
    with pytest.raises(neo_gpu._native.NeoHipError):
        neo_gpu.OverlapStage("save", 1, 100, 8)  # block not a power of two
    with pytest.raises(neo_gpu._native.NeoHipError):
        neo_gpu.OverlapStage("add", 0, 128, 8)
    with pytest.raises(ValueError):
        neo_gpu.OverlapStage("both", 1, 128, 8)
    with pytest.raises(neo_gpu._native.NeoHipError):
        neo_gpu.OverlapStage("save", 1, 1 << 27, 2)  # n = 2^28 > 2^max_order
