"""Offline windows (neo_hip_upols_set_offline; upols_levels.hip k_off_mac, upols_batch.hip
launch_offline): with every block of a call known up front -- the reference's offline harness,
extra/plugin/src/dsp/DenseConvolution.hpp:39-70 run by extra/plugin/src/ui/BenchmarkTab.hpp:47-66 --
each 128-block window of a bin is a convolution along the block axis,
Y[t] = sum_p H[p] X[t - p] (uniform_partitioned_convolver.hpp:47-65, fdl_index.hpp:23-36), computed
per 128-partition segment by 256-point transforms along that axis (the far level's decomposition,
from partition 0). Outputs against the oracle's dense_convolve: every block size, segment counts
1..8 with a partial last segment, one and two windows per pass, the T-block passes and streaming
steps for the rest of a call and between calls, ring wraparound, OLS and OLA."""
import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _case(oracle, C, B, P, nb, seed, method="upols"):
    L = B * (P - 1) + B // 3 + 1
    ir = np.stack([oracle.noise(seed + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    assert parts.shape[1] == P
    sig = np.stack([oracle.noise(seed + 50 + c, B * nb) for c in range(C)])
    return parts, sig, oracle.dense_convolve(sig, parts, method=method)


@pytest.mark.parametrize("method", ["upols", "upola"])
@pytest.mark.parametrize("C,B,P,nb", [(2, 64, 128, 300), (1, 16, 129, 420), (2, 256, 300, 700), (1, 32, 700, 1300),
                                      (3, 128, 938, 600), (1, 1024, 200, 300), (2, 512, 938, 400), (1, 512, 1000, 300)])
def test_offline_windows_vs_oracle(neo_gpu, oracle, method, C, B, P, nb):
    """One call over nb blocks: passes of two windows, then one, then T-block passes and single
    blocks for the rest; several calls wrap the ring (128 (nseg + 2) rows)."""
    torch = pytest.importorskip("torch")
    parts, sig, ref = _case(oracle, C, B, P, nb, 4000 + P + B, method)
    conv = neo_gpu.UpolsConvolver(C, B, P, method=method)
    assert conv.offline_info() == (True, -(-P // 128))
    conv.filter(parts)
    t = torch.from_numpy(sig).cuda()
    conv.set_timing(True)
    conv.process_blocks(t)
    torch.cuda.synchronize()
    conv.set_timing(False)
    assert peak_err(t.cpu().numpy(), ref) <= TOL


@pytest.mark.parametrize("B,P", [(64, 300), (256, 938)])
def test_offline_mixed_with_streaming_and_refilter(neo_gpu, oracle, B, P):
    """Offline passes, streaming blocks (the levels re-prime after a pass), T-block passes and a
    filter change, in one handle, against the oracle; and the same with offline windows off."""
    torch = pytest.importorskip("torch")
    C = 2
    for off in (True, False):
        conv = neo_gpu.UpolsConvolver(C, B, P)
        conv.set_offline(off)
        for k in range(2):
            parts, sig, ref = _case(oracle, C, B, P, 700, 4100 + 13 * k + P)
            conv.filter(parts)
            out = np.empty_like(sig)
            pos = 0
            for batch, n in [(True, 256), (False, 37), (True, 160), (False, 5), (True, 128), (True, 40), (False, 74)]:
                conv.set_batch(batch)
                seg = torch.from_numpy(np.ascontiguousarray(sig[:, pos * B:(pos + n) * B])).cuda()
                conv.process_blocks(seg)
                torch.cuda.synchronize()
                out[:, pos * B:(pos + n) * B] = seg.cpu().numpy()
                pos += n
            assert pos == 700
            assert peak_err(out, ref) <= TOL, (off, k)
        conv.close()


def test_offline_small_filters_and_errors(neo_gpu, oracle):
    """Below 128 partitions (and for upola_v2) offline windows are off and cannot be switched on;
    the batched passes run as before."""
    torch = pytest.importorskip("torch")
    conv = neo_gpu.UpolsConvolver(2, 64, 100)
    assert conv.offline_info() == (False, 1)
    with pytest.raises(RuntimeError):
        conv.set_offline(True)
    v2 = neo_gpu.UpolsConvolver(1, 64, 300, method="upola_v2")
    assert not v2.offline_info()[0]
    with pytest.raises(RuntimeError):
        v2.set_offline(True)
    parts, sig, ref = _case(oracle, 2, 64, 100, 300, 4200)
    conv.filter(parts)
    t = torch.from_numpy(sig).cuda()
    conv.process_blocks(t)
    torch.cuda.synchronize()
    assert peak_err(t.cpu().numpy(), ref) <= TOL


def test_dense_convolve_offline(neo_gpu, oracle):
    """neo.dense_convolve (DenseConvolution.hpp:39-70) over 600 blocks at a 10 s-class filter shape:
    whole 256-block chunks go through the offline windows."""
    C, B, P = 2, 512, 400
    L = B * P
    ir = np.stack([oracle.noise(4300 + c, L) for c in range(C)])
    sig = np.stack([oracle.noise(4310 + c, B * 600 - 77) for c in range(C)])
    ref = oracle.dense_convolve(sig, oracle.uniform_partition(oracle.normalize_impulse(ir), B))
    assert peak_err(neo_gpu.dense_convolve(sig, ir, B), ref) <= TOL
