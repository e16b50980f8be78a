"""Paced background work (neo_hip_upols_set_paced): a step group's background launch issued as G
per-call pieces, or as two pieces per group (workgroup ranges of the same launch), with the block
of each call that issues a piece waiting for the piece before it. The same kernels compute the same sums, so the outputs equal the unpaced
step groups' bit for bit (until a switch re-primes the levels: the far level's windows then start
elsewhere, float summation order); pinned to the oracle (uniform_partitioned_convolver.hpp:47-65)
throughout. The shape has step groups (128 channels x B = 512: 4096 16-column units, G = 4) and a
far level (P = 600), 700 blocks (five far windows), switched off and on again mid-stream."""
import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [1, 2])
def test_paced_equals_step_groups(neo_gpu, oracle, mode):
    """mode 1: a piece per call; mode 2: two pieces per group (calls 0 and G / 2)"""
    torch = pytest.importorskip("torch")
    C, B, P, nb = 128, 512, 600, 700
    ir = np.stack([oracle.noise(6100 + c, B * P) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    convs = []
    for _ in range(2):
        c = neo_gpu.UpolsConvolver(C, B, P)
        c.filter(parts)
        c.set_batch(False)
        assert c.step_group() == 4
        convs.append(c)
    paced, plain = convs
    paced.set_paced(mode)
    x = torch.from_numpy(np.stack([oracle.noise(6300 + c, B * nb) for c in range(C)])).cuda()
    outs = []
    for conv in convs:
        t = x.clone()
        torch.cuda.synchronize()
        for i in range(nb):
            if conv is paced and i in (300, 333):  # off, then on again: the levels re-prime each time
                conv.set_paced(mode if i == 333 else 0)
            p = t.data_ptr() + 4 * i * B
            conv.process_blocks_ptr(p, p, nb * B, 1, 0)
        conv.join_background(None)
        torch.cuda.synchronize()
        outs.append(t.cpu().numpy())
    assert np.array_equal(outs[0][:, :300 * B], outs[1][:, :300 * B])
    assert peak_err(outs[0], outs[1]) <= 1e-6
    chans = [0, 77, 127]
    ref = oracle.dense_convolve(x.cpu().numpy()[chans], parts[chans])
    assert peak_err(outs[0][chans], ref) <= 1e-5
