"""Groups of single-channel convolvers (neo_hip_upols_group_*, upols_group.hip): the plugin's
std::vector<upols_convolver> called channel by channel per frame
(extra/plugin/src/dsp/DenseConvolution.hpp:35, DenseConvolution.cpp:62-74). Every member's
outputs must equal its own sequential convolver's bit for bit (the group forces the shared
handle's code-path choices on every handle), whatever the call pattern; in the plugin's
pattern a frame is one launch."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setup(neo_gpu, oracle, C, B, L, seed, method="upols"):
    ir = np.stack([oracle.noise(seed + c, L) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    g = neo_gpu.UpolsGroup(B, parts.shape[1], method=method)
    ids = [g.join() for _ in range(C)]
    for i, c in zip(ids, range(C)):
        g.filter(i, parts[c])
    ref = neo_gpu.UpolsConvolver(C, B, parts.shape[1], method=method)
    ref.filter(parts)
    return g, ids, parts, ref


@pytest.mark.parametrize("method", ["upols", "upola"])
def test_group_frames_equal_multichannel(neo_gpu, oracle, method):
    """16 members, the plugin's pattern (per frame: the channel buffers filled, then one call per
    member in order): frames 0-2 run member by member (the group sees each member's buffer
    reused twice), then every frame is one launch; the
    outputs equal one 16-channel handle over the same blocks bit for bit. A member whose buffer
    changes after the frame's first call (a caller filling channels inside the loop) re-runs its
    own block step and still matches."""
    C, B, L, nf = 16, 128, 128 * 300, 40
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 1100, method)
    bufs = [np.zeros(B, np.float32) for _ in range(C)]
    x = np.stack([oracle.noise(1200 + c, B * nf) for c in range(C)])
    for f in range(nf):
        blk = np.ascontiguousarray(x[:, f * B:(f + 1) * B])
        expect = ref(blk.copy())
        late = f == 20  # frame 20: members 5 and 9 get their blocks only right before their calls
        for c in range(C):
            if not (late and c in (5, 9)):
                bufs[c][:] = blk[c]
            else:
                bufs[c][:] = 0.0
        for c in range(C):
            if late and c in (5, 9):
                bufs[c][:] = blk[c]
            g(ids[c], bufs[c])
        got = np.stack(bufs)
        assert np.array_equal(got, expect), f
    st = g.stats()
    assert st["coalesced"] and st["frame_steps"] == nf - 3 and st["redos"] == 2 and st["switches"] == 1, st


def test_group_pattern_breaks_split(neo_gpu, oracle):
    """A member called twice within a frame, a filter change and a shared scratch buffer (the
    harness dense_convolve<Convolver> pattern, DenseConvolution.hpp:56-67): the group leaves
    the one-launch mode, moves every state back into a handle per member (a member stepped
    ahead of its call one block back) and each member still equals its own convolver."""
    C, B, L = 6, 128, 128 * 150
    g, ids, parts, _ = _setup(neo_gpu, oracle, C, B, L, 1300)
    P = parts.shape[1]
    singles = []
    for c in range(C):
        s = neo_gpu.UpolsConvolver(1, B, P, options={"far_group": g_far(neo_gpu, C, B, P),
                                                      "toep_split": g_split(C, B)})
        s.filter(parts[c][None])
        singles.append(s)
    bufs = [np.zeros(B, np.float32) for _ in range(C)]
    rng = np.random.default_rng(5)

    def call(c, blk):
        bufs[c][:] = blk
        g(ids[c], bufs[c])
        e = blk[None].copy()
        singles[c](e)
        assert np.array_equal(bufs[c], e[0]), c

    for f in range(5):  # coalesces after frame 2
        for c in range(C):
            bufs[c][:] = rng.random(B, dtype=np.float32) - 0.5
        for c in range(C):
            call(c, bufs[c].copy())
    assert g.stats()["coalesced"]
    # member 3 twice before the others: split, member 3 one block ahead of the rest
    call(0, rng.random(B, dtype=np.float32))
    call(3, rng.random(B, dtype=np.float32))
    call(3, rng.random(B, dtype=np.float32))
    assert not g.stats()["coalesced"]
    for c in (1, 2, 4, 5):
        call(c, rng.random(B, dtype=np.float32))
    # a shared scratch buffer for every member: never coalesces, still exact
    scratch = np.zeros(B, np.float32)
    for f in range(4):
        for c in range(C):
            blk = rng.random(B, dtype=np.float32)
            scratch[:] = blk
            g(ids[c], scratch)
            e = blk[None].copy()
            singles[c](e)
            assert np.array_equal(scratch, e[0])
    assert not g.stats()["coalesced"]
    # a new filter for member 2 resets it (uniform_partitioned_convolver::filter)
    newp = oracle.uniform_partition(oracle.normalize_impulse(oracle.noise(1400, L)[None]), B)[0]
    g.filter(ids[2], newp)
    singles[2].filter(newp[None])
    for f in range(4):
        for c in range(C):
            call(c, rng.random(B, dtype=np.float32))


def g_far(neo_gpu, C, B, P):
    c = neo_gpu.UpolsConvolver(C, B, P)
    k = c.far_group()
    c.close()
    return k


def g_split(C, B):
    return 2 if C * (B // 16) < 256 else 1
