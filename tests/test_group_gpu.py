"""Groups of single-channel convolvers (neo_hip_upols_group_*, upols_group.hip): the plugin's
std::vector<upols_convolver> called channel by channel per frame
(extra/plugin/src/dsp/DenseConvolution.hpp:35, DenseConvolution.cpp:62-74). Every member's
outputs must equal its own sequential convolver's (a member alone runs a one-channel handle
with that shape's code paths, the shared handle its channel count's): bit for bit while only
the levels whose summation order is the same in both contribute, and within the oracle's bar
over long runs (a mode switch re-primes the levels, so the far windows may be aligned
elsewhere); in the plugin's pattern, with the members' buffers registered by their owner, a
frame is one launch. The group never reads a buffer that is not registered."""
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
    for b in bufs:
        g.register(b)
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
    for b in bufs:
        g.register(b)
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


def test_group_unregistered_buffers_never_read(neo_gpu, oracle):
    """The plugin's pattern on buffers the owner did NOT register: the group never coalesces
    (it would have to read them at the next frame's first call). Registered, it coalesces; the
    owner then frees the buffers and allocates new ones (a prepare() with another block size
    would): after unregister the group stops reading the old ones at once (the next frame's
    leader splits), re-coalesces on the new registered buffers, and every output stays its
    own convolver's."""
    C, B, L = 8, 128, 128 * 100
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 1500)
    rng = np.random.default_rng(9)

    def frame(bufs):
        blk = (rng.random((C, B), dtype=np.float32) - 0.5)
        expect = ref(blk.copy())
        for c in range(C):
            bufs[c][:] = blk[c]
        for c in range(C):
            g(ids[c], bufs[c])
        assert np.array_equal(np.stack(bufs), expect)

    bufs = [np.zeros(B, np.float32) for _ in range(C)]
    for _ in range(6):
        frame(bufs)
    assert not g.stats()["coalesced"] and g.stats()["frame_steps"] == 0
    for b in bufs:
        g.register(b)
    for _ in range(4):
        frame(bufs)
    assert g.stats()["coalesced"]
    n0 = g.stats()["frame_steps"]
    g.unregister(None)
    del bufs  # freed (no reference left on our side either)
    bufs = [np.full(B, np.nan, np.float32) for _ in range(C)]  # new allocations
    for b in bufs:
        g.register(b)
    frame(bufs)  # leader: neighbours' last buffers unregistered -> split, independent
    st = g.stats()
    assert not st["coalesced"] and st["frame_steps"] == n0
    for _ in range(4):
        frame(bufs)
    assert g.stats()["coalesced"]


def test_group_step_groups_late_blocks_and_split(neo_gpu, oracle):
    """A shape with step groups (64 members x B = 512: 2048 16-column units, G = 4, the block
    of a redo runs k_lvl_block): members whose blocks change after the frame's first call
    (redos) and a member called twice (split mid-frame, one member stepped back a block),
    against independent one-channel convolvers (to float rounding: the shared handle's step
    groups sum in another order)."""
    C, B, L = 64, 512, 512 * 100
    g, ids, parts, _ = _setup(neo_gpu, oracle, C, B, L, 1600)
    P = parts.shape[1]
    probe = neo_gpu.UpolsConvolver(C, B, P)
    assert probe.step_group() == 4
    probe.close()
    singles = []
    for c in range(C):
        s = neo_gpu.UpolsConvolver(1, B, P)
        s.filter(parts[c][None])
        singles.append(s)
    bufs = [np.zeros(B, np.float32) for _ in range(C)]
    for b in bufs:
        g.register(b)
    rng = np.random.default_rng(11)
    for f in range(14):
        blk = rng.random((C, B), dtype=np.float32) - 0.5
        late = {3, 40} if f in (6, 9) else set()
        for c in range(C):
            bufs[c][:] = 0.0 if c in late else blk[c]
        order = list(range(C))
        if f == 11:  # member 7 twice before the others: the group splits mid-frame
            order = [0, 7, 7] + [c for c in range(1, C) if c != 7]
        seen = set()
        for c in order:
            if c in late:
                bufs[c][:] = blk[c]
            if c in seen:  # the second call of a member: a new block
                bufs[c][:] = rng.random(B, dtype=np.float32) - 0.5
            e = bufs[c][None].copy()
            g(ids[c], bufs[c])
            singles[c](e)
            assert np.allclose(bufs[c], e[0], rtol=0, atol=1e-5 * max(1e-3, float(np.abs(e).max()))), (f, c)
            seen.add(c)
        if f == 8:
            st = g.stats()
            assert st["coalesced"] and st["redos"] >= 2, st
    assert g.stats()["switches"] >= 2


def test_group_long_run_vs_oracle(neo_gpu, oracle):
    """Far level contributing (P = 600 > 256 partitions) over 700 frames with mode switches (new
    filters for every member at frame 350: the group splits, then re-coalesces with its levels
    re-primed at another block): every member's output against the oracle's dense_convolve of its
    own input, each run from its filter on (a filter restarts the state,
    uniform_partitioned_convolver::filter)."""
    C, B, P, nf = 4, 128, 600, 700
    L = B * P
    g, ids, parts, _ = _setup(neo_gpu, oracle, C, B, L, 1700)
    bufs = [np.zeros(B, np.float32) for _ in range(C)]
    for b in bufs:
        g.register(b)
    x = np.stack([oracle.noise(1800 + c, B * nf) for c in range(C)])
    y = np.zeros_like(x)
    for f in range(nf):
        if f == 350:
            for c in range(C):
                g.filter(ids[c], parts[c])  # every member restarts
        for c in range(C):
            bufs[c][:] = x[c, f * B:(f + 1) * B]
        for c in range(C):
            g(ids[c], bufs[c])
            y[c, f * B:(f + 1) * B] = bufs[c]
    assert g.stats()["switches"] >= 3
    for lo, hi in ((0, 350), (350, nf)):
        ref = oracle.dense_convolve(np.ascontiguousarray(x[:, lo * B:hi * B]), parts)
        got = y[:, lo * B:hi * B]
        err = np.abs(got - ref).max() / np.abs(ref).max()
        assert err <= 1e-5, (lo, err)



def test_group_large_frame_in_place(neo_gpu, oracle):
    """A frame of >= 1 MiB read in place (one registered [C][B] buffer, the plugin's AudioBuffer):
    520 members, B = 512, P = 100 (streaming levels, step groups): every frame against one
    520-channel handle over the same blocks (to float rounding: the group re-primes its levels
    when it coalesces); members whose block changes after the frame's first call (spread over the
    frame) run their block step again."""
    C, B, L, nf = 520, 512, 512 * 100, 14
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 1800)
    frame = np.zeros((C, B), np.float32)
    g.register(frame)
    x = np.stack([oracle.noise(1900 + c, B * nf) for c in range(C)])
    late = (5, 140, 300, 519)
    for f in range(nf):
        blk = np.ascontiguousarray(x[:, f * B:(f + 1) * B])
        expect = ref(blk.copy())
        frame[:] = blk
        if f >= 8:  # coalesced by now: these members' blocks change after the leader's call
            frame[list(late)] = 0.0
        for c in range(C):
            if f >= 8 and c in late:
                frame[c] = blk[c]
            g(ids[c], frame[c])
        err = np.abs(frame - expect).max(axis=1) / np.maximum(np.abs(expect).max(axis=1), 1e-3)
        assert err.max() <= 1e-5, (f, int(err.argmax()), float(err.max()))
    st = g.stats()
    assert st["coalesced"] and st["frame_steps"] == nf - 3 and st["redos"] == len(late) * (nf - 8), st


@pytest.mark.parametrize("C", [16, 520])
def test_group_frame_stable_in_place(neo_gpu, oracle, C):
    """The owner's frame-stable promise (register(frame, frame_stable=True):
    NEO_HIP_GROUP_FRAME_STABLE): a coalesced frame read in place takes no snapshot and the members
    commit without comparing, so the outputs come from the blocks the frame held at the leader's
    call -- equal to one C-channel handle over the same blocks (to float rounding after the group
    re-primes), never a redo. Switching the flag off again restores the exact comparison: a member
    whose block changes after the leader's call is re-stepped and still matches."""
    B, L, nf = 512, 512 * 100, 16
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 2100 + C)
    frame = np.zeros((C, B), np.float32)
    g.register(frame, frame_stable=True)
    x = np.stack([oracle.noise(2200 + c, B * nf) for c in range(C)])
    late = (3, C - 1)
    for f in range(nf):
        if f == 11:
            g.register(frame, frame_stable=False)  # the same range again: the flag is updated
        blk = np.ascontiguousarray(x[:, f * B:(f + 1) * B])
        expect = ref(blk.copy())
        frame[:] = blk
        if f >= 12:  # not stable any more: these blocks change after the leader's call
            frame[list(late)] = 0.0
        for c in range(C):
            if f >= 12 and c in late:
                frame[c] = blk[c]
            g(ids[c], frame[c])
        err = np.abs(frame - expect).max(axis=1) / np.maximum(np.abs(expect).max(axis=1), 1e-3)
        assert err.max() <= 1e-5, (f, int(err.argmax()), float(err.max()))
    st = g.stats()
    assert st["coalesced"] and st["frame_steps"] == nf - 3 and st["redos"] == len(late) * (nf - 12), st


@pytest.mark.parametrize("C", [16, 520])
def test_group_frame_in_place(neo_gpu, oracle, C):
    """NEO_HIP_GROUP_FRAME_INPLACE (register(frame, in_place=True)): the frame's first call writes
    every member's output into its own block of the frame, and the later members' calls return at
    once -- the frame equals one C-channel handle over the same blocks after the last call (to float
    rounding: the group re-primes when it coalesces), with no redo. A member called once on a
    buffer outside the frame is still stepped exactly (its own block step again)."""
    B, L, nf = 512, 512 * 100, 14
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 2400 + C)
    frame = np.zeros((C, B), np.float32)
    g.register(frame, in_place=True)
    x = np.stack([oracle.noise(2500 + c, B * nf) for c in range(C)])
    odd = np.zeros(B, np.float32)
    for f in range(nf):
        blk = np.ascontiguousarray(x[:, f * B:(f + 1) * B])
        expect = ref(blk.copy())
        frame[:] = blk
        for c in range(C):
            if f == 10 and c == 1:  # one call on another buffer: exact, the frame's block 1 is stale
                odd[:] = blk[c]
                g(ids[c], odd)
                frame[c] = odd
            else:
                g(ids[c], frame[c])
        err = np.abs(frame - expect).max(axis=1) / np.maximum(np.abs(expect).max(axis=1), 1e-3)
        assert err.max() <= 1e-5, (f, int(err.argmax()), float(err.max()))
    st = g.stats()
    assert st["coalesced"] and st["redos"] == 1, st


def test_group_frame_stable_foreign_buffer(neo_gpu, oracle):
    """Under the frame-stable promise the members skip the comparison only on the buffer the
    leader's step read in place: a member called once on another buffer, holding another block than
    its frame block, is stepped again on that block (exact), and the frame's own block is left as it
    was."""
    C, B, L, nf = 12, 512, 512 * 100, 12
    g, ids, parts, ref = _setup(neo_gpu, oracle, C, B, L, 2700)
    frame = np.zeros((C, B), np.float32)
    g.register(frame, frame_stable=True)
    x = np.stack([oracle.noise(2800 + c, B * nf) for c in range(C)])
    odd = np.zeros(B, np.float32)
    for f in range(nf):
        blk = np.ascontiguousarray(x[:, f * B:(f + 1) * B])
        expect = ref(blk.copy())
        frame[:] = blk
        if f == 8:
            frame[2] = 0.0  # the leader reads zeros for member 2; its call brings the real block
        for c in range(C):
            if f == 8 and c == 2:
                odd[:] = blk[c]
                g(ids[c], odd)
                frame[c] = odd
            else:
                g(ids[c], frame[c])
        err = np.abs(frame - expect).max(axis=1) / np.maximum(np.abs(expect).max(axis=1), 1e-3)
        assert err.max() <= 1e-5, (f, int(err.argmax()), float(err.max()))
    st = g.stats()
    assert st["coalesced"] and st["redos"] == 1, st
