"""The streaming level schedule (neo-dsp_amd/csrc/upols_levels.hip), restated in float64
numpy and checked against the direct block-axis convolution — no GPU needed.

Per bin the convolver output is Y[t] = sum_p H[p] X[t - p]
(uniform_partitioned_convolver.hpp:47-65; fdl_index.hpp:23-36: partition p meets FDL row
t - p). The HIP path splits the partitions into the bands of neo_hip_upols_level_plan: the
block itself takes partitions 0..a0-1, each Toeplitz level computes its next window during
the current one (a slice of the bins per step, from FDL rows before the current window), and
the far level does the same in three phases (phase 1 and 2a in one step, 2b in the next). All of it runs in ONE launch per
step (k_lvl_step), so no role may read what another role of the same step writes. This test
replays exactly that schedule — the ring positions the host passes (tw), the slice ranges,
the double-buffered slabs, the far level's XF ring of row-pair spectra, its partial sums (phase 1 in window pairs) and
256-point partition-axis transforms — on random spectra, with history before the levels
start, ring wraparound and re-priming, running the roles of every step in a random order
(with the block's FDL row written at a random point among them), and checks every output
block. With step groups (neo_hip_upols_opts.step_group) the levels of T >= 2 G run in background
launches every G steps on a second stream; the replay runs their roles at random points between
the blocks they wait for and the block that waits for them (test_level_schedule_step_groups).
It pins the index arithmetic the kernels share with the host code; the kernels' arithmetic
itself is pinned by the GPU parity tests against the oracle.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "neo-dsp_amd"))

FT, FA, FN = 128, 256, 256  # far window, first far partition, transform length
FS = FT - 1  # far slices per window (kFarS)


def plan(P):
    import neo

    try:
        return neo.convolution.level_plan(P)
    except OSError as e:  # pragma: no cover - library not built
        pytest.skip(f"libneo_hip.so not loadable: {e}")


class Sim:
    """float64 replay of the level pipeline for one channel of K bins."""

    def __init__(self, H, lp, G=4, Kw=None, sg=1, whole=False, raw=False):
        self.H, self.lp, self.G, self.sg = H, lp, G, sg
        self.whole = whole  # G = 1: far phase 2 in one workgroup per unit (far2_whole)
        self.raw = raw  # the recomputed far level (far2r_role: every segment from ring rows each window)
        self.ns = FS if sg == 1 else FT // sg - 2  # far slices per window (far_nslices)
        self.pending = []  # step groups: background launches [roles left, due block] in stream order
        # step groups: a background level of window 4 sg <= T <= 32 starts its windows half a window
        # later (part_phi), and a window's units are cut into its parts at arbitrary points (the
        # library balances the groups' bytes; any cuts must give the same outputs: random here)
        self.phi = [T // 2 if sg > 1 and 4 * sg <= T <= 32 else 0 for T in lp["T"]]
        self.cuts = {}
        # and the far slices' cuts (the same every window), arbitrary too with step groups
        K_ = H.shape[1]
        self.fcut = None
        if sg > 1:
            self.fcut = [0] + sorted(np.random.default_rng(H.shape[0] + 7).integers(0, K_ + 1, size=self.ns - 1).tolist()) + [K_]
        ns = lp["nseg"]
        self.P, self.K = H.shape
        # windows per phase-1 pass: the kernel's automatic choice for this many 16-column units
        # (bench.far_group restates upols_levels.hip far_group), or a forced value
        # (neo_hip_upols_opts.far_group)
        if Kw is None:
            sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
            import bench

            Kw = bench.far_group(ns, max(1, self.K // 16))
        self.Kw = Kw
        self.R = self.P + 31
        if lp["nseg"]:
            self.R = max(self.R, 2 * FA)
        if lp["nseg"] and raw:
            self.R = max(self.R, self.P + 2 * FT)  # upols.hip: the recomputed level reads back P + 128 rows
        self.ring = np.zeros((self.R, self.K), complex)
        self.w = 0
        self.n = -1
        self.slab = [np.zeros((2, T, self.K), complex) for T in lp["T"]]
        self.rng = np.random.default_rng(self.P)
        ns = lp["nseg"]
        if ns:
            self.M = ns
            # segment spectra: s -> partitions [128 (s + 2), 128 (s + 3)), zero-padded to 256
            seg = np.zeros((ns, FN, self.K), complex)
            for s in range(ns):
                lo = FT * (s + 2)
                hi = min(self.P, lo + FT)
                seg[s, : hi - lo] = H[lo:hi]
            self.HF = np.fft.fft(seg, axis=1)
            self.XF = np.zeros((ns, FN, self.K), complex)
            self.ff = np.zeros((2, FT, self.K), complex)
            self.acc = np.zeros((self.Kw, FN, self.K), complex)

    def join(self):
        """lvl_join: every background launch enqueued so far completes"""
        while self.pending:
            roles, _ = self.pending.pop(0)
            for r in roles:
                r()

    def plain(self, x):
        """One plain step (all partitions from the ring); the levels re-prime after it."""
        self.join()
        self.ring[self.w] = x
        y = (self.H * self.ring[(self.w - np.arange(self.P)) % self.R]).sum(0)
        self.w = (self.w + 1) % self.R
        self.n = -1
        return y

    def toep(self, l, tw, k0, k1, buf):
        T, a, b = self.lp["T"][l], self.lp["a"][l], self.lp["b"][l]
        ps = np.arange(a, b)
        for j in range(T):
            rows = (tw + j - ps) % self.R
            self.slab[l][buf, j, k0:k1] = (self.H[a:b, k0:k1] * self.ring[rows, k0:k1]).sum(0)

    def cls(self, k):
        """phase-1 class of column k (the kernels: 16-column unit u, group u // 4, class mod K)"""
        return (k // self.G) % self.Kw

    def first(self, c):
        """first window >= 1 whose phase-1 pass a class starts (far_first)"""
        return 1 + ((c - 1) % self.Kw)

    def far1(self, wn, k0, k1, nfresh, mode=0, cls=0):
        """phase 1: the stored segments' products into the partial sums of window wn; mode 1:
        the columns of class cls, each for the windows wn .. wn + K - 1 (segments s >= j + 1 of
        wn + j use the slots of s - j of wn); mode 2: those, and the classes that have not
        started for wn alone"""
        ns, K = self.lp["nseg"], self.Kw
        for k in range(k0, k1):
            c = self.cls(k) if mode else 0
            if mode and c != cls:
                if self.first(c) <= wn:
                    continue  # inside a group started earlier
                nw = 1
            else:
                nw = K if mode else 1
            for j in range(nw):
                acc = np.zeros(FN, complex)
                for s in range(max(min(nfresh, ns), j + 1), ns):
                    acc += self.XF[(wn - (s - j) - 1) % self.M, :, k] * self.HF[s, :, k]
                self.acc[(wn + j) % K, :, k] = acc

    def far2a(self, tw, wn, k0, k1, nfresh):
        """phase 2a: the fresh row pairs' transforms, stored to their slots"""
        ns = self.lp["nseg"]
        for s in range(min(nfresh, ns)):
            slot = (wn - s - 1) % self.M
            rows = [(tw - (s + 3) * FT + i) % self.R for i in range(FN)]
            self.XF[slot, :, k0:k1] = np.fft.fft(self.ring[rows, k0:k1], axis=0)

    def far2b(self, wn, k0, k1, nfresh, grp=False):
        """phase 2b (one step after 2a): the partial sums, the fresh segments' products from
        their slots, segments 1 .. j for window j of a phase-1 group, the inverse transform
        into the far field"""
        ns, K = self.lp["nseg"], self.Kw
        acc = self.acc[wn % K, :, k0:k1].copy()
        for s in range(min(nfresh, ns)):
            slot = (wn - s - 1) % self.M
            acc += self.XF[slot, :, k0:k1] * self.HF[s, :, k0:k1]
        if grp:
            for k in range(k0, k1):
                c = self.cls(k)
                j = (wn - c) % K if wn >= self.first(c) else 0
                for s in range(1, min(j, ns - 1) + 1):
                    acc[:, k - k0] += self.XF[(wn - s - 1) % self.M, :, k] * self.HF[s, :, k]
        self.ff[wn & 1, :, k0:k1] = np.fft.ifft(acc, axis=0)[FT:]

    def far2r(self, tw, wn, k0, k1):
        """the recomputed far level (far2r_role): window wn's field from the row pairs of every
        segment (rows tw - (s + 3) 128 + r, r < 256) and the segment spectra, nothing stored"""
        acc = np.zeros((FN, k1 - k0), complex)
        for s in range(self.lp["nseg"]):
            rows = [(tw - (s + 3) * FT + i) % self.R for i in range(FN)]
            acc += np.fft.fft(self.ring[rows, k0:k1], axis=0) * self.HF[s, :, k0:k1]
        self.ff[wn & 1, :, k0:k1] = np.fft.ifft(acc, axis=0)[FT:]

    def span(self, q):
        """columns of far slice q (far_nslices: 127 slices per window, kFarT / G - 2 with step groups,
        cut where part_plan puts it: arbitrary here)"""
        if self.fcut is not None:
            return self.fcut[q], self.fcut[q + 1]
        return q * self.K // self.ns, (q + 1) * self.K // self.ns

    def far1_slice(self, W, q):
        """phase 1 for slice q of window W, in groups"""
        k0, k1 = self.span(q)
        if k1 > k0:
            K = self.Kw
            self.far1(W, k0, k1, 1, 0 if K == 1 else (2 if W < K else 1), W % K)

    def roles(self, n, w):
        """the slice roles of step n's launch (block at ring row w), as closures; step groups: the
        levels of T < 2 sg (block_levels)"""
        lp, K, R = self.lp, self.K, self.R
        out = []
        for l, T in enumerate(lp["T"]):
            if self.sg > 1 and T >= 2 * self.sg:
                break
            U = K // 16 if K >= 16 else K  # 16-column units (toep_geom: one window part each)
            st, W = n % T, n // T + 1
            u0, u1 = st * U // T, (st + 1) * U // T
            if u1 > u0:
                k0, k1 = u0 * K // U, u1 * K // U
                out.append(lambda l=l, T=T, W=W, k0=k0, k1=k1: self.toep(l, (w + W * T - n) % R, k0, k1, W & 1))
        if lp["nseg"] and self.sg == 1 and self.raw:
            q, W = n % FT, n // FT + 1
            if 1 <= q <= FS:  # slice q - 1 of window W whole
                k0, k1 = self.span(q - 1)
                out.append(lambda k0=k0, k1=k1, tw=(w + W * FT - n) % R: self.far2r(tw, W, k0, k1))
        elif lp["nseg"] and self.sg == 1 and self.whole:
            q, W = n % FT, n // FT + 1
            if q < FS:  # phase 1 of slice q
                out.append(lambda: self.far1_slice(W, q))
            if q >= 1:  # phase 2 of slice q - 1: 2a and 2b in one workgroup (far2c_role)
                k0, k1 = self.span(q - 1)
                tw = (w + W * FT - n) % R

                def far2c(k0=k0, k1=k1, tw=tw):
                    self.far2a(tw, W, k0, k1, 1)
                    self.far2b(W, k0, k1, 1, self.Kw > 1)
                out.append(far2c)
        elif lp["nseg"] and self.sg == 1:
            q, W = n % FT, n // FT + 1
            if q < FS:  # phase 1 and 2a of slice q
                k0, k1 = self.span(q)
                out.append(lambda: self.far1_slice(W, q))
                out.append(lambda k0=k0, k1=k1: self.far2a((w + W * FT - n) % R, W, k0, k1, 1))
            if q >= 1:  # 2b of slice q - 1
                k0, k1 = self.span(q - 1)
                out.append(lambda k0=k0, k1=k1: self.far2b(W, k0, k1, 1, self.Kw > 1))
        return out

    def bg_roles(self, n0, w0):
        """step groups: the background launch issued at step n0 (slice_part), as closures"""
        lp, K, R, G = self.lp, self.K, self.R, self.sg
        out = []
        for l, T in enumerate(lp["T"]):
            if T < 2 * G:
                continue
            m0 = n0 + self.phi[l]
            j, np_, W = (m0 % T) // G, T // G - 1, m0 // T + 1  # part j of window W (the next one)
            if j >= 1:
                if (l, W) not in self.cuts:
                    self.cuts[(l, W)] = [0] + sorted(self.rng.integers(0, K + 1, size=np_ - 1).tolist()) + [K]
                k0, k1 = self.cuts[(l, W)][j - 1], self.cuts[(l, W)][j]
                if k1 > k0:
                    out.append(lambda l=l, T=T, W=W, k0=k0, k1=k1, m0=m0: self.toep(l, (w0 + W * T - m0) % R, k0, k1, W & 1))
        if lp["nseg"] and self.raw:
            q, W = (n0 % FT) // G, n0 // FT + 1
            if 2 <= q and q - 2 < self.ns:  # slice q - 2 of window W whole, at phase 2's time
                k0, k1 = self.span(q - 2)
                out.append(lambda k0=k0, k1=k1, tw=(w0 + W * FT - n0) % R: self.far2r(tw, W, k0, k1))
        elif lp["nseg"]:
            q, W = (n0 % FT) // G, n0 // FT + 1
            if 1 <= q <= self.ns:  # phase 1 of slice q - 1
                out.append(lambda: self.far1_slice(W, q - 1))
            if q >= 2:  # phase 2 of slice q - 2: 2a and 2b in one workgroup (far2c_role)
                k0, k1 = self.span(q - 2)
                tw = (w0 + W * FT - n0) % R

                def far2c(k0=k0, k1=k1, tw=tw):
                    self.far2a(tw, W, k0, k1, 1)
                    self.far2b(W, k0, k1, 1, self.Kw > 1)
                out.append(far2c)
        return [out[i] for i in self.rng.permutation(len(out))]  # any order inside a launch

    def prime(self):
        self.join()
        self.cuts = {}
        for l, T in enumerate(self.lp["T"]):
            self.toep(l, (self.w - self.phi[l]) % self.R, 0, self.K, 0)  # window 0 began phi steps ago
            if self.phi[l]:  # and window 1 whole (its parts before step 0 never ran)
                self.toep(l, (self.w + T - self.phi[l]) % self.R, 0, self.K, 1)
        if self.lp["nseg"] and self.raw:
            self.far2r(self.w, 0, 0, self.K)
        elif self.lp["nseg"]:
            ns = self.lp["nseg"]  # phase 1 and 2a of every column, then 2b (two launches)
            self.far1(0, 0, self.K, ns)
            self.far2a(self.w, 0, 0, self.K, ns)
            self.far2b(0, 0, self.K, ns)
        self.n = 0

    def step(self, x):
        if self.n < 0:
            self.prime()
        n, lp, R, w = self.n, self.lp, self.R, self.w
        y = [None]

        def block_read():  # partitions 1..a0-1, the block's slabs and far field
            r = (self.H[1: lp["a0"]] * self.ring[(w - np.arange(1, lp["a0"])) % R]).sum(0)
            for l, T in enumerate(lp["T"]):
                m = n + self.phi[l]
                r = r + self.slab[l][(m // T) & 1, m % T]
            if lp["nseg"]:
                r = r + self.ff[(n // FT) & 1, n % FT]
            y[0] = r + self.H[0] * x

        def block_write():
            self.ring[w] = x

        jobs = self.roles(n, w) + [block_read, block_write]
        jobs = [jobs[i] for i in self.rng.permutation(len(jobs))]
        G = self.sg
        if G > 1:
            if n % G == 0:
                # issued now; it waits for the blocks before n - G (odd group) / n - 2 G (even:
                # its predecessor waited for those), so it may run beside the blocks from there on
                # (those already done here); due before the next even group's block
                odd = (n // G) & 1
                self.pending.append([self.bg_roles(n, w), n + G if odd else n + 2 * G])
            # the block of an even group waits for every background launch due by now
            while self.pending and self.pending[0][1] <= n:
                roles, _ = self.pending.pop(0)
                for r in roles:
                    r()
            # background roles (in stream order) interleaved at random with this launch's
            bgq = [r for p in self.pending for r in p[0]]
            k = int(self.rng.integers(0, len(bgq) + 1))
            slots = set(self.rng.choice(len(jobs) + k, size=k, replace=False).tolist()) if k else set()
            it, jt = iter(bgq[:k]), iter(jobs)
            jobs = [next(it) if i in slots else next(jt) for i in range(len(jobs) + k)]
            left = k  # drop the executed roles from the pending launches
            while left:
                p = self.pending[0]
                d = min(left, len(p[0]))
                del p[0][:d]
                left -= d
                if not p[0]:
                    self.pending.pop(0)
        for j in jobs:
            j()
        self.w = (w + 1) % R
        self.n = n + 1
        return y[0]


def test_level_plan_bands():
    """Bands tile [0, P) exactly; every band [a, b) with window T starts at >= 2T."""
    for P in [1, 2, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 256, 257, 383, 384, 385, 938, 1875, 4000]:
        lp = plan(P)
        cover = [(0, lp["a0"])] + list(zip(lp["a"], lp["b"]))
        if lp["nseg"]:
            cover.append((FA, FA + FT * lp["nseg"]))
            assert FA + FT * (lp["nseg"] - 1) < P <= FA + FT * lp["nseg"]
        assert cover[0][0] == 0
        for (lo, hi), (lo2, _) in zip(cover, cover[1:]):
            assert hi == lo2, (P, cover)
        assert min(cover[-1][1], P) == P or (lp["nseg"] and cover[-1][1] >= P)
        for T, a in zip(lp["T"], lp["a"]):
            assert a >= 2 * T


@pytest.mark.parametrize("P", [5, 20, 40, 100, 257, 300, 700, 1100])
def test_level_schedule_matches_direct(P):
    lp = plan(P)
    rng = np.random.default_rng(P)
    K = 16
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp)
    nb = max(3 * P, 2 * P + 300) if lp["nseg"] else 3 * P + 40
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        # plain steps first (history before the levels start), and again midway (re-prime)
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("P", [300, 700])
def test_level_schedule_big_level(P):
    """The same schedule with [256, P) as the 128-block Toeplitz level instead of the far
    level (neo_hip_upols_opts.far_level = 0)."""
    lp = dict(plan(P))
    assert lp["nseg"]
    lp["T"], lp["a"], lp["b"] = list(lp["T"]) + [128], list(lp["a"]) + [256], list(lp["b"]) + [P]
    lp["nseg"] = 0
    rng = np.random.default_rng(P + 1)
    K = 16
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp)
    nb = 3 * P + 40
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("P,Kw", [(700, 2), (700, 4), (1100, 3), (1100, 4), (450, 3)])
def test_level_schedule_window_groups(P, Kw):
    """The far level's phase 1 over groups of Kw windows (far_group picks one per nseg; every
    group size must give the same outputs), across re-priming."""
    lp = plan(P)
    rng = np.random.default_rng(P + Kw)
    K = 32
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp, Kw=Kw)
    nb = 2 * P + 700
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("P,sg,Kw", [(40, 2, None), (100, 4, None), (300, 4, None), (300, 8, None), (700, 2, 3),
                                     (700, 4, 2), (1100, 8, 4), (450, 4, 3)])
def test_level_schedule_step_groups(P, sg, Kw):
    """Step groups (neo_hip_upols_opts.step_group = sg): the block launch of every step (the
    block and the levels of T < 2 sg) and a background launch every sg steps (slice_part: level
    T's window W + 1 in T / sg - 1 parts at t_W + sg j, the far level's slices phase 1 / 2a one
    group and 2b two groups after the window start), the background launches running at random
    points between the blocks they wait for (before n - sg, odd groups) and the even-group block
    that waits for them; across plain steps (join) and re-priming."""
    lp = plan(P)
    rng = np.random.default_rng(P + 10 * sg)
    K = 32
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp, Kw=Kw, sg=sg)
    nb = max(3 * P, 2 * P + 300) if lp["nseg"] else 3 * P + 60
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("P,Kw", [(300, 2), (700, 2), (700, 3), (1100, 4), (450, 1)])
def test_level_schedule_far_phase2_whole(P, Kw):
    """G = 1 with far phase 2 in one workgroup per unit (neo_hip_upols_opts.far_phase2 = 1,
    far2_whole): phase 1 of slice q at step q, the fresh transform, the products and the inverse
    of slice q - 1 at step q, in one role (the fresh spectrum written to its slot in the same
    role), across re-priming."""
    lp = plan(P)
    rng = np.random.default_rng(P + 100 * Kw)
    K = 32
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp, Kw=Kw, whole=True)
    nb = 2 * P + 700
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("P,sg", [(257, 1), (300, 1), (700, 1), (450, 4), (700, 4), (1100, 8), (1100, 2), (385, 4)])
def test_level_schedule_far_recomputed(P, sg):
    """The recomputed far level (neo_hip_upols_opts.far_level = 2, far2r_role): slice q of window W takes every segment from the ring's rows and the segment
    spectra at once (G = 1: at step q + 1 of window W - 1; step groups: with phase 2's background
    launch, group q + 2), nothing stored between windows but the field; the ring of P + 256 rows
    the handle allocates, background launches at random points inside their windows, across
    plain steps and re-priming."""
    lp = plan(P)
    assert lp["nseg"]
    rng = np.random.default_rng(P + 1000 * sg)
    K = 32
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    sim = Sim(H, lp, sg=sg, raw=True)
    nb = 2 * P + 700
    X = rng.standard_normal((nb, K)) + 1j * rng.standard_normal((nb, K))
    worst = 0.0
    for t in range(nb):
        y = sim.plain(X[t]) if (t < 37 or nb // 2 <= t < nb // 2 + 3) else sim.step(X[t])
        m = min(P, t + 1)
        ref = (H[:m] * X[t - np.arange(m)]).sum(0)
        worst = max(worst, float(np.abs(y - ref).max() / (np.abs(ref).max() + 1e-300)))
    assert worst < 1e-12, worst


@pytest.mark.parametrize("C,B,P,G", [(2048, 512, 938, 4), (256, 512, 938, 4), (256, 256, 1875, 4), (64, 256, 700, 8),
                                     (16, 64, 300, 2), (4, 256, 300, 4), (1, 512, 188, 4)])
def test_part_plan_valid_and_balanced(C, B, P, G):
    """The library's background plan (part_plan, upols_levels.hip): window offsets phi = T / 2 for
    the background levels of 4 G <= T <= 32 (the replay above runs the same offsets with arbitrary
    cuts); every window's cuts run 0 .. U in order; at the 256- and 2048-channel shapes every step
    group of the far window carries 0.99-1.01 of the mean background bytes (before: an empty group
    every 8), and so any 5 consecutive groups (a 20-step sample)."""
    import neo

    lp = plan(P)
    p = neo.convolution.part_plan(C, B, P, G)
    for l, T in enumerate(lp["T"]):
        assert p["phi"][l] == (T // 2 if 4 * G <= T <= 32 else 0)
    for l, wins in p["cuts"].items():
        T = lp["T"][l]
        JH = (2 if C * (B // 16) < 256 else 1) if T == 32 else 1
        U = C * (B // 16) * JH
        assert len(wins) == p["cycle"] // (T // G)
        for c in wins:
            assert len(c) == T // G and c[0] == 0 and all(x <= y for x, y in zip(c, c[1:]))
            assert c[-1] == U
    if C >= 256:
        ld = np.array(p["loads"])
        m = ld.mean()
        assert 0.99 * m <= ld.min() and ld.max() <= 1.01 * m, (ld.min() / m, ld.max() / m)
        w5 = [ld[[(g + i) % len(ld) for i in range(5)]].mean() / m for g in range(len(ld))]
        assert 0.99 <= min(w5) and max(w5) <= 1.01, (min(w5), max(w5))
        u = np.array(neo.convolution.part_plan(C, B, P, G, uniform=True)["loads"])
        assert u.min() < 0.1 * u.mean()  # the plan before: empty groups


def _offline_replay(H, X, R, wp, w0, ring0):
    """float64 replay of the offline windows (launch_offline + k_off_mac): the FDL ring of R rows
    holds history (ring0, next write position w0); each pass inserts 128 wp rows at w, then per window walks the pairs from the
    newest back (pair i = rows w + 128 (wp - 2) - 128 i ... + 255 mod R, i = 0 .. nseg + wp - 2),
    each pair's second half being the previous pair's first half, multiplies segment q's spectrum
    with the pair of window j's segment q (pair index q + wp - 1 - j), and keeps samples 128..255
    of one inverse transform per window."""
    P, K = H.shape
    nseg = -(-P // FT)
    Hp = np.zeros((nseg * FT, K), complex)
    Hp[:P] = H
    HF = [np.fft.fft(np.concatenate([Hp[q * FT:(q + 1) * FT], np.zeros((FT, K))]), axis=0) for q in range(nseg)]
    ring = ring0.copy()
    w = w0
    out = []
    t = 0
    nb = X.shape[0]
    while t + FT * wp <= nb:
        for j in range(FT * wp):  # k_batch_window: rows w .. w + 128 wp - 1
            ring[(w + j) % R] = X[t + j]
        acc = [np.zeros((FN, K), complex) for _ in range(wp)]
        half = None
        for i in range(nseg + wp - 1):
            start = w + FT * (wp - 2) - FT * i
            rows = np.array([(start + r) % R for r in range(FN)])
            pair = ring[rows].copy()
            if half is not None:
                assert np.array_equal(pair[FT:], half)  # the previous pair's first half
            half = pair[:FT].copy()
            XF = np.fft.fft(pair, axis=0)
            for jw in range(wp):
                q = i - (wp - 1 - jw)
                if 0 <= q < nseg:
                    acc[jw] += XF * HF[q]
        for jw in range(wp):
            out.append(np.fft.ifft(acc[jw], axis=0)[FT:])
        w = (w + FT * wp) % R
        t += FT * wp
    return np.concatenate(out) if out else np.zeros((0, K))


@pytest.mark.parametrize("P,wp", [(128, 1), (129, 2), (300, 2), (300, 1), (700, 2), (938, 2), (1000, 1)])
def test_offline_windows_match_direct(P, wp):
    """The offline windows' decomposition and ring arithmetic (upols_levels.hip k_off_mac,
    upols_batch.hip launch_offline; ring of 128 (nseg + 2) rows, upols.hip create): random
    spectra with history before the first pass, several passes wrapping the ring, against the
    direct block-axis convolution Y[t] = sum_p H[p] X[t - p] (uniform_partitioned_convolver.hpp:47-65,
    fdl_index.hpp:23-36)."""
    rng = np.random.default_rng(P + wp)
    K = 3
    nseg = -(-P // FT)
    R = max(P + 31, FT * (nseg + 2))
    H = rng.standard_normal((P, K)) + 1j * rng.standard_normal((P, K))
    hist = R - FT * 2  # blocks before the first pass (already in the ring)
    nb = FT * wp * 5
    Xall = rng.standard_normal((hist + nb, K)) + 1j * rng.standard_normal((hist + nb, K))
    # direct reference over the whole history
    Y = np.zeros((hist + nb, K), complex)
    for t in range(hist + nb):
        p = np.arange(min(P, t + 1))
        Y[t] = (H[p] * Xall[t - p]).sum(0)
    # the ring after `hist` single steps from write position 0: row t mod R holds block t
    w0 = hist % R
    ring_hist = np.zeros((R, K), complex)
    for t in range(hist):
        ring_hist[t % R] = Xall[t]
    got = _offline_replay(H, Xall[hist:], R, wp, w0, ring_hist)
    np.testing.assert_allclose(got, Y[hist:hist + got.shape[0]], rtol=0, atol=1e-9 * np.abs(Y).max())
