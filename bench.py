#!/usr/bin/env python3
"""bench.py — MI355X throughput of neo's UPOLS convolver (and FFT) hot path.

Headline (BASELINE.json metric "Msamples/sec UPOLS convolver (block=512,
IR=10s@48k); achieved HBM GB/s"): configs[4], the 2048-channel UPOLS, B = 512,
L = 480000 taps (P = 938), channel-sharded across the GPUs of one node. `--workload c5full`
(the default) is that configuration: 2048 channels IN ALL, rank r of N owning the
contiguous channel range shard(2048, N, r) — at N = 1 all 2048 on one GPU (the whole
configuration fits one MI355X: ~60 GB of filter, FDL and level buffers of 288 GB), at
N = 8 exactly the 256-channel shard per GPU (`scaling` "strong"). The channels are
independent, so there is no collective on the data path — torch.distributed (gloo) only
carries the timing barrier and the max over ranks. For N > 1 a secondary `weak` object
also times 2048 channels per GPU (N x 2048 in all). `--workload c5` is one GPU's
256-channel shard of the 8-GPU split on its own.

A "step" = one block of B samples through the whole convolver for every channel, inputs
already resident in HBM, one call per block. The timed region enqueues the K calls on the
convolver's stream and synchronizes once at the end (the GPU runs the blocks in stream
order, each step's kernel after the previous one's); `latency.host_roundtrip_*` is the
real-time caller's view instead: one call per block and a host wait for that block's output
before the next call. The convolver's default streaming form is the level pipeline
(upols_levels.hip): every step runs the block step (window r2c, FDL insert, the 8 newest
partitions, c2r) plus 1/T of the next window of each partition level, so every step does
the same work and the line is the same at any --steps. `roofline` holds the step kernel with
its HIP-event time, algorithmic bytes by role and PMC traffic. `latency` is the per-step GPU
time distribution plus the host round trip, `parity` the last timed blocks against the
oracle, `per_block_step` the plain one-pass-per-block step, `offline` the batched form
(blocks up front), `host_io` the host-buffer boundary (neo_hip_upols_process: the block in
host memory, PCIe-inclusive, one synchronous call per block), all timed in the same run;
`c2_fft` the 4096 x 65536 batched FFT.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5full|c5|c4|c3|c2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd")]

PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP32_TFLOPS = 157.3  # MI355X fp32 vector (packed FMA) peak, 256 CU x 4 SIMD x 64 flop/clk x 2.4 GHz
# Untimed warm-up: at least --warmup steps AND at least this much GPU time. MI355X runs
# the first ~20 ms of sustained HBM load measurably slower (clock ramp; measured 0.93 vs
# 0.74 ms for the 4096 x 65536 FFT), which a few warm-up steps do not cover.
WARM_SECONDS = 0.25

WORKLOADS = {
    # name: (channels, block, taps); c5full's 2048 are split over the ranks (strong scaling),
    # the others run per GPU (weak scaling)
    "c5full": (2048, 512, 480000),  # headline: configs[4], 2048 channels sharded over the GPUs
    "c5": (256, 512, 480000),  # one GPU's shard of 2048 ch / 8 GPUs, B=512, IR 10 s @ 48 kHz
    "c4": (256, 256, 480000),  # 256 ch, B=256, IR 10 s @ 48 kHz
    "c3": (1, 512, 96000),     # 1 ch, B=512, IR 2 s @ 48 kHz
    "c3long": (1, 512, 480000),  # 1 ch with the headline's 10 s IR (far level): the plugin's real-time case
    # the reference benchmark's own shape (extra/benchmark/src/convolution.cpp:47-55, its longest
    # IR): 1 ch, B=4096, IR 2^17 taps, P=32: the plain step (no streaming levels)
    "ref4096": (1, 4096, 131072),
}
STRONG = {"c5full"}  # workloads whose channel count is the whole job's, split over the ranks


def cpu_threads() -> int:
    """Host threads this process may use: its CPU affinity mask (the box's CPU share), at
    most 16 (the pool's per-GPU share; os.cpu_count() reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c5full", choices=sorted(WORKLOADS) + ["c2"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ahead", action="store_true", help="headline = the plain one-pass-per-block step")
    ap.add_argument("--no-offline", action="store_true", help="skip the batched (blocks up front) line")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the timed output")
    ap.add_argument("--no-fft", action="store_true", help="skip the c2_fft sub-object of UPOLS runs")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the affinity mask's CPUs, at most 16")
    ap.add_argument("--no-host-io", action="store_true", help="skip the host_io sub-object")
    ap.add_argument("--no-paced", action="store_true",
                    help="skip latency.paced (its per-call background pieces would mix into kernel-level profiles)")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the secondary weak-scaling object")
    ap.add_argument("--far-group", type=int, default=0,
                    help="neo_hip_upols_opts.far_group: 0 auto, 1..4 windows per far phase-1 pass")
    ap.add_argument("--step-group", type=int, default=0,
                    help="neo_hip_upols_opts.step_group: 0 auto, 1 one launch per step, 2 / 4 step groups")
    ap.add_argument("--far-level", type=int, default=-1,
                    help="neo_hip_upols_opts.far_level: -1 auto, 0 128-block Toeplitz, 1 transform with stored "
                         "spectra, 2 transform recomputed every window")
    ap.add_argument("--far-phase2", type=int, default=0,
                    help="neo_hip_upols_opts.far_phase2 (G = 1): 0 auto, 1 one workgroup per unit, 2 two steps")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="single process: run rank 0's channel shard of an N-GPU strong-scaling job (the per-GPU "
                         "shape the driver's N-GPU run gives each rank; diagnostic, never the headline)")
    ap.add_argument("--host-io", action="store_true",
                    help="time the host-buffer boundary (neo_hip_upols_process on pinned-staged host memory): "
                         "PCIe-inclusive, reported for DESIGN.md, never the headline value")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints connection chatter on fd 1; keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)
    return world, rank, local


def shard(total: int, world: int, rank: int):
    """Contiguous channel range [lo, hi) owned by `rank` (sizes differ by at most one)."""
    return total * rank // world, total * (rank + 1) // world


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def gather_over_ranks(x: float, world: int) -> list:
    """x of every rank, in rank order (gloo all_gather; [x] at world 1)."""
    if world == 1:
        return [x]
    import torch
    import torch.distributed as dist

    out = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, torch.tensor([x], dtype=torch.float64))
    return [float(t.item()) for t in out]


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# the translation units whose kernels the PMC passes measure (the streaming step, the plain and
# batched steps, the FFT) and every shared header; host-only units (groups, multi-device shards,
# setup, one-shot convolution, overlap stages, the library glue) do not change what they measured
PMC_SOURCES = ("upols_levels.hip", "upols.hip", "upols_batch.hip", "fft.hip")


def code_tag() -> str:
    """Hash of the measured kernels' sources: PMC summaries count only for the code they measured."""
    import glob
    import hashlib

    h = hashlib.sha1()
    csrc = os.path.join(REPO, "neo-dsp_amd", "csrc")
    paths = sorted(glob.glob(os.path.join(csrc, "*.hpp"))) + [os.path.join(csrc, f) for f in PMC_SOURCES]
    for path in paths:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:12]


def pmc_workload(workload: str, C: int):
    """The workload whose PMC summary measured this rank's shape (C channels of `workload`'s
    B and L), or None: at N GPUs a strong-scaled c5full rank runs 2048 / N channels, so N = 8
    reads c5's (256-channel) summary, and N = 2 / 4 (no summary of that shape) report no
    traffic rather than the 2048-channel figure."""
    if workload not in WORKLOADS:
        return workload
    _, B, L = WORKLOADS[workload]
    for w in (workload, *WORKLOADS):
        if WORKLOADS[w] == (C, B, L):
            return w
    return None


def _pmc_sfx(workload, suffix: str):
    return None if workload is None else workload + suffix


def load_pmc_traffic(workload, kernel: str = ""):
    """HBM bytes per launch (per step for the streaming parts) of `kernel` from a committed
    rocprofv3 --pmc summary (tools/pmc_summary.py) for `workload` measured on THIS code
    (same code_tag), or None (also for workload None: no summary of the rank's shape)."""
    import glob

    if workload is None:
        return None
    tag = code_tag()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            if (d.get("code_tag") == tag and d.get("workload") == workload and kernel in d.get("kernel", "")
                    and d.get("hbm_bytes_per_launch")):
                return float(d["hbm_bytes_per_launch"])
        except (OSError, ValueError):
            continue
    return None


def cpu_baseline_upols(C, B, L, threads):
    """The reference's SIMD CPU path (kind "port"): dense_convolve<upols_convolver> with the
    xsimd interleaved FDL MAC of a -march=native build (multiply_add.hpp:196-223) restated in
    oracle/neo_baseline.c, on bounded samples of the same workload on this box's host cores:
    1 thread, and `threads` threads (the cores this job may use). `value` is the all-threads
    figure. A reported baseline, not the target."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O

    # ~4 s each on the box's EPYC host (4.4 / 67 Msamples/s measured at B=512, P=938)
    nb1, nba = 8192 * 512 // B, 4096 * 512 // B
    cs_all = max(threads, 1) * 4
    ir = np.stack([O.noise(8 + c, L) for c in range(cs_all)])
    parts = O.uniform_partition(O.normalize_impulse(ir), B)
    sig = np.stack([O.noise(7000 + c, B * nb1) for c in range(cs_all)])

    def run(cs, nb, th):
        x = np.ascontiguousarray(sig[:cs, :nb * B])
        t0 = time.perf_counter()
        O.dense_convolve_simd(x, parts[:cs], threads=th)
        dt = time.perf_counter() - t0
        return cs * nb * B / dt / 1e6, dt

    v1, d1 = run(2, nb1, 1)
    va, da = run(cs_all, nba, threads)
    lvl = O.simd_level()
    return {"value": va, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "threads_1": v1, "threads_all": va, "simd": O.SIMD_NAMES[lvl],
            "sample": f"B={B}, L={L} (P={parts.shape[1]}): 2 channels x {nb1} blocks on 1 thread ({d1:.2f} s), "
                      f"{cs_all} channels x {nba} blocks on {threads} threads ({da:.2f} s); dense_convolve with "
                      f"the SIMD MAC ({O.SIMD_NAMES[lvl]}) over the oracle's c2c_dit2 r2c/c2r"}


def cpu_baseline_fft(threads):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O

    nb = 65536  # the whole C2 batch: ~4-10 s of one core
    x = O.noise(2, 2 * 4096 * nb).view(np.complex64).reshape(nb, 4096)
    t0 = time.perf_counter()
    O.fft(x)
    dt = time.perf_counter() - t0
    return {"value": nb * 4096 / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{nb} of the 65536 4096-pt transforms, oracle c2c_dit2 (bitrev + radix-2), 1 thread, "
                      f"{dt:.2f} s"}


def copy_ceiling_gbs(dev) -> float:
    """Practical HBM ceiling measured in the same run: a 1 GiB device-to-device copy
    (torch copy_ -> hipMemcpy D2D), read + write bytes over the best of 5."""
    import torch

    n = 1 << 28
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    best = None
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    del a, b
    return 2 * 4 * n / (best * 1e-3) / 1e9


def device_for(local: int) -> int:
    """One process per GPU: LOCAL_RANK -> device (modulo the visible devices, so a
    multi-rank rehearsal on a smaller box shares GPUs)."""
    import torch

    return local % max(1, torch.cuda.device_count())


class Feed:
    """Feeds the convolver the blocks of a cyclic input x [C][NX*B] (block g of the stream is
    block g mod NX of x; outputs land in y at the same place), so that the input history of
    any output block is known — the parity check replays it through the oracle."""

    def __init__(self, conv, x, y, nx, B, stream):
        self.conv, self.x, self.y, self.nx, self.B, self.stream = conv, x, y, nx, B, stream
        self.ld = nx * B
        self.g = 0  # blocks processed so far

    def run(self, n):
        while n > 0:
            i = self.g % self.nx
            k = min(n, self.nx - i)
            off = 4 * i * self.B
            self.conv.process_blocks_ptr(self.x.data_ptr() + off, self.y.data_ptr() + off, self.ld, k, self.stream)
            self.g += k
            n -= k


def far_group(nseg: int, units: int) -> int:
    """Windows per far phase-1 pass, as upols_levels.hip far_group: round(sqrt(2 (nseg - 1)))
    clamped to [2, 4] from 16384 16-column units (C * B / 16) on, else 2 (1 below two segments)."""
    import math

    if nseg < 2:
        return 1
    if units < 16384:
        return 2
    return min(4, max(2, int(math.floor(math.sqrt(2.0 * (nseg - 1)) + 0.5))))


def algorithmic_bytes(C, B, P, plan, G=1, far_k=0, far_form=1):
    """Algorithmic bytes per streaming step of the step kernel k_lvl_step, by role:
    block:     window (previous block + this block), previous-block write, output (4 x 4B per
               sample), FDL row write and H0 (2 x 8B per bin), partitions 1 .. a0 - 1 (filter +
               FDL row, 16B per bin each), one slab row per level and the far-field row (8B each)
    Toeplitz level (window T, band [a, b)), C*B/T columns per step: per column b - a filter
               rows + b - a + T - 1 FDL rows + T slab entries (8 B each)
    far level, C*B/128 columns per step (on average: 127 slices per 128-block window): per
               column 256 FDL rows and the new row-pair spectrum (256 f) stored by phase 2a,
               read back with its segment spectrum by phase 2b one step later (step groups: kept
               in registers, one workgroup doing both, far2c_role), 128 far-field
               entries; phase 1 takes K windows per pass over the nseg - 1 older row-pair and
               segment spectra (1/K per window), and 2b segments 1 .. j of window j of a group
               (K - 1 spectrum pairs per window on average): 256 (4 + 2 (nseg - 1) / K + K - 1)
               + 128 values per window, K = far_group(nseg, units) (upols_levels.hip); plus phase
               1's partial sums, 256 values per column and window written and read back by
               phase 2 (included in "far", also reported alone as "far_partial_sums").
               far_form 2 (recomputed every window, far2r_role): per column and window the
               (nseg + 1) 128 FDL rows of the segments' row pairs, the P - 256 filter rows of the
               band and the 128 field rows.
    Step groups (G > 1): the levels with T < 2 G run in the block's launch ("toeplitz_block"), the
    others in the background launches of G steps ("toeplitz")."""
    nlev = len(plan["T"]) + (1 if plan["nseg"] else 0)
    block = C * B * (16 + 16 + 16 * (plan["a0"] - 1) + 8 * nlev)
    lv = [(T, C * B / T * 8 * (2 * (b - a) + 2 * T - 1)) for T, a, b in zip(plan["T"], plan["a"], plan["b"])]
    toep = sum(v for T, v in lv if G == 1 or T >= 2 * G)
    toep_block = sum(v for T, v in lv if G > 1 and T < 2 * G)
    ns = plan["nseg"]
    K = far_group(ns, C * B // 16) if not far_k else far_k
    # step groups: phase 2 keeps the fresh spectrum in registers (far2c_role), 3 instead of 4
    fresh = 4 if G == 1 else 3
    far = C * B / 128 * 8 * (256 * (fresh + 2 * (ns - 1) / K + K - 1) + 128) if ns else 0.0
    # phase 1's partial sums: 256 values per column and window written by phase 1 and read back
    # by phase 2 (the two phases' hand-off; none in the recomputed form)
    partials = C * B / 128 * 8 * 2 * 256 if ns else 0.0
    if ns and far_form == 2:
        far = C * B / 128 * 8 * ((ns + 1) * 128 + (P - 256) + 128)
        partials = 0.0
    out = {"block": block, "toeplitz": toep, "far": far + partials, "far_partial_sums": partials}
    if G > 1:
        out["toeplitz_block"] = toep_block
    return out


def oracle_parity(x, y, feed, irh, B, chans, K=4, threads=16):
    """Peak-normalized error of the last K processed blocks of channels `chans` against the
    oracle's dense_convolve over their full input history (the P + 1 blocks before them: an
    output block depends on no older input, fdl_index.hpp:23-36)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O

    P = O.uniform_partition(irh[:1], B).shape[1]
    G = feed.g
    start = max(0, G - K - P - 1)
    idx = [g % feed.nx for g in range(start, G)]
    worst = 0.0
    for c in chans:
        xc = x[c].view(feed.nx, B)[idx].cpu().numpy().reshape(1, -1)
        yc = y[c].view(feed.nx, B)[idx[-K:]].cpu().numpy().reshape(-1)
        ref = O.dense_convolve(xc, O.uniform_partition(irh[c:c + 1], B), threads=threads)[0, -K * B:]
        worst = max(worst, float(np.abs(yc - ref).max() / np.abs(ref).max()))
    return worst


def spin_wait(local: int) -> None:
    """hipDeviceScheduleSpin on this process's device: a real-time caller waits for each
    block by spinning (HIP's auto mode yields on a host with more cores than contexts, which
    adds tens of microseconds of wake-up to every wait). torch's HIP runtime is already
    loaded, so the soname resolves to it."""
    import ctypes

    if os.environ.get("NEO_BENCH_SPIN", "1") != "1":
        return
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipSetDevice(ctypes.c_int(local))
    hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin


SHARD_OF = 1  # --shard-of


def rank_channels(workload: str, world: int, rank: int, strong: bool = None):
    """(channels of this rank, channels of the whole job): a strong workload's channels are
    split over the ranks (shard), the others are per GPU."""
    C, _, _ = WORKLOADS[workload]
    if strong is None:
        strong = workload in STRONG
    if strong and world == 1 and SHARD_OF > 1:  # --shard-of: one rank's share, measured alone
        lo, hi = shard(C, SHARD_OF, 0)
        return hi - lo, hi - lo
    if strong:
        lo, hi = shard(C, world, rank)
        return hi - lo, C
    return C, C * world


def host_io_times(conv, C, B, nblocks, kind, seed=0):
    """One synchronous neo_hip_upols_process call per block on a host buffer [C][B] (the
    plugin's processFrame pattern, DenseConvolution.cpp:62-74): kind "pageable" (numpy, the
    handle's mapped staging) or "pinned" (page-locked torch tensor, read and written in place
    by the step kernel). The caller's write of the next block into the buffer is not timed.
    Returns per-call seconds."""
    import numpy as np
    import torch

    src = np.random.default_rng(seed).random((C, B), dtype=np.float32) * 2 - 1
    if kind == "pinned":
        buf = torch.empty((C, B), dtype=torch.float32).pin_memory()
        arr = buf.numpy()
    else:
        arr = np.empty((C, B), np.float32)
        buf = arr
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < WARM_SECONDS:
        arr[:] = src
        conv(buf)
    dt = []
    for _ in range(nblocks):
        arr[:] = src
        t0 = time.perf_counter()
        conv(buf)
        dt.append(time.perf_counter() - t0)
    return dt


def group_frames(C, frames, B, L, mode=0):
    """tests/cpp/bench_group (C++, NEO_HIP_CONVOLVER_GROUPS): the plugin's processFrame over C
    single-channel convolvers of one owner-registered frame buffer (one launch per frame once
    coalesced), and the dense_convolve<Convolver> harness pattern (one shared scratch block: one
    launch and one host wait per channel-block). Host memory, PCIe-inclusive; None if the binary
    cannot be built here."""
    import subprocess

    cpp = os.path.join(REPO, "tests", "cpp")
    exe = os.path.join(cpp, "bin", "bench_group")
    try:
        subprocess.run(["make", "-s", "-C", cpp, "bin/bench_group"], check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe, str(C), str(frames), str(B), str(L), str(mode)], capture_output=True,
                           text=True, timeout=600)
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except (OSError, subprocess.SubprocessError, ValueError, IndexError) as e:
        return {"error": str(e)[:200]}
    d["note"] = ("tests/cpp/bench_group: per frame = C calls of upols_convolver::operator() on the owner's "
                 "registered frame buffer (DenseConvolution.cpp:62-74); shared_scratch = the "
                 "dense_convolve<Convolver> harness (DenseConvolution.hpp:56-67), per channel-block")
    return d


def plugin_frames(C, frames, B, L, latency):
    """tests/cpp/bench_plugin (C++): the plugin's own processing class, neo::Convolution
    (extra/plugin/src/dsp/Convolution.hpp:60-63,112): std::vector<split_upols_convolver>, one call
    per channel and block on the host's channel buffer, never grouped; normal mode (a launch and a
    host wait per call) or latency mode (a resident kernel per channel). Host memory,
    PCIe-inclusive; an error entry if the binary cannot be built here."""
    import subprocess

    cpp = os.path.join(REPO, "tests", "cpp")
    exe = os.path.join(cpp, "bin", "bench_plugin")
    try:
        subprocess.run(["make", "-s", "-C", cpp, "bin/bench_plugin"], check=True, capture_output=True, timeout=300)
        r = subprocess.run([exe, str(C), str(frames), str(B), str(L), "1" if latency else "0"], capture_output=True,
                           text=True, timeout=600)
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except (OSError, subprocess.SubprocessError, ValueError, IndexError) as e:
        return {"error": str(e)[:200]}
    d["note"] = ("tests/cpp/bench_plugin: per frame = C calls of split_upols_convolver::operator() in place on "
                 "the channel buffers (Convolution.hpp:60-63), back to back")
    return d


def host_io_summary(dt, C, B):
    import numpy as np

    a = np.array(dt)
    return {"msamples_s": C * B / a.mean() / 1e6, "mean_us": float(a.mean() * 1e6),
            "p50_us": float(np.percentile(a, 50) * 1e6), "p99_us": float(np.percentile(a, 99) * 1e6),
            "max_us": float(a.max() * 1e6), "blocks": int(a.size), "pcie_bytes_per_block": 2 * 4 * C * B}


def run_upols(args, world, rank, local):
    import numpy as np
    import torch
    import neo

    _, B, L = WORKLOADS[args.workload]
    C, C_total = rank_channels(args.workload, world, rank)
    local = device_for(local)
    spin_wait(local)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    P = neo.num_partitions(L, B)
    conv = neo.UpolsConvolver(C, B, P, device=local, options={"step_group": args.step_group,
                                                              "far_group": args.far_group,
                                                              "far_phase2": args.far_phase2,
                                                              "far_level": args.far_level})
    conv.set_batch(False)  # streaming: one block per step, as a real-time caller runs it
    levels = conv.ahead_info()[0] and not args.no_ahead
    conv_far_group = conv.far_group()
    conv_far_form = conv.far_form()
    G = conv.step_group()
    plan = neo.convolution.level_plan(P)
    g = torch.Generator(device=dev).manual_seed(8 + rank)
    ir = torch.rand((C, L), generator=g, device=dev).mul_(2).sub_(1)  # synthetic white-noise IR
    irh = ir.cpu().numpy() if (rank == 0 and not args.no_parity) else None
    conv.set_impulse(ir, normalize=True)
    del ir
    nx = P + 192  # cyclic input: covers the parity check's history window (P + 5 blocks)
    x = torch.rand((C, nx * B), generator=g, device=dev).mul_(2).sub_(1)
    y = torch.empty_like(x)
    # a stream of its own (not the null stream): the steps and the events around them
    sobj = torch.cuda.Stream(dev) if os.environ.get("NEO_BENCH_NULL_STREAM") != "1" else torch.cuda.current_stream(dev)
    stream = sobj.cuda_stream
    torch.cuda.synchronize(dev)  # x, y and the filter were made on the default stream
    feed = Feed(conv, x, y, nx, B, stream)

    def warm():
        t_warm = time.perf_counter()
        feed.run(max(args.warmup, 1))
        torch.cuda.synchronize()
        while time.perf_counter() - t_warm < WARM_SECONDS:  # untimed
            feed.run(64)
            torch.cuda.synchronize()
        # end the warm-up on a step-group boundary: a timed region then starts with its group's
        # background launch, as every group does in steady state (starting k calls into a group,
        # the region would open with k blocks and no background work beside them, then still
        # hold the same number of background launches)
        G_, ph = conv.step_group(), conv.ahead_info()[1]  # ph: the next step's position in its far window
        if G_ > 1 and ph % G_:
            feed.run(G_ - ph % G_)
            torch.cuda.synchronize()

    gpu_ms = {}

    def timed_region(tag):
        """args.steps single-block steps, nothing else in the timed region (wall clock); then
        the same number of steps again with HIP events on the launch stream around them: the
        GPU time per step (gpu_ms[tag]) and the host's enqueue time."""
        mark = os.environ.get("NEO_BENCH_MARK") == "1"  # diagnostic: marker kernels around the region in traces
        if mark:
            torch.zeros(1, device=dev).add_(1)
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        feed.run(args.steps)
        torch.cuda.synchronize()
        barrier(world)
        t1 = time.perf_counter()
        if mark:
            torch.zeros(1, device=dev).mul_(3)
        if os.environ.get("NEO_BENCH_NO_CHECK") != "1":  # role-masked diagnostic builds compute garbage
            assert torch.isfinite(y).all().item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        e0.record(sobj)
        feed.run(args.steps)
        conv.join_background(stream)  # step groups: the background slice launches issued by these steps
        e1.record(sobj)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        gpu_ms[tag] = max_over_ranks(e0.elapsed_time(e1) / args.steps, world)
        gpu_ms[tag + "_host_launch_ms"] = (t3 - t2) * 1e3
        gpu_ms[tag + "_per_rank_ms"] = [v * 1e3 / args.steps for v in gather_over_ranks(t1 - t0, world)]
        return max_over_ranks(t1 - t0, world)

    def wall_region(n):
        """n steps timed like the headline (barrier + sync on both sides, max over ranks): seconds"""
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        feed.run(n)
        torch.cuda.synchronize()
        barrier(world)
        return max_over_ranks(time.perf_counter() - t0, world)

    def instrumented():
        """max(steps, 64) more steps with HIP events the C-ABI records on the launch stream
        around every part of every step: the per-part kernel times."""
        conv.timing_detail()  # drain
        conv.set_timing(True, every=1)
        feed.run(max(args.steps, 64))
        torch.cuda.synchronize()
        conv.set_timing(False)
        det = [(ms / n if n else None) for ms, n in conv.timing_detail()]
        return [max_over_ranks(d, world) if d is not None else None for d in det]

    samples = C_total * B * args.steps  # all ranks
    # the plain single-block step: one pass over filter + FDL per block (k_upols_step)
    conv.set_ahead(False)
    warm()
    el_plain = timed_region("plain")
    det_plain = instrumented()
    bytes_plain = C * (16 * P * B + 20 * B)  # filter + FDL stream (packed bins) + FDL row write + in/prev
    gbs_plain = bytes_plain / (det_plain[0] * 1e-3) / 1e9
    plain = {"value": samples / el_plain / 1e6, "ms_per_step": el_plain * 1e3 / args.steps,
             "kernel": f"k_upols_step<{B}>", "kernel_avg_ms": det_plain[0], "algorithmic_bytes_per_launch": bytes_plain,
             "achieved_gbs": gbs_plain, "frac": gbs_plain / PEAK_HBM_GBS,
             "traffic": load_pmc_traffic(_pmc_sfx(pmc_workload(args.workload, C), "_plain"), "k_upols_step")}
    if levels:
        conv.set_ahead(True)
    warm()
    elapsed = timed_region("levels")
    parity = None
    if irh is not None:
        irn = None
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O

        irn = O.normalize_impulse(irh)
        # 16 channels spread over the shard (first and last included), every one of them a different
        # IR, against the oracle over its input history
        pch = sorted({0, C - 1} | {(C * i) // 16 + i % 7 for i in range(16) if (C * i) // 16 + i % 7 < C})
        parity = {"parity_err": oracle_parity(x, y, feed, irn, B, pch, threads=args.cpu_threads),
                  "channels": pch, "blocks": 4,
                  "what": "last 4 blocks of the timed region vs oracle dense_convolve over their input history "
                          "(peak-normalized; bar 1e-5)"}
    det = instrumented()
    # the real-time caller's round trip: one call per block, the host waits for that block's
    # output (stream sync, spinning) before the next call
    rt = []
    for _ in range(200):
        t0 = time.perf_counter()
        feed.run(1)
        sobj.synchronize()
        rt.append(time.perf_counter() - t0)
    rt = np.array(rt)
    rt_p50 = max_over_ranks(float(np.percentile(rt, 50)) * 1e6, world)
    rt_p99 = max_over_ranks(float(np.percentile(rt, 99)) * 1e6, world)
    rt_mean = max_over_ranks(float(rt.mean()) * 1e6, world)
    # per-step latency: every step of a separate 256-step run bracketed by events (GPU time of the
    # step, first to last event), the distribution a per-block real-time caller sees
    conv.step_times()
    conv.set_timing(True, every=1)
    feed.run(256)
    torch.cuda.synchronize()
    conv.set_timing(False)
    st = np.array(conv.step_times())
    paced = paced2 = None
    if levels and G > 1 and not args.no_paced:
        # the same round trip with the background work paced (neo_hip_upols_set_paced: the group's
        # launch in pieces, each block that issues one after the piece before it): even calls.
        # mode 1: a piece per call; mode 2: two pieces per group
        def paced_run(mode):
            conv.set_paced(mode)
            warm()
            prt = []
            for _ in range(200):
                t0 = time.perf_counter()
                feed.run(1)
                sobj.synchronize()
                prt.append(time.perf_counter() - t0)
            prt = np.array(prt) * 1e6
            el_p = wall_region(args.steps)
            conv.set_paced(0)
            warm()
            return {"host_roundtrip_p50_us": max_over_ranks(float(np.percentile(prt, 50)), world),
                    "host_roundtrip_p99_us": max_over_ranks(float(np.percentile(prt, 99)), world),
                    "host_roundtrip_mean_us": max_over_ranks(float(prt.mean()), world),
                    "value": samples / el_p / 1e6, "ms_per_step": el_p * 1e3 / args.steps,
                    "note": f"neo_hip_upols_set_paced({mode}): round trip as above; value = the timed steps back "
                            "to back"}
        paced = paced_run(1)
        paced2 = paced_run(2)
    # the same round trip at a real-time cadence (default mode, no pacing): calls issued on a fixed
    # clock instead of back to back -- the audio clock of a B-sample block at 48 kHz, and a period
    # 1.25 x the timed step (the GPU 80 % loaded); a call that overruns its period starts the next
    # one late, counted in "overruns"
    def cadence_run(period, n):
        crt = []
        nxt = time.perf_counter()
        over = 0
        for _ in range(n):
            while time.perf_counter() < nxt:
                pass
            t0 = time.perf_counter()
            feed.run(1)
            sobj.synchronize()
            d = time.perf_counter() - t0
            crt.append(d)
            over += d > period
            nxt = max(nxt + period, t0 + d)
        crt = np.array(crt) * 1e6
        return {"period_us": period * 1e6, "calls": n,
                "host_roundtrip_p50_us": max_over_ranks(float(np.percentile(crt, 50)), world),
                "host_roundtrip_p99_us": max_over_ranks(float(np.percentile(crt, 99)), world),
                "host_roundtrip_max_us": max_over_ranks(float(crt.max()), world),
                "overruns": int(max_over_ranks(float(over), world))}
    cadence = None
    if not args.no_paced:
        warm()
        cadence = {"audio_48k": cadence_run(B / 48000.0, 200), "load_80pct": cadence_run(1.25 * elapsed / args.steps, 400),
                   "note": "default mode (no pacing): one call per period on the host's clock, each followed by a "
                           "host wait for its output; audio_48k = a B-sample block's period at 48 kHz, load_80pct = "
                           "1.25 x the headline's ms_per_step"}
    # steady state: one whole far window (128 steps = 32 step groups: every group's background
    # launch once, whatever their sizes), timed like the headline
    n_steady = 128
    el_steady = wall_region(n_steady)
    latency = {"steps": int(st.size), "mean_ms": float(st.mean()), "p50_ms": float(np.percentile(st, 50)),
               "p99_ms": float(np.percentile(st, 99)), "max_ms": float(st.max()),
               "max_over_mean": float(st.max() / st.mean()),
               "host_roundtrip_p50_us": rt_p50, "host_roundtrip_p99_us": rt_p99, "host_roundtrip_mean_us": rt_mean,
               "host_roundtrip_msamples_s": C_total * B / rt_mean, "paced": paced, "paced_two_pieces": paced2,
               "cadence": cadence,
               "note":"p50/p99/max: GPU time per step (HIP events around every step, which add their own records); "
                       "host_roundtrip: 200 device-resident single-block calls, each followed by a host wait for its "
                       "output before the next call (max over ranks)"}

    if levels and G == 1:
        roles = algorithmic_bytes(C, B, P, plan, 1, conv_far_group, conv_far_form)
        # one launch per step: HIP events around a second run of the timed steps, or the wall
        # time of the timed steps where that is smaller (with timing events on it the stream's
        # launches slow down; at one channel the event run is host-bound)
        step_ms = min(gpu_ms["levels"], elapsed * 1e3 / args.steps)
        by = sum(v for k, v in roles.items() if k != "far_partial_sums")
        gbs = by / (step_ms * 1e-3) / 1e9
        name = f"k_lvl_step<{B}>"
        kernels = [{"kernel": name + " (block, Toeplitz T = %s, far %d segments)"
                    % ("/".join(map(str, plan["T"])), plan["nseg"]),
                    "ms_per_step": step_ms, "share_of_step": 1.0, "algorithmic_bytes_per_step": by,
                    "bytes_by_role": roles, "achieved_gbs": gbs, "frac": gbs / PEAK_HBM_GBS,
                    "traffic": load_pmc_traffic(pmc_workload(args.workload, C), "k_lvl_step")}]
        dom = kernels[0]
        roof = {"bound": "hbm", "achieved": dom["achieved_gbs"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": dom["frac"], "traffic": dom["traffic"],
                "traffic_over_algorithmic": dom["traffic"] / by if dom["traffic"] else None, "kernel": name,
                "kernel_avg_ms": step_ms, "steps_per_launch": 1, "launches_per_step": 1,
                "timing": "min(HIP events on the launch stream around a second run of the timed steps, wall time "
                          "of the timed steps) per step, one launch per step; with events around every step: "
                          "%.4f ms" % det[0],
                "algorithmic_bytes_per_launch": by,
                "kernels": kernels, "d2d_copy_gbs": copy_ceiling_gbs(dev)}
    elif levels:
        # step groups: the block launch of every step on the caller's stream and one background
        # launch of the level slices per G steps, overlapping; per-kernel HIP events (the C-ABI's
        # timing parts 0 / 1, on the stream each kernel runs on) give each kernel's launch time,
        # the wall time of the timed steps the whole step's
        roles = algorithmic_bytes(C, B, P, plan, G, conv_far_group, conv_far_form)
        by_blk = roles["block"] + roles["toeplitz_block"]
        by_sl = G * (roles["toeplitz"] + roles["far"])
        by = by_blk + by_sl / G
        kb, ks = f"k_lvl_block<{B}>", f"k_lvl_slices<{1 if conv_far_form == 2 else (2 if conv_far_group <= 2 else 4)}>"
        kernels = []
        for kname, b, ms, per in ((ks, by_sl, det[1], G), (kb, by_blk, det[0], 1)):
            g = b / (ms * 1e-3) / 1e9
            kernels.append({"kernel": kname, "ms_per_launch": ms, "launches_per_step": 1.0 / per,
                            "algorithmic_bytes_per_launch": b, "achieved_gbs_alone": g,
                            "traffic": load_pmc_traffic(_pmc_sfx(pmc_workload(args.workload, C), "_" + kname.split('<')[0]), kname.split("<")[0]),
                            "note": "launch time measured while the other kernel runs beside it (shared HBM), so "
                                    "bytes / launch time understates the kernel; the step pair is the roofline unit"})
        kernels[0]["bytes_by_role"] = {"toeplitz": G * roles["toeplitz"], "far": G * roles["far"]}
        kernels[1]["bytes_by_role"] = {"block": roles["block"], "toeplitz": roles["toeplitz_block"]}
        # the roofline unit is the step: G block launches and one slice launch per G steps run side
        # by side on two streams, so the dominant "kernel" is that pair; its GPU time per step is the
        # HIP-event time on the launch stream around a second run of the timed steps with the
        # background launches joined onto it (neo_hip_upols_join_background), or the wall time of
        # the timed steps where that is smaller
        step_ms = min(gpu_ms["levels"], elapsed * 1e3 / args.steps)
        gbs = by / (step_ms * 1e-3) / 1e9
        tr = [k["traffic"] for k in kernels]
        traffic = tr[0] / G + tr[1] if all(tr) else None
        roof = {"bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": gbs / PEAK_HBM_GBS, "traffic": traffic,
                "traffic_over_algorithmic": traffic / by if traffic else None,
                "kernel": f"{kb} x{G} + {ks} x1 (one step group, two streams, overlapped)",
                "kernel_avg_ms": step_ms, "steps_per_launch": 1, "step_group": G,
                "timing": "GPU time per step: min(HIP events on the launch stream around a second run of the timed "
                          "steps, background slice launches joined onto that stream before the closing event; "
                          "wall time of the timed steps); per-kernel launch times in kernels[] (events around "
                          "every launch, each on its own stream)",
                "algorithmic_bytes_per_launch": by, "bytes_by_role": roles, "kernels": kernels,
                "d2d_copy_gbs": copy_ceiling_gbs(dev)}
    else:
        roof = {"bound": "hbm", "achieved": gbs_plain, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": gbs_plain / PEAK_HBM_GBS, "traffic": plain["traffic"], "kernel": plain["kernel"],
                "kernel_avg_ms": det_plain[0], "steps_per_launch": 1, "algorithmic_bytes_per_launch": bytes_plain,
                "d2d_copy_gbs": copy_ceiling_gbs(dev)}
    step_bytes = roof["algorithmic_bytes_per_launch"]
    steady = {"steps": n_steady, "value": C_total * B * n_steady / el_steady / 1e6, "unit": "Msamples/s",
              "ms_per_step": el_steady * 1e3 / n_steady,
              "achieved": step_bytes / (el_steady / n_steady) / 1e9, "unit_achieved": "GB/s",
              "frac": step_bytes / (el_steady / n_steady) / 1e9 / PEAK_HBM_GBS,
              "value_over_headline": (args.steps / elapsed) / (n_steady / el_steady),
              "note": "one whole far window (128 steps, every step group's background launch once), wall clock "
                      "with barrier + sync on both sides like the headline; frac on the headline's bytes per step"}
    ir_change = None
    if levels:
        # IR change (DenseConvolution.cpp:78-108: normalize_impulse + uniform_partition + filter per
        # channel): set_impulse on a device-resident IR, then the first block after it, which
        # primes the levels (far segment spectra and window 0 of every level)
        g2 = torch.Generator(device=dev).manual_seed(1008 + rank)
        ir2 = torch.rand((C, L), generator=g2, device=dev).mul_(2).sub_(1)
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        conv.set_impulse(ir2, normalize=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        feed.run(1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        del ir2
        ir_change = {"set_impulse_ms": max_over_ranks((t1 - t0) * 1e3, world),
                     "first_block_ms": max_over_ranks((t2 - t1) * 1e3, world),
                     "total_ms": max_over_ranks((t2 - t0) * 1e3, world),
                     "note": "device-resident IR [C][L]: normalize (sequential-float energy, min over channels), "
                             "partition r2c, then the first streaming block (far segment spectra + level priming); "
                             "max over ranks"}
    latency_mode = run_latency_mode(args, conv, feed, C, B, world, C_total)
    offline = run_upols_offline(args, conv, C, B, P, x, y, nx * B, stream, world, C_total)
    host_io = None
    if not args.no_host_io:
        conv.set_batch(False)
        host_io = {"note": "neo_hip_upols_process on a host buffer, one synchronous call per block through the "
                           "Python binding (PCIe-inclusive; never the headline value)"}
        for kind in ("pinned", "pageable"):
            host_io[f"{args.workload}_{kind}"] = host_io_summary(host_io_times(conv, C, B, 200, kind), C, B)
    del x, y, feed
    if host_io is not None and args.workload == "c5full" and world == 1:
        # the 8-GPU split's per-GPU shard (256 channels) as its own handle
        cs = WORKLOADS["c5"][0]
        c5 = neo.UpolsConvolver(cs, B, P, device=local)
        g5 = torch.Generator(device=dev).manual_seed(99)
        c5.set_impulse(torch.rand((cs, L), generator=g5, device=dev).mul_(2).sub_(1), normalize=True)
        c5.set_batch(False)
        for kind in ("pinned", "pageable"):
            host_io[f"c5_{kind}"] = host_io_summary(host_io_times(c5, cs, B, 200, kind), cs, B)
        c5.close()
        del c5
        torch.cuda.empty_cache()
        # the plugin's std::vector<upols_convolver> (group-backed alias, C++) at 256 and 2048 channels
        # (frame buffer registered plainly: exact snapshot comparison per member; with the owner's
        # frame-stable promise, NEO_HIP_GROUP_FRAME_STABLE: no snapshot, no comparison; in place,
        # NEO_HIP_GROUP_FRAME_INPLACE: every output written into the frame by its first call)
        for cs_, nf_ in ((256, 64), (2048, 32)):
            for sfx, mode in (("", 0), ("_stable", 1), ("_inplace", 2)):
                host_io[f"group_{cs_}{sfx}"] = group_frames(cs_, nf_, B, L, mode)
        # the plugin's processing class (stereo split_upols_convolver, 10 s IR), both modes
        for lat in (False, True):
            host_io["plugin_stereo" + ("_latency" if lat else "")] = plugin_frames(2, 400, B, L, lat)
    weak = None
    if world > 1 and args.workload in STRONG and not args.no_weak:
        conv.close()
        del conv
        weak = run_weak(args, world, rank, local, B, L)
    res = {
        "metric": "Msamples/sec UPOLS convolver (block=512, IR=10s@48k); achieved HBM GB/s",
        "value": samples / elapsed / 1e6,
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "gpu_ms_per_step": gpu_ms.get("levels" if levels else "plain"),  # HIP events around the same steps
        "host_launch_ms": gpu_ms.get(("levels" if levels else "plain") + "_host_launch_ms"),  # t0 -> all steps enqueued
        "per_rank_ms": gpu_ms.get(("levels" if levels else "plain") + "_per_rank_ms"),  # each rank's wall ms per step
        "higher_is_better": True,
        "scaling": "strong" if args.workload in STRONG else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (U[-1,1) white-noise input and IR, torch.rand on device)",
        "config": {"workload": f"UPOLS {args.workload}: {C_total} channels in all, {C} on rank 0 of {world} GPU(s) "
                               f"({'split over the ranks' if args.workload in STRONG else 'per GPU'}), B={B}, "
                               f"L={L} taps (P={P}), one block per step",
                   "channels_per_gpu": C, "channels_total": C_total, "shard_of": SHARD_OF, "block": B, "taps": L, "partitions": P,
                   "far_group": conv_far_group, "step_group": G,
                   "far_form": {0: "none", 1: "transform, stored spectra", 2: "transform recomputed every window",
                                3: "128-block Toeplitz"}[conv_far_form],
                   "streaming": ("levels: block step p<%d, Toeplitz %s, far %d segments" %
                                 (plan["a0"], list(zip(plan["T"], plan["a"], plan["b"])), plan["nseg"])
                                 if levels else "plain step"),
                   "parallelism": f"channel-shard x{world} (no collective)"},
        "roofline": roof,
        "steady": steady,
        "ir_change": ir_change,
        "latency_mode": latency_mode,
        "latency": latency,
        "parity": parity,
        "per_block_step": plain,
        "offline": offline,
        "host_io": host_io,
    }
    if weak is not None:
        res["weak"] = weak
    if args.workload == "c3":
        res["roofline"]["note"] = "working set L2/MALL-resident: effective GB/s, launch-latency bound"
    return res


def run_latency_mode(args, conv, feed, C, B, world, C_total):
    """The latency mode (neo_hip_upols_set_persistent: one persistent kernel steps every block,
    each call synchronous) on the same convolver and input, for the shapes it takes (C3): the
    host round trip per block (one call, complete on return), the same number of steps as the
    headline back to back (wall clock), and the GPU time per step (record read -> done, on the
    GPU clock). available False where the shape is not latency-bound (the handle refuses it).
    Without the streaming levels (ref4096) it is the plain step's persistent kernel."""
    import numpy as np

    try:
        conv.set_persistent(True)
    except RuntimeError as e:
        return {"available": False, "reason": str(e).split(": ", 1)[-1]}
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < WARM_SECONDS:
        feed.run(16)  # synchronous calls: no device sync while the persistent kernel is resident
    rt = []
    for _ in range(400):
        t0 = time.perf_counter()
        feed.run(1)
        rt.append(time.perf_counter() - t0)
    st = np.array(conv.persist_step_times())
    barrier(world)
    t0 = time.perf_counter()
    feed.run(args.steps)
    el = max_over_ranks(time.perf_counter() - t0, world)
    info = conv.persistent_info()
    conv.set_persistent(False)
    rt = np.array(rt) * 1e6
    return {"available": True, "value": C_total * B * args.steps / el / 1e6, "unit": "Msamples/s",
            "ms_per_step": el * 1e3 / args.steps,
            "host_roundtrip_p50_us": max_over_ranks(float(np.percentile(rt, 50)), world),
            "host_roundtrip_p99_us": max_over_ranks(float(np.percentile(rt, 99)), world),
            "host_roundtrip_mean_us": max_over_ranks(float(rt.mean()), world),
            "gpu_step_p50_us": float(np.percentile(st, 50)) if st.size else None,
            "gpu_step_p99_us": float(np.percentile(st, 99)) if st.size else None,
            "gpu_steps_sampled": int(st.size), "persistent_launches": info["launches"],
            "note": "neo_hip_upols_set_persistent: round trip = one synchronous call per block (device-resident "
                    "blocks), 400 calls; value = --steps calls back to back (pipelined records, wall clock); "
                    "gpu_step = record read -> completion signal on the GPU clock (last 63 steps)"}


def run_upols_offline(args, conv, C, B, P, x, y, ld, stream, world, C_total):
    """Same convolver and input, blocks available up front (dense_convolve / process_blocks;
    the reference's offline harness, extra/plugin/src/dsp/DenseConvolution.hpp:39-70 run by
    extra/plugin/src/ui/BenchmarkTab.hpp:47-66). Not the headline (which is the real-time
    one-block-per-call step); reported beside it. 256 blocks per timed call: with offline windows
    (>= 128 partitions) ONE pass of two 128-block windows (k_off_mac: partition-axis transforms of
    every 128-partition segment), else 8 T-block MAC passes (k_batch_mac)."""
    import torch

    if args.no_offline:
        return None
    conv.set_batch(True)
    T, splits = conv.batch_info()
    off, nseg = conv.offline_info()
    nb = min(256, ld // B)  # the input buffer's blocks (ref4096: P + 192 = 224)
    off = off and nb >= 128
    conv.reset()
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < WARM_SECONDS:
        conv.process_blocks_ptr(x.data_ptr(), y.data_ptr(), ld, nb, stream)
        torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    conv.timing()
    conv.set_timing(True)
    t0 = time.perf_counter()
    conv.process_blocks_ptr(x.data_ptr(), y.data_ptr(), ld, nb, stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    conv.set_timing(False)
    mac_ms, launches = conv.timing()
    conv.set_batch(False)
    elapsed = max_over_ranks(t1 - t0, world)
    mac_avg_ms = max_over_ranks(mac_ms / max(launches, 1), world)
    if off:
        wp = 2 if nb >= 256 else 1
        # per column and pass: (nseg + wp) 128 FDL rows, nseg 256-row segment spectra, wp 128 output rows
        bytes_pass = C * B * 8 * ((nseg + wp) * 128 + nseg * 256 + wp * 128)
        kernel, per_pass, pmc = f"k_off_mac<{wp}>", wp * 128, "k_off_mac"
    else:
        bytes_pass = C * 16 * P * B  # filter + FDL streamed once per pass of T blocks
        kernel, per_pass, pmc = f"k_batch_mac<{B},{T},1>", T, "k_batch_mac"
    gbs = bytes_pass / (mac_avg_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic(_pmc_sfx(pmc_workload(args.workload, C), "_offline"), pmc)
    return {"value": C_total * B * nb / elapsed / 1e6, "unit": "Msamples/s", "blocks": nb, "blocks_per_pass": per_pass,
            "offline_windows": off, "segments": nseg if off else None,
            "traffic": traffic, "traffic_over_algorithmic": traffic / bytes_pass if traffic else None,
            "ms_per_block": elapsed * 1e3 / nb, "splits": None if off else splits, "kernel": kernel,
            "algorithmic_bytes_per_launch": bytes_pass, "kernel_avg_ms": mac_avg_ms,
            "achieved_gbs": gbs, "frac": gbs / PEAK_HBM_GBS}


def run_weak(args, world, rank, local, B, L):
    """The secondary weak-scaling line: 2048 channels per GPU (N x 2048 in all), the same
    streaming steps, timed like the headline (barrier + sync around args.steps calls)."""
    import torch
    import neo

    C = WORKLOADS[args.workload][0]
    dev = torch.device("cuda", local)
    P = neo.num_partitions(L, B)
    conv = neo.UpolsConvolver(C, B, P, device=local)
    conv.set_batch(False)
    g = torch.Generator(device=dev).manual_seed(18 + rank)
    conv.set_impulse(torch.rand((C, L), generator=g, device=dev).mul_(2).sub_(1), normalize=True)
    nx = 64
    x = torch.rand((C, nx * B), generator=g, device=dev).mul_(2).sub_(1)
    sobj = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    feed = Feed(conv, x, x, nx, B, sobj.cuda_stream)
    t_warm = time.perf_counter()
    feed.run(max(args.warmup, 1))
    torch.cuda.synchronize()
    while time.perf_counter() - t_warm < WARM_SECONDS:
        feed.run(64)
        torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    feed.run(args.steps)
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world)
    conv.close()
    return {"value": world * C * B * args.steps / el / 1e6, "unit": "Msamples/s", "scaling": "weak",
            "ms_per_step": el * 1e3 / args.steps, "channels_per_gpu": C, "channels_total": C * world,
            "note": "secondary: 2048 channels per GPU (not a BASELINE config), the headline's streaming step"}


def run_upols_host_io(args, world, rank, local):
    """Host-buffer boundary: every block is copied host->device, processed and copied back
    (the plugin's processFrame pattern, DenseConvolution.cpp:62-74)."""
    import numpy as np
    import torch
    import neo

    _, B, L = WORKLOADS[args.workload]
    C, C_total = rank_channels(args.workload, world, rank)
    local = device_for(local)
    spin_wait(local)
    torch.cuda.set_device(local)
    P = neo.num_partitions(L, B)
    conv = neo.UpolsConvolver(C, B, P, device=local)
    g = torch.Generator(device="cuda").manual_seed(8 + rank)
    conv.set_impulse(torch.rand((C, L), generator=g, device="cuda").mul_(2).sub_(1), normalize=True)
    out = {}
    for kind in ("pinned", "pageable"):
        barrier(world)
        dt = host_io_times(conv, C, B, args.steps, kind, seed=rank)
        barrier(world)
        out[kind] = host_io_summary(dt, C, B)
    el = max_over_ranks(sum(host_io_times(conv, C, B, args.steps, "pinned", seed=rank)), world)
    return {"metric": "Msamples/sec UPOLS convolver, host buffers (PCIe-inclusive, not the headline)",
            "value": C_total * B * args.steps / el / 1e6, "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "ms_per_step": el * 1e3 / args.steps, "host_io": out,
            "config": {"workload": f"UPOLS {args.workload} host io (pinned buffer; pageable in host_io)",
                       "bytes_per_step_pcie": 2 * 4 * C * B}}


def run_fft(args, world, rank, local):
    import torch
    import neo

    local = device_for(local)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    N, batch = 4096, 65536
    g = torch.Generator(device=dev).manual_seed(2 + rank)
    x = torch.view_as_complex(torch.rand((batch, N, 2), generator=g, device=dev).mul_(2).sub_(1))
    y = torch.empty_like(x)
    plan = neo.fft.FFTPlan(0, 12, batch, device=local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    t_warm = time.perf_counter()
    for _ in range(args.warmup):
        plan.execute_device(x.data_ptr(), y.data_ptr(), -1, stream)
    torch.cuda.synchronize()
    while time.perf_counter() - t_warm < WARM_SECONDS:  # untimed clock-ramp warm-up
        plan.execute_device(x.data_ptr(), y.data_ptr(), -1, stream)
        torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    # kernel time: two events around the K back-to-back launches (the plan issues one
    # kernel per transform batch, so this is the kernel's average launch duration)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for i in range(args.steps):
        plan.execute_device(x.data_ptr(), y.data_ptr(), -1, stream)
    e1.record()
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    kms = e0.elapsed_time(e1) / args.steps
    elapsed = max_over_ranks(t1 - t0, world)
    kms = max_over_ranks(kms, world)
    bytes_launch = 16 * N * batch
    achieved = bytes_launch / (kms * 1e-3) / 1e9
    return {
        "metric": "Msamples/sec batched c2c FFT 4096 x 65536 (complex points per transform)",
        "value": world * N * batch * args.steps / elapsed / 1e6,
        "unit": "Msamples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (U[-1,1) complex, torch.rand on device)",
        "config": {"workload": "C2 batched c2c FFT, N=4096, batch 65536 per GPU, out of place",
                   "parallelism": f"batch-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": load_pmc_traffic("c2"),
                     "kernel": "k_c2c_lds<4096,-1>", "kernel_avg_ms": kms, "algorithmic_bytes_per_launch": bytes_launch,
                     "d2d_copy_gbs": copy_ceiling_gbs(dev)},
    }


def main():
    args = parse()
    if args.cpu_threads <= 0:
        args.cpu_threads = cpu_threads()
    world, rank, local = dist_setup(args)
    global SHARD_OF
    SHARD_OF = args.shard_of if world == 1 else 1
    if args.workload == "c2":
        res = run_fft(args, world, rank, local)
    elif args.host_io:
        res = run_upols_host_io(args, world, rank, local)
        args.no_cpu_baseline = True
    else:
        res = run_upols(args, world, rank, local)
        if not args.no_fft:
            import argparse as _ap

            f = run_fft(_ap.Namespace(steps=20, warmup=5), world, rank, local)
            res["c2_fft"] = {"value": f["value"], "unit": f["unit"], "ms_per_step": f["ms_per_step"],
                             "metric": f["metric"], "roofline": f["roofline"]}
    if rank == 0:
        if not args.no_cpu_baseline:  # rank 0, after every timed region (N > 1 too: the other ranks wait)
            C, B, L = WORKLOADS.get(args.workload, (0, 0, 0))
            res["cpu_baseline"] = (cpu_baseline_fft(args.cpu_threads) if args.workload == "c2"
                                   else cpu_baseline_upols(C, B, L, args.cpu_threads))
            try:
                import platform

                model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")]
                res["cpu_baseline"]["host_cpu"] = (model[0] if model else platform.processor())
                res["cpu_baseline"]["host_cpus_visible"] = os.cpu_count()
            except OSError:
                pass
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
