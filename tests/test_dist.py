"""world_size-2 gloo tests (CPU) of the multi-GPU path: bench.py's distributed
helpers (barrier, max over ranks) and the claim the sharding relies on — UPOLS
channels are independent, so a channel-sharded run equals the unsharded one
exactly (checked with the oracle's dense_convolve on each rank's shard)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    import bench
    import oracle as O
    import torch.distributed as dist

    try:
        w, r, _ = bench.dist_setup(None)
        assert (w, r) == (world, rank)
        bench.barrier(w)
        m = bench.max_over_ranks(float(rank + 1) * 0.5, w)
        # shard 6 channels over the ranks, B=128, 1500-tap IR, 9 blocks
        C, B, L, nb = 6, 128, 1500, 9
        lo, hi = bench.shard(C, w, r)
        ir = np.stack([O.noise(40 + c, L) for c in range(C)])
        parts = O.uniform_partition(O.normalize_impulse(ir), B)  # global normalization, then shard
        sig = np.stack([O.noise(50 + c, B * nb) for c in range(C)])
        out = O.dense_convolve(sig[lo:hi], parts[lo:hi])
        q.put((rank, m, lo, hi, out))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, "error", repr(e), None, None))


@pytest.mark.timeout(300)
def test_gloo_world2_shard_equals_unsharded():
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    import oracle as O

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    assert all(r[1] == 1.0 for r in res)  # max over ranks of {0.5, 1.0}
    res.sort()
    spans = [(r[2], r[3]) for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == 6 and spans[0][1] == spans[1][0]
    C, B, L, nb = 6, 128, 1500, 9
    ir = np.stack([O.noise(40 + c, L) for c in range(C)])
    parts = O.uniform_partition(O.normalize_impulse(ir), B)
    sig = np.stack([O.noise(50 + c, B * nb) for c in range(C)])
    full = O.dense_convolve(sig, parts)
    sharded = np.concatenate([r[4] for r in res])
    assert np.array_equal(full, sharded)


def test_shard_ranges():
    sys.path.insert(0, REPO)
    import bench

    for total in (1, 7, 256, 2048):
        for world in (1, 2, 4, 8):
            spans = [bench.shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_bench_strong_scaling_spans():
    """bench.py --gpus N runs configs[4] itself: 2048 channels IN ALL split over the ranks
    (N = 8: exactly the 256-channel shard per GPU, DenseConvolution.hpp:50-67 over the
    node), the other workloads per GPU."""
    sys.path.insert(0, REPO)
    import bench

    for world in (1, 2, 4, 8):
        per = [bench.rank_channels("c5full", world, r) for r in range(world)]
        assert all(tot == 2048 for _, tot in per)
        assert sum(c for c, _ in per) == 2048
        assert [c for c, _ in per] == [2048 // world] * world
    assert bench.rank_channels("c5full", 8, 7) == (256, 2048)
    assert bench.rank_channels("c5full", 2, 1) == (1024, 2048)
    assert bench.rank_channels("c5", 8, 3) == (256, 2048)  # per GPU: weak
    assert bench.rank_channels("c4", 2, 0) == (256, 512)
    # --shard-of N (one process): rank 0's share of an N-GPU strong run, measured alone
    try:
        for n in (2, 4, 8):
            bench.SHARD_OF = n
            assert bench.rank_channels("c5full", 1, 0) == (2048 // n, 2048 // n)
            assert bench.rank_channels("c5full", 2, 1) == (1024, 2048)  # never under torchrun
            assert bench.rank_channels("c4", 1, 0) == (256, 256)  # per-GPU workloads unchanged
    finally:
        bench.SHARD_OF = 1


def _bench_rank_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path[:0] = [REPO]
    import bench
    import torch.distributed as dist

    try:
        w, r, _ = bench.dist_setup(None)
        c, tot = bench.rank_channels("c5full", w, r)
        lo, hi = bench.shard(tot, w, r)
        m = bench.max_over_ranks(float(c), w)
        q.put((r, lo, hi, c, tot, m))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, "error", repr(e), None, None, None))


@pytest.mark.timeout(300)
def test_gloo_world8_strong_shards():
    """Eight gloo ranks (CPU) take bench.py's strong-scaling shards of the 2048 channels:
    contiguous, disjoint, covering [0, 2048), 256 each."""
    world, port = 8, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    assert [(r[1], r[2]) for r in res] == [(256 * i, 256 * (i + 1)) for i in range(8)]
    assert all(r[3] == 256 and r[4] == 2048 and r[5] == 256.0 for r in res)


def _hip_worker(rank, world, port, q, C, B, L, nb):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.path[:0] = [REPO, os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle")]
    import bench
    import neo
    import oracle as O
    import torch
    import torch.distributed as dist

    try:
        w, r, local = bench.dist_setup(None)
        lo, hi = bench.shard(C, w, r)
        dev = bench.device_for(local)
        ir = np.stack([O.noise(60 + c, L) for c in range(C)])
        irn = neo.normalize_impulse(ir, device=dev)  # one factor over all channels, then shard
        P = neo.num_partitions(L, B)
        conv = neo.UpolsConvolver(hi - lo, B, P, device=dev)
        conv.set_impulse(irn[lo:hi], normalize=False)
        conv.set_batch(False)  # streaming steps (levels from 64 partitions)
        sig = np.stack([O.noise(70 + c, B * nb) for c in range(C)])[lo:hi]
        t = torch.from_numpy(np.ascontiguousarray(sig)).to(f"cuda:{dev}")
        conv.process_blocks(t)
        torch.cuda.synchronize(dev)
        bench.barrier(w)
        q.put((rank, lo, hi, t.cpu().numpy()))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, "error", repr(e), None))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_gloo_world2_hip_shards_equal_unsharded():
    """Two gloo ranks (both on the box's device 0 when only one is visible) each run the HIP
    convolver on their bench.shard channel range, streaming steps through the level
    pipeline; the assembled output equals one unsharded HIP run bit for bit."""
    sys.path[:0] = [REPO, os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle")]
    C, B, L, nb = 5, 128, 128 * 300, 40
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hip_worker, args=(r, world, port, q, C, B, L, nb)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r
    res.sort(key=lambda r: r[0])
    sharded = np.concatenate([r[3] for r in res])
    import neo
    import oracle as O
    import torch

    ir = np.stack([O.noise(60 + c, L) for c in range(C)])
    conv = neo.UpolsConvolver(C, B, neo.num_partitions(L, B))
    conv.set_impulse(ir, normalize=True)
    conv.set_batch(False)
    t = torch.from_numpy(np.stack([O.noise(70 + c, B * nb) for c in range(C)])).cuda()
    conv.process_blocks(t)
    torch.cuda.synchronize()
    assert np.array_equal(sharded, t.cpu().numpy())
