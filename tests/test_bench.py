"""bench.py's host-side accounting (no GPU): the algorithmic bytes per streaming step by role
 counted independently from the level plan, and the workload / shard layout the
driver's runs use."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402

PLAN = {"a0": 8, "T": [4, 8, 16, 32], "a": [8, 16, 32, 64], "b": [16, 32, 64, 256]}


def count_step_bytes(C, B, P, nseg, G, K, form):
    """rows of 8 B per bin and channel, per step, role by role (independent restatement)"""
    row = 8 * B * C  # one spectrum row of every channel
    block = (2 * 4 * B * C) + (2 * 4 * B * C) + 2 * row + 2 * 7 * row + (len(PLAN["T"]) + 1) * row
    lv = {}
    for T, a, b in zip(PLAN["T"], PLAN["a"], PLAN["b"]):
        filt, fdl, slab = b - a, b - a + T - 1, T  # per window and column
        lv[T] = (filt + fdl + slab) * row / T
    if form == 2:
        far = ((nseg + 1) * 128 + (P - 256) + 128) * row / 128
    else:
        fresh = 4 if G == 1 else 3
        far = (256 * (fresh + 2 * (nseg - 1) / K + K - 1) + 128) * row / 128
        far += 2 * 256 * row / 128  # phase 1's partial sums: written, read back by phase 2
    return block, lv, far


@pytest.mark.parametrize("C,B,P,nseg,G,K,form", [(256, 512, 938, 6, 4, 2, 1), (2048, 512, 938, 6, 4, 3, 1),
                                                 (256, 256, 1875, 13, 4, 2, 1), (4, 512, 938, 6, 1, 2, 1),
                                                 (256, 512, 938, 6, 4, 1, 2)])
def test_algorithmic_bytes_by_role(C, B, P, nseg, G, K, form):
    plan = dict(PLAN, nseg=nseg)
    got = bench.algorithmic_bytes(C, B, P, plan, G, K, form)
    block, lv, far = count_step_bytes(C, B, P, nseg, G, K, form)
    assert got["block"] == pytest.approx(block)
    assert got["far"] == pytest.approx(far)
    bg = sum(v for T, v in lv.items() if G == 1 or T >= 2 * G)
    assert got["toeplitz"] == pytest.approx(bg)
    if G > 1:
        assert got["toeplitz_block"] == pytest.approx(sum(v for T, v in lv.items() if T < 2 * G))
    else:
        assert "toeplitz_block" not in got


def test_headline_byte_totals():
    """the per-step totals DESIGN.md quotes, far partial sums included: c5full 639.2 MB (K = 3), the
    C5 shard 81.3 MB, C4 48.0 MB (605.6 / 77.1 / 45.9 without them, round 3's count)"""
    def tot(*a):
        r = bench.algorithmic_bytes(*a)
        return sum(v for k, v in r.items() if k != "far_partial_sums") / 1e6, r["far_partial_sums"] / 1e6
    for args, full, partials in (((2048, 512, 938, dict(PLAN, nseg=6), 4, 3, 1), 639.2, 33.6),
                                 ((256, 512, 938, dict(PLAN, nseg=6), 4, 2, 1), 81.3, 4.2),
                                 ((256, 256, 1875, dict(PLAN, nseg=13), 4, 2, 1), 48.0, 2.1)):
        t, p = tot(*args)
        assert t == pytest.approx(full, abs=0.05) and p == pytest.approx(partials, abs=0.05)
        assert t - p == pytest.approx({639.2: 605.6, 81.3: 77.1, 48.0: 45.9}[full], abs=0.05)


def test_far_group_rule():
    """bench.far_group restates upols_levels.hip far_group_auto: 2 below 16384 16-column units,
    round(sqrt(2 (nseg - 1))) in [2, 4] from there, 1 without two segments"""
    assert bench.far_group(6, 256 * 32) == 2
    assert bench.far_group(6, 512 * 32) == 3  # the 4-GPU shard of the headline
    assert bench.far_group(6, 2048 * 32) == 3
    assert bench.far_group(13, 2048 * 32) == 4
    assert bench.far_group(1, 2048 * 32) == 1
    assert bench.far_group(13, 256 * 16) == 2


def test_workloads_match_baseline_configs():
    """configs[2..4] of BASELINE.json: the bench's workload shapes"""
    assert bench.WORKLOADS["c5full"] == (2048, 512, 480000)
    assert bench.WORKLOADS["c5"] == (256, 512, 480000)
    assert bench.WORKLOADS["c4"] == (256, 256, 480000)
    assert bench.WORKLOADS["c3"] == (1, 512, 96000)
    assert bench.STRONG == {"c5full"}


def test_pmc_summary_follows_rank_shape():
    """The PMC traffic a rank reports is the summary of its own shape: a strong-scaled c5full
    rank at N = 8 runs c5's 256 channels, at N = 2 / 4 no summary of its shape exists."""
    for world, want in ((1, "c5full"), (2, None), (4, None), (8, "c5")):
        C, total = bench.rank_channels("c5full", world, 0)
        assert total == 2048 and C == 2048 // world
        assert bench.pmc_workload("c5full", C) == want
    assert bench.pmc_workload("c4", 256) == "c4"
    assert bench.pmc_workload("c5", 256) == "c5"
    assert bench.pmc_workload("c2", 0) == "c2"
    assert bench.load_pmc_traffic(None) is None
    assert bench._pmc_sfx(None, "_plain") is None and bench._pmc_sfx("c5", "_plain") == "c5_plain"
