"""Offline windows alone (k_off_mac): one handle at a workload's shape, 256 blocks per timed call
(two 128-block windows per pass), median of `--reps` calls, and the k_off_mac launch time from the
handle's HIP events. For same-box A/B of library builds (NEO_HIP_LIBRARY). Prints one JSON line."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neo-dsp_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5full")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--off", type=int, default=1)
    a = ap.parse_args()
    import torch

    import bench
    import neo

    C, B, L = bench.WORKLOADS[a.workload][:3]
    P = neo.num_partitions(L, B)
    conv = neo.UpolsConvolver(C, B, P)
    g = torch.Generator(device="cuda").manual_seed(5)
    conv.set_impulse(torch.rand((C, L), generator=g, device="cuda").mul_(2).sub_(1), normalize=True)
    conv.set_offline(bool(a.off))
    nb = 256
    x = torch.rand((C, nb * B), generator=g, device="cuda")
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    for _ in range(2):
        conv.process_blocks_ptr(x.data_ptr(), y.data_ptr(), nb * B, nb, s.cuda_stream)
    torch.cuda.synchronize()
    wall, mac = [], []
    for _ in range(a.reps):
        conv.timing()
        conv.set_timing(True)
        t0 = time.perf_counter()
        conv.process_blocks_ptr(x.data_ptr(), y.data_ptr(), nb * B, nb, s.cuda_stream)
        s.synchronize()
        wall.append(time.perf_counter() - t0)
        conv.set_timing(False)
        ms, n = conv.timing()
        mac.append(ms / max(n, 1))
    wall.sort()
    mac.sort()
    off, nseg = conv.offline_info()
    print(json.dumps({"workload": a.workload, "offline": off, "segments": nseg, "blocks": nb,
                      "msamples_s": C * B * nb / wall[len(wall) // 2] / 1e6, "ms_per_call": wall[len(wall) // 2] * 1e3,
                      "mac_ms": mac[len(mac) // 2], "lib": os.environ.get("NEO_HIP_LIBRARY", "main")}))


if __name__ == "__main__":
    main()
