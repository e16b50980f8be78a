#!/usr/bin/env python3
"""Per-workgroup timeline of the streaming step kernel (k_lvl_step) from a NEO_TIMELINE build
(tools/build_timeline.sh): for `--steps` single-block steps of a bench workload, every
workgroup's start / end (wall_clock64, 100 MHz) and role; prints per role the median over
steps of: workgroups, first / median / last start, median / max duration, last end (us from
the launch's first start), and the step span.

    NEO_HIP_LIBRARY=tools/ab/tl/libneo_hip.so python tools/timeline.py --workload c4
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "neo-dsp_amd")]

ROLES = {1: "far2b", 2: "far2a", 3: "block", 4: "toep4", 5: "toep8", 6: "toep16", 7: "toep32", 8: "toepbig",
         9: "far1"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--json", default="")
    ap.add_argument("--raw", default="", help="save the first 16 samples' records (start, end, role, cu, xcc) to this .npz")
    ap.add_argument("--part", type=int, default=0, help="0 the one-launch step, 1 the step groups' block launch, "
                    "2 their slices launch (sampled once per step group)")
    args = ap.parse_args()
    import torch
    import bench
    import neo

    C, B, L = bench.WORKLOADS[args.workload]
    lib = neo._native.load()
    fn0 = lib.neo_hip_diag_timeline_part
    fn0.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    fn = lambda *xs: fn0(args.part, *xs)
    P = neo.num_partitions(L, B)
    conv = neo.UpolsConvolver(C, B, P)
    conv.set_batch(False)
    g = torch.Generator(device="cuda").manual_seed(1)
    conv.set_impulse(torch.rand((C, L), generator=g, device="cuda") * 2 - 1)
    nx = 64
    x = torch.rand((C, nx * B), generator=g, device="cuda") * 2 - 1
    s = torch.cuda.current_stream().cuda_stream
    feed = bench.Feed(conv, x, x, nx, B, s)
    feed.run(args.warmup)
    torch.cuda.synchronize()
    cap = 1 << 16
    buf = np.zeros((cap, 4), np.uint64)
    cnt = ctypes.c_int64()
    per = {}
    per_xcc = {}
    spans = []
    per_sample = conv.step_group() if args.part == 2 else 1
    raw = {}
    for it in range(args.steps):
        feed.run(per_sample)
        fn(buf.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(cnt))
        n = int(cnt.value)
        r = buf[:n].astype(np.int64)
        t0 = r[:, 0].min()
        st = (r[:, 0] - t0) / 100.0  # us
        en = (r[:, 1] - t0) / 100.0
        role = r[:, 2] & 0xffffffff
        xcc = (r[:, 2] >> 56) & 15
        if args.raw and it < 16:
            raw[f"s{it}"] = np.stack([st, en, role.astype(np.float64), ((r[:, 2] >> 32) & 0xffffff).astype(np.float64),
                                      xcc.astype(np.float64)], axis=1)
        spans.append(en.max())
        for xc in range(8):
            m = xcc == xc
            if m.any():
                xs = per_xcc.setdefault(xc, {"n": [], "s0": [], "e1": []})
                xs["n"].append(int(m.sum()))
                xs["s0"].append(st[m].min())
                xs["e1"].append(en[m].max())
        for k in np.unique(role):
            m = role == k
            d = per.setdefault(int(k), {"n": [], "s0": [], "smed": [], "s1": [], "dmed": [], "dmax": [], "e1": []})
            d["n"].append(int(m.sum()))
            d["s0"].append(st[m].min())
            d["smed"].append(np.median(st[m]))
            d["s1"].append(st[m].max())
            dur = en[m] - st[m]
            mid = r[:, 3][m]
            if (mid > 0).all():  # the role's mid-point stamp: loads landed (us after the workgroup's start)
                d.setdefault("mid", []).append(np.median((mid - r[:, 0][m]) / 100.0))
            d["dmed"].append(np.median(dur))
            d["dmax"].append(dur.max())
            d["e1"].append(en[m].max())
    out = {"workload": args.workload, "steps": args.steps, "span_us_median": float(np.median(spans)),
           "span_us_p90": float(np.percentile(spans, 90)), "roles": {}}
    print(f"{args.workload}: step span median {np.median(spans):.2f} us, p90 {np.percentile(spans, 90):.2f}")
    print(f"{'role':8s} {'wgs':>5s} {'start0':>7s} {'startmed':>8s} {'start1':>7s} {'durmed':>7s} {'durmax':>7s} {'end1':>7s} "
          f"{'midmed':>7s}")
    for k in sorted(per):
        d = {key: float(np.median(v)) for key, v in per[k].items()}
        out["roles"][ROLES.get(k, str(k))] = d
        print(f"{ROLES.get(k, str(k)):8s} {d['n']:5.0f} {d['s0']:7.2f} {d['smed']:8.2f} {d['s1']:7.2f} {d['dmed']:7.2f} "
              f"{d['dmax']:7.2f} {d['e1']:7.2f} {d.get('mid', float('nan')):7.2f}")
    out["xcc"] = {}
    for xc in sorted(per_xcc):
        d = {key: float(np.median(v)) for key, v in per_xcc[xc].items()}
        out["xcc"][xc] = d
        print(f"xcc {xc}: wgs {d['n']:.0f} first start {d['s0']:.2f} last end {d['e1']:.2f}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if args.raw:
        np.savez_compressed(args.raw, **raw)


if __name__ == "__main__":
    main()
