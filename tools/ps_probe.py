#!/usr/bin/env python3
"""Latency-mode probe (NEO_PS_PROBE build, tools/build_variant.sh probe -DNEO_PS_PROBE): C3 shape,
one synchronous call per block; per step the block role's points on the GPU clock relative to
the record being seen: 1 wave 0's loads issued, 2 r2c done, 3 all pair loads landed (barrier),
4 joined spectrum (barrier), 5 output stores issued, done = completion signal. Median over the
last 63 steps, us.
    NEO_HIP_LIBRARY=tools/ab/probe/libneo_hip.so python tools/ps_probe.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd")]


def main():
    import torch
    import neo

    B, P = 512, 188
    conv = neo.UpolsConvolver(1, B, P)
    conv.set_impulse(np.random.default_rng(1).random((1, 96000), dtype=np.float32) - 0.5)
    conv.set_batch(False)
    conv.set_persistent(True)
    x = torch.rand((1, 400 * B), device="cuda")
    torch.cuda.current_stream().synchronize()
    lib = neo._native.load()
    fn = lib.neo_hip_diag_persist_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for mode, per in (("roundtrip", 1), ("pipelined", 64)):
        for i in range(0, 400, per):
            conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, 400 * B, per, 0)
        buf = (ctypes.c_ulonglong * (10 * 64))()
        neo._native.check(fn(conv._h, buf))
        a = np.array(buf[:], dtype=np.float64)
        st = a[:128].reshape(64, 2)
        pr = a[128:].reshape(64, 8)
        rel = (pr[:, :6] - st[:, :1]) * 1e-2
        done = (st[:, 1] - st[:, 0]) * 1e-2
        gap = np.diff(np.sort(st[:, 0])) * 1e-2
        print(mode, "points (us after seen):", np.round(np.median(rel, axis=0), 2), "done", round(float(np.median(done)), 2),
              "seen-to-seen", round(float(np.median(gap)), 2))
    conv.set_persistent(False)


if __name__ == "__main__":
    main()
