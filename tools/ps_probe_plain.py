#!/usr/bin/env python3
"""Plain-step latency-mode probe (NEO_PS_PROBE build: SRC=upols bash tools/build_variant.sh
probep -DNEO_PS_PROBE, then NEO_HIP_LIBRARY=tools/ab/probep/libneo_hip.so): one channel, one
synchronous call per block; per step the points of channel 0 on the GPU clock relative to the
record being seen: 1 split 0's window r2c done, 2 split 0's MAC done, 3 split 1's MAC done,
4 the tail found every split arrived, 5 slabs summed, 6 output stores issued; done = completion
signal. Median over the last 63 steps, us."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd")]


def main():
    import torch
    import neo

    lib = neo._native.load()
    fn = lib.neo_hip_diag_persist_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for B, L in ((4096, 131072), (1024, 32768)):
        for S in (0, 4, 8):
            P = neo.num_partitions(L, B)
            conv = neo.UpolsConvolver(1, B, P, options={"split_workgroups": S, "levels": 0})
            conv.set_impulse(np.random.default_rng(1).random((1, L), dtype=np.float32) - 0.5)
            conv.set_batch(False)
            conv.set_persistent(True)
            x = torch.rand((1, 400 * B), device="cuda")
            torch.cuda.current_stream().synchronize()
            for i in range(400):
                conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, 400 * B, 1, 0)
            buf = (ctypes.c_ulonglong * (10 * 64))()
            neo._native.check(fn(conv._h, buf))
            a = np.array(buf[:], dtype=np.float64)
            st = a[:128].reshape(64, 2)
            pr = a[128:].reshape(64, 8)
            rel = (pr[:, 1:7] - st[:, :1]) * 1e-2
            done = (st[:, 1] - st[:, 0]) * 1e-2
            print(f"B={B} P={P} S={conv.splits}", "points 1-6 (us after seen):", np.round(np.median(rel, axis=0), 2),
                  "done", round(float(np.median(done)), 2), flush=True)
            conv.set_persistent(False)
            conv.close()


if __name__ == "__main__":
    main()
