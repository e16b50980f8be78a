"""Replicates test_api.cpp's upola_convolver_v2 piece pattern through the Python API."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "neo-dsp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np
import neo, oracle

for B in (128, 256, 512, 1024):
    h = np.zeros((3, B + 1), np.complex64); h[0] = 1
    sig = oracle.noise(B, B * 20)
    conv = neo.upola_convolver_v2(); conv.filter(h)
    out = sig.copy(); i = 0; step = B // 3; pieces = []
    while i < len(out):
        n = min(step, len(out) - i)
        blk = out[i:i + n].copy(); conv(blk); out[i:i + n] = blk
        err = np.abs(blk - sig[i:i + n]).max()
        pieces.append((i, n, i % B, float(err)))
        i += step; step = step * 2 % (3 * B) + 1
    bad = [p for p in pieces if p[3] > 1e-5]
    print(B, "max", np.abs(out - sig).max(), "bad pieces (start, n, pos, err):", bad[:6])
