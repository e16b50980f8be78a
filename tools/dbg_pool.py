"""debug: one-channel C5-shape handles through host I/O, outputs vs the oracle per handle"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np
import neo
import oracle
from conftest import peak_err
B, P, nb = 512, int(sys.argv[2]) if len(sys.argv) > 2 else 938, 6
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ir = oracle.noise(6100, B * P)[None]
parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
x = np.stack([oracle.noise(6200, B * nb)])
ref = oracle.dense_convolve(x, parts)
hs = []
for i in range(N):
    c = neo.UpolsConvolver(1, B, P)
    c.filter(parts)
    c.set_batch(False)
    hs.append(c)
for i, c in enumerate(hs):
    y = np.empty_like(x)
    for t in range(nb):
        blk = np.ascontiguousarray(x[:, t * B:(t + 1) * B])
        c(blk)
        y[:, t * B:(t + 1) * B] = blk
    print(i, "err", peak_err(y, ref), "max|y|", float(np.abs(y).max()), "eq-in", bool(np.array_equal(y, x)), flush=True)
