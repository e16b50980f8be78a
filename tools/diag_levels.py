"""Diagnostic: streaming-level steps vs the oracle, per block — first block whose output
differs and the error profile, for a list of (B, P, C, nb) shapes. GPU box only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle")]

import torch  # noqa: E402

import neo  # noqa: E402
import oracle as O  # noqa: E402


def run(B, P, C, nb, method="upols", seed=1):
    L = B * (P - 1) + B // 2 + 1
    ir = np.stack([O.noise(seed + c, L) for c in range(C)])
    parts = O.uniform_partition(O.normalize_impulse(ir), B)
    sig = np.stack([O.noise(seed + 10 + c, B * nb) for c in range(C)])
    ref = O.dense_convolve(sig, parts, method=method)
    conv = neo.UpolsConvolver(C, B, P, method=method)
    conv.filter(parts)
    conv.set_batch(False)
    conv.set_ahead(True)
    t = torch.from_numpy(sig).cuda()
    conv.process_blocks(t)
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    peak = np.abs(ref).max()
    err = np.abs(got - ref).reshape(C, nb, B).max(axis=(0, 2)) / peak
    bad = np.nonzero(err > 1e-5)[0]
    print(f"B={B} P={P} C={C} nb={nb} {method}: max {err.max():.2e}", end=" ")
    if len(bad):
        print(f"first bad block {bad[0]}, bad blocks {len(bad)}, err at first bad {err[bad[0]]:.2e}; "
              f"bad bins of block {bad[0]}:", end=" ")
        d = np.fft.rfft(got.reshape(C, nb, B)[0, bad[0]]) - np.fft.rfft(ref.reshape(C, nb, B)[0, bad[0]])
        print(np.nonzero(np.abs(d) > 1e-4 * np.abs(np.fft.rfft(ref.reshape(C, nb, B)[0, bad[0]])).max())[0][:20])
    else:
        print("ok")


if __name__ == "__main__":
    for args in [(32, 16, 2, 60), (32, 20, 2, 80), (32, 40, 2, 120), (32, 70, 2, 200), (32, 200, 2, 500),
                 (32, 257, 1, 700), (32, 300, 1, 800), (32, 700, 1, 1500), (256, 300, 2, 500)]:
        run(*args)
