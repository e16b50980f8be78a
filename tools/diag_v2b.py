import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "neo-dsp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np, neo, oracle
B, L, C = 64, 64, 2
ir = np.stack([oracle.noise(180 + c, L) for c in range(C)])
parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
N = B * 9
sig = np.stack([oracle.noise(190 + c, N) for c in range(C)])
cuts = sorted({0, 1, B // 2 + 1, B + B // 2 + 1, 3 * B + 1, 4 * B + 1, 4 * B + 2, 6 * B, 8 * B, N})
ref = np.empty_like(sig)
for c in range(C):
    o = oracle.Upola2(parts[c])
    for a, b in zip(cuts[:-1], cuts[1:]):
        ref[c, a:b] = o(sig[c, a:b])
for batch in (True, False):
    conv = neo.UpolsConvolver(C, B, parts.shape[1], method="upola_v2")
    conv.set_batch(batch)
    conv.filter(parts)
    got = np.concatenate([conv.process(np.ascontiguousarray(sig[:, a:b])) for a, b in zip(cuts[:-1], cuts[1:])], axis=1)
    err = np.abs(got - ref).max(axis=0)
    blocks = [int(i // B) for i in np.nonzero(err > 1e-5)[0]]
    print("batch", batch, "bad blocks", sorted(set(blocks)), "cuts", cuts, "T", conv.batch_info())
# plain upola with process_blocks of 2 blocks
conv = neo.UpolsConvolver(C, B, parts.shape[1], method="upola")
conv.filter(parts)
import torch
t = torch.from_numpy(sig[:, :2*B].copy()).cuda(); conv.process_blocks(t); torch.cuda.synchronize()
r2 = oracle.dense_convolve(sig[:, :2*B].copy(), parts, method="upola")
print("upola 2 blocks err", float(np.abs(t.cpu().numpy()-r2).max()))
