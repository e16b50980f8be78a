import sys, numpy as np
sys.path[:0] = ["neo-dsp_amd", "oracle"]
import neo, oracle as O
B, P = 128, 5
sig = O.noise(60, B * 16)
for p in range(P):
    H = np.zeros((P, B + 1), np.complex64); H[p] = 1
    c = neo.UpolsConvolver(1, B, P); c.filter(H[None])
    ref = O.Upols(H).run(sig)
    out = np.empty_like(sig)
    for t in range(16):
        blk = np.ascontiguousarray(sig[t*B:(t+1)*B][None]); c(blk); out[t*B:(t+1)*B] = blk[0]
    errs = [float(np.abs(out[t*B:(t+1)*B] - ref[t*B:(t+1)*B]).max()) for t in range(16)]
    print("p", p, "splits", c.splits, "per-block err", ["%.1e" % e for e in errs])
    # shifted comparison
    for d in range(-2, 3):
        if d >= 0: e = np.abs(out[d*B:] - ref[:len(ref)-d*B]).max()
        else: e = np.abs(out[:len(out)+d*B] - ref[-d*B:]).max()
        print("   shift", d, "%.2e" % e)
