"""debug: latency mode vs the normal streaming step, max |difference| (0 = bit-equal)"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle")]
import numpy as np
import torch
import neo
import oracle
for method, C, B, P in (("upols", 1, 512, 188), ("upols", 4, 256, 100), ("upola", 3, 128, 240), ("upols", 16, 64, 200)):
    ir = np.stack([oracle.noise(7000 + c, B * P) for c in range(C)])
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    outs = []
    for persist in (False, True):
        cv = neo.UpolsConvolver(C, B, P, method=method)
        cv.filter(parts); cv.set_batch(False)
        if persist:
            cv.set_persistent(True)
        nb = 3 * P // 2 + 37
        x = np.stack([oracle.noise(7100 + c, B * nb) for c in range(C)])
        t = torch.from_numpy(x.copy()).cuda()
        s = torch.cuda.current_stream()
        s.synchronize()
        for i in range(nb):
            cv.process_blocks_ptr(t.data_ptr() + 4 * i * B, t.data_ptr() + 4 * i * B, nb * B, 1, s.cuda_stream)
        s.synchronize()
        outs.append(t.cpu().numpy())
        cv.close()
    print(method, C, B, P, "max|diff|", float(np.abs(outs[0] - outs[1]).max()), "peak", float(np.abs(outs[0]).max()), flush=True)
