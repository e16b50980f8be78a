import sys, ctypes
order = sys.argv[1]
sys.path[:0] = ["neo-dsp_amd"]
if order == "torch_first":
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
    x = torch.ones(4, device="cuda"); print("torch ok", x.sum().item())
    import neo
    print("neo sees", neo._native.device_count())
    import numpy as np
    print(neo.fft.fft(np.ones(8, np.complex64))[:2])
    t = torch.ones(8, dtype=torch.complex64, device="cuda")
    print("device fft", neo.fft.fft(t)[:2].cpu())
else:
    import neo, numpy as np
    print("neo sees", neo._native.device_count())
    print(neo.fft.fft(np.ones(8, np.complex64))[:2])
    import torch
    print("torch sees", torch.cuda.device_count(), torch.cuda.is_available())
import os
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip" in l or "hsa-runtime" in l)))
