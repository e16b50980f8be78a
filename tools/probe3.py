"""Phase stamps of k_upols_ahead3 (direct-head block step), diagnostic build: ns since entry
of channel 0 for wave 0 (window in LDS, r2c done, row stored), the MAC waves (rest done),
the c2r wave (start after the MAC, z done) and convolution wave 0 (start, partial done,
all inputs ready, output stored). usage: python tools/probe3.py [c5|c4|c3]"""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["NEO_HIP_LIBRARY"] = os.path.join(R, "tools", "probe", "libneo_hip_probe.so")
sys.path[:0] = [os.path.join(R, "neo-dsp_amd"), R]
import torch  # noqa: E402
import neo  # noqa: E402
import bench  # noqa: E402
from neo import _native  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
C, B, L = bench.WORKLOADS[wl]
P = neo.num_partitions(L, B)
g = torch.Generator(device="cuda").manual_seed(1)
cv = neo.UpolsConvolver(C, B, P)
cv.set_impulse(torch.rand((C, L), generator=g, device="cuda") * 2 - 1)
cv.set_batch(False)
cv.set_ahead(True)
lib = _native.load()
buf = (ctypes.c_ulonglong * 16)()
x = torch.rand((C, B), generator=g, device="cuda") * 2 - 1
y = torch.empty_like(x)
names = ["win", "fft", "row", "rest", "c2r0", "z", "conv0", "convP", "ready", "out"]
rows = {}
for it in range(4 * 32):
    ph = cv.ahead_info()[1]
    cv.process_device(x.data_ptr(), B, y.data_ptr(), B, 0)
    torch.cuda.synchronize()
    assert lib.neo_hip_debug_probe(buf) == 0
    t = list(buf)
    if it >= 64:
        rows.setdefault(ph, []).append([(t[k] - t[0]) * 10 for k in range(1, 11)])
print(f"{wl}: ns since entry (channel 0), median over 2 windows")
print("  j " + " ".join(f"{n:>6s}" for n in names))
for j in sorted(rows):
    v = rows[j]
    med = [sorted(c)[len(c) // 2] for c in zip(*v)]
    print(f"{j:3d} " + " ".join(f"{m:6d}" for m in med))
