"""Phase stamps of k_upols_ahead2 (channel 0) from the diagnostic build (tools/probe/,
-DNEO_AHEAD_PROBE): s_memrealtime (100 MHz) at kernel entry, after the input loads,
after the window FFT, before/after each workgroup barrier, after the c2r; wave 1 (MAC
group) at entry and when its slab sum + rows are done. usage: python tools/probebench.py [c5|c4]"""
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
ir = torch.rand((C, L), generator=g, device="cuda") * 2 - 1
cv = neo.UpolsConvolver(C, B, P)
cv.set_impulse(ir)
cv.set_batch(False)
cv.set_ahead(True)
lib = _native.load()
buf = (ctypes.c_ulonglong * 16)()
x = torch.rand((C, B), generator=g, device="cuda") * 2 - 1
y = torch.empty_like(x)
names = ["entry", "loaded", "fft", "r2c+row", "bar1", "bar2", "c2r"]
rows = {}
for it in range(4 * 32):
    ph = cv.ahead_info()[1]
    cv.process_device(x.data_ptr(), B, y.data_ptr(), B, 0)
    torch.cuda.synchronize()
    assert lib.neo_hip_debug_probe(buf) == 0
    t = list(buf)
    if it >= 64:
        rows.setdefault(ph, []).append([(t[k] - t[0]) * 10 for k in range(7)] + [(t[8] - t[0]) * 10, (t[9] - t[0]) * 10])
print(f"{wl}: ns since wave-0 entry, median over 2 windows; MAC wave: entry / done")
print("  j " + " ".join(f"{n:>8s}" for n in names) + "  macIn  macDone")
for j in sorted(rows):
    v = rows[j]
    med = [sorted(c)[len(c) // 2] for c in zip(*v)]
    print(f"{j:3d} " + " ".join(f"{m:8d}" for m in med[:7]) + f" {med[7]:6d} {med[8]:8d}")

# clock during the window pass under sustained load: 8 windows back to back, stamps of the
# last pass (workgroup 0: s_memtime shader cycles over s_memrealtime 100 MHz ticks)
xs = torch.rand((C, 255 * B), generator=g, device="cuda") * 2 - 1  # ends mid-window
ys = torch.empty_like(xs)
for rep in range(3):
    while cv.ahead_info()[1] != 0:
        cv.process_device(x.data_ptr(), B, y.data_ptr(), B, 0)
    cv.process_blocks_ptr(xs.data_ptr(), ys.data_ptr(), 255 * B, 255, 0)
    torch.cuda.synchronize()
    assert lib.neo_hip_debug_probe(buf) == 0
    t = list(buf)
    cyc, rt = t[12] - t[10], t[13] - t[11]
    print(f"window pass (workgroup 0): {rt * 10 / 1e3:.1f} us, {cyc} cycles -> {cyc / (rt * 10):.3f} GHz")
    print("  last block step of the sustained run (ns):", [(t[k] - t[0]) * 10 for k in range(7)],
          "MAC wave:", (t[8] - t[0]) * 10, (t[9] - t[0]) * 10)

# per-workgroup entry/exit of the last window pass: how many workgroups run at once
span = (ctypes.c_ulonglong * (4096 * 2))()
assert lib.neo_hip_debug_wgspan(span) == 0
nwg = C * cv.ahead_info()[3] * max(1, B // 256)
ent = [span[2 * i] for i in range(nwg)]
ext = [span[2 * i + 1] for i in range(nwg)]
t0 = min(ent)
ent = [(e - t0) * 10 / 1e3 for e in ent]
ext = [(e - t0) * 10 / 1e3 for e in ext]
dur = sorted(b - a for a, b in zip(ent, ext))
print(f"{nwg} workgroups: entry us min/median/max {min(ent):.1f}/{sorted(ent)[nwg // 2]:.1f}/{max(ent):.1f}; "
      f"exit max {max(ext):.1f}; duration min/median/max {dur[0]:.1f}/{dur[nwg // 2]:.1f}/{dur[-1]:.1f}")
hist = [0] * 10
for e in ent:
    hist[min(9, int(e / (max(ext) / 10)))] += 1
print("entry histogram over the pass (10 bins):", hist)
by_xcd = {}
for i in range(nwg):
    by_xcd.setdefault(i % 8, []).append(ext[i] - ent[i])
print("duration by blockIdx % 8 (XCD):", {k: round(sum(v) / len(v), 1) for k, v in sorted(by_xcd.items())})
by_g = {}
for i in range(nwg):
    by_g.setdefault(i % 2, []).append(ext[i] - ent[i])
print("duration by bin half (blockIdx % 2):", {k: round(sum(v) / len(v), 1) for k, v in sorted(by_g.items())})
d16 = [round(ext[i] - ent[i]) for i in range(64)]
print("first 64 workgroups:", d16)
print("mean duration per 32 consecutive workgroups:", [round(sum(ext[i] - ent[i] for i in range(k, k + 32)) / 32) for k in range(0, nwg, 32)])
print("exit time per 32 consecutive workgroups (max):", [round(max(ext[i] for i in range(k, k + 32))) for k in range(0, nwg, 32)])
