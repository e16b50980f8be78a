"""A/B the batched MAC pass (process_blocks, T blocks per pass) in one process, interleaved.
usage: python tools/batchbench.py [c5|c4|c3|CxBxL] [rounds] [blocks] spec...   spec = ENV=V[,ENV=V]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), REPO]
import torch  # noqa: E402
import neo  # noqa: E402
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 96
C, B, L = bench.WORKLOADS[wl] if wl in bench.WORKLOADS else map(int, wl.split("x"))  # or CxBxL
P = neo.num_partitions(L, B)
g = torch.Generator(device="cuda").manual_seed(1)
ir = torch.rand((C, L), generator=g, device="cuda") * 2 - 1
variants = {}
for spec in sys.argv[4:] or ["NEO_HIP_BATCH_T=8,NEO_HIP_BATCH_NB=2"]:
    for kv in spec.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
    c = neo.UpolsConvolver(C, B, P)
    c.set_impulse(ir)
    variants[spec] = c
x = torch.rand((C, nb * B), generator=g, device="cuda") * 2 - 1
y = torch.empty_like(x)
res = {k: [] for k in variants}
wall = {k: [] for k in variants}
outs = {}
for r in range(rounds + 1):
    for name, c in variants.items():
        c.reset()
        c.timing()
        c.set_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.process_blocks(x, y)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        c.set_timing(False)
        ms, n = c.timing()
        if r:
            res[name].append(ms / n)
            wall[name].append((t1 - t0) * 1e3 / nb)
        outs[name] = y.clone()
bytes_pass = C * 16 * P * B
for name in variants:
    v, w = sorted(res[name]), sorted(wall[name])
    med, wm = v[len(v) // 2], w[len(w) // 2]
    flop_pass = 8.0 * C * P * B * min(32, nb)
    print(f"{wl} {name:44s} MAC/pass {med:.4f} ms ({bytes_pass / med / 1e6:.0f} GB/s H+FDL, "
          f"{flop_pass / med / 1e9:.1f} TFLOP/s) "
          f"wall/block {wm:.4f} ms -> {C * B / wm / 1e3:.0f} Msamples/s")
first = next(iter(outs.values()))
print("max |y - y_first| per variant:", [float((o - first).abs().max()) for o in outs.values()],
      "peak", float(first.abs().max()))
