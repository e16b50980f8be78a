"""A/B the UPOLS MAC kernel variants in one process (interleaved rounds; §5.4 rule 24).
usage: python tools/macbench.py [c5|c4] [rounds] [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), REPO]
import torch  # noqa: E402
import neo  # noqa: E402
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
C, B, L = bench.WORKLOADS[wl]
P = neo.num_partitions(L, B)
g = torch.Generator(device="cuda").manual_seed(1)
ir = torch.rand((C, L), generator=g, device="cuda") * 2 - 1
variants = {}
specs = sys.argv[4:] or ["NEO_HIP_NT=0", "NEO_HIP_NT=1"]  # each: comma-separated env assignments
for spec in specs:
    for kv in spec.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
    c = neo.UpolsConvolver(C, B, P)
    c.set_batch(False)  # the streaming step (one MAC pass per block)
    c.set_impulse(ir)
    variants[spec] = c
x = torch.rand((C, steps * B), generator=g, device="cuda") * 2 - 1
y = torch.empty_like(x)
res = {k: [] for k in variants}
outs = {}
for r in range(rounds):
    for name, c in variants.items():
        c.reset()
        c.timing()
        c.set_timing(True)
        c.process_blocks(x, y)
        torch.cuda.synchronize()
        c.set_timing(False)
        ms, n = c.timing()
        res[name].append(ms / n)
        outs[name] = y.clone()
bytes_mac = C * (16 * P * B + 20 * B)
for name, v in res.items():
    v.sort()
    med = v[len(v) // 2]
    print(f"{wl} {name:36s} S={variants[name].splits:3d} MAC median {med:.4f} ms  min {v[0]:.4f}  -> {bytes_mac / med / 1e6:.0f} GB/s "
          f"({bytes_mac / med / 1e6 / 8000:.3f} of 8 TB/s)")
first = next(iter(outs.values()))
print("max |y - y_first| per variant:", [float((o - first).abs().max()) for o in outs.values()],
      "peak", float(first.abs().max()))
