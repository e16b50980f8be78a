"""Does a batched MAC pass on one stream overlap with lookahead block steps on another?
A = offline convolver (process_blocks of 32 blocks, one k_batch_mac pass) on stream a;
B = streaming convolver (32 single-block lookahead steps) on stream b; times alone and
concurrent. usage: python tools/overlapbench.py [c5|c4] [A-env ENV=V,...]"""
import os
import sys
import time

import torch

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neo-dsp_amd"),
                os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
import neo  # noqa: E402
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
C, B, L = bench.WORKLOADS[wl]
P = neo.num_partitions(L, B)
g = torch.Generator(device="cuda").manual_seed(1)
ir = torch.rand((C, L), generator=g, device="cuda") * 2 - 1
cb = neo.UpolsConvolver(C, B, P)
cb.set_impulse(ir)
cb.set_batch(False)  # process_blocks = single-block steps
cb.set_ahead(True)
for spec in sys.argv[2:]:
    for kv in spec.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
ca = neo.UpolsConvolver(C, B, P)
ca.set_impulse(ir)
nb = 32
x = torch.rand((C, nb * B), generator=g, device="cuda") * 2 - 1
ya = torch.empty_like(x)
yb = torch.empty((nb, C, B), device="cuda")
xb = x.view(C, nb, B).transpose(0, 1).contiguous()
sa = torch.cuda.Stream(priority=0)
sb = torch.cuda.Stream(priority=-1)  # block steps on a high-priority queue


def run_a():
    ca.process_blocks(x, ya, stream=sa.cuda_stream)


def step0():  # up to and including phase 0 (B's own window pass), untimed
    while True:
        ph = cb.ahead_info()[1]
        cb.process_device(xb[0].data_ptr(), B, yb[0].data_ptr(), B, sb.cuda_stream)
        if ph == 0:
            return


yb2 = torch.empty_like(x)


def run_b():  # the 31 block steps that follow it (k_upols_ahead2 only), looped in the C-ABI
    cb.process_blocks_ptr(x.data_ptr() + 4 * B, yb2.data_ptr() + 4 * B, nb * B, nb - 1, sb.cuda_stream)


def sync():  # both side streams explicitly (a device-wide synchronize did not wait for them)
    sa.synchronize()
    sb.synchronize()
    torch.cuda.synchronize()


def timed(fn, reps=20):
    ts = []
    for r in range(reps + 2):
        step0()
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        if r >= 2:
            ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for _ in range(3):
    step0()
    run_b()
    run_a()
torch.cuda.synchronize()
ta = timed(run_a)
tb = timed(run_b)
tab = timed(lambda: (run_a(), run_b()))
tba = timed(lambda: (run_b(), run_a()))
print(f"{wl} A-env={sys.argv[2:]} A(pass of 32) {ta:.3f} ms  B(31 lookahead block steps) {tb:.3f} ms  "
      f"A||B {tab:.3f} ms  B||A {tba:.3f} ms  (sum {ta + tb:.3f}, max {max(ta, tb):.3f})")
