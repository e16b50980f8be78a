"""debug: do other streams' work wait for a resident latency-mode kernel (hardware queue sharing)?"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle")]
import torch
import neo
import oracle
B, P = 256, 100
ir = oracle.noise(1, B * P)[None]
parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
pre = [torch.cuda.Stream() for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 0)]
a = neo.UpolsConvolver(1, B, P); a.filter(parts); a.set_batch(False)
a.set_persistent(True, idle_ms=1500.0)
t = torch.from_numpy(oracle.noise(2, B * 4)[None].copy()).cuda()
torch.cuda.current_stream().synchronize()
a.process_blocks_ptr(t.data_ptr(), t.data_ptr(), B * 4, 4, torch.cuda.current_stream().cuda_stream)
res = []
for i, s in enumerate(pre + [torch.cuda.Stream() for _ in range(8)]):
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        z = torch.ones(16, device="cuda") * 2
    s.synchronize()
    res.append(round(1e3 * (time.perf_counter() - t0), 2))
hs = []
for i in range(6):
    t0 = time.perf_counter()
    h = neo.UpolsConvolver(1, B, P); h.filter(parts); h.reset()
    res.append(("h", round(1e3 * (time.perf_counter() - t0), 2)))
    hs.append(h)
print("ms per stream op:", res, "running", a.persistent_info()["running"], flush=True)
a.set_persistent(False)
