"""debug: which setup call on handle B waits for handle A's resident latency-mode kernel"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np
import torch
import neo
import oracle
B, P = 256, 100
ir = oracle.noise(1, B * P)[None]
parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
a = neo.UpolsConvolver(1, B, P); a.filter(parts); a.set_batch(False)
b = neo.UpolsConvolver(1, B, P); b.filter(parts); b.set_batch(False)
c = neo.UpolsConvolver(1, B, P)
a.set_persistent(True, idle_ms=3000.0)
t = torch.from_numpy(oracle.noise(2, B * 4)[None].copy()).cuda()
torch.cuda.current_stream().synchronize()
s = torch.cuda.current_stream().cuda_stream
a.process_blocks_ptr(t.data_ptr(), t.data_ptr(), B * 4, 4, s)
print("running", a.persistent_info(), flush=True)
def tm(name, f):
    t0 = time.perf_counter(); f(); print(f"{name}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
tm("b.reset", b.reset)
tm("b.reset again", b.reset)
tm("b.filter host", lambda: b.filter(parts))
tm("b.set_persistent", lambda: b.set_persistent(True, idle_ms=50.0))
tm("b.set_persistent off", lambda: b.set_persistent(False))
tm("c.create", lambda: neo.UpolsConvolver(1, B, P).close())
tm("torch stream sync", lambda: torch.cuda.current_stream().synchronize())
print("still running", a.persistent_info(), flush=True)
a.set_persistent(False)
