"""A/B: the batched 4096-pt FFT on torch-allocated vs raw hipMalloc'd buffers (same process)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd")]
import torch  # noqa: E402
import neo  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
N, B = 4096, 65536
nbytes = N * B * 8
x = torch.view_as_complex((torch.rand((B, N, 2), device="cuda") * 2 - 1))
y = torch.empty_like(x)
raw = []
for _ in range(2):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
    raw.append(p.value)
hip.hipMemcpy(ctypes.c_void_p(raw[0]), ctypes.c_void_p(x.data_ptr()), ctypes.c_size_t(nbytes), 3)
torch.cuda.synchronize()
plan = neo.fft.FFTPlan(0, 12, B)
print("torch x ptr %x y %x raw %x %x" % (x.data_ptr(), y.data_ptr(), raw[0], raw[1]))


def timeit(inp, out, n=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        plan.execute_device(inp, out, -1, 0)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for r in range(3):
    a = timeit(x.data_ptr(), y.data_ptr())
    b = timeit(raw[0], raw[1])
    c = timeit(x.data_ptr(), raw[1])
    d = timeit(raw[0], y.data_ptr())
    print(f"round {r}: torch->torch {a:.4f}  raw->raw {b:.4f}  torch->raw {c:.4f}  raw->torch {d:.4f} ms")
print(torch.cuda.memory.memory_stats().get("num_alloc_retries"), os.environ.get("PYTORCH_HIP_ALLOC_CONF"),
      os.environ.get("PYTORCH_CUDA_ALLOC_CONF"))
