"""Time large c2c FFT plans (N > 4096) on the device: effective GB/s = 16 B per point / time.
usage: python tools/largefft.py [orders...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neo-dsp_amd")]
import torch  # noqa: E402
import neo  # noqa: E402

orders = [int(a) for a in sys.argv[1:]] or [13, 16, 20, 24, 27]
for order in orders:
    n = 1 << order
    batch = max(1, (1 << 28) // n)  # 2 GiB of complex64
    x = torch.randn(batch * n, dtype=torch.complex64, device="cuda")
    y = torch.empty_like(x)
    plan = neo.fft.FFTPlan(0, order, batch)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        plan.execute_device(x.data_ptr(), y.data_ptr(), -1, s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        plan.execute_device(x.data_ptr(), y.data_ptr(), -1, s)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"order {order:2d} batch {batch:6d}: {ms:.3f} ms  {16 * n * batch / ms / 1e6:.0f} GB/s effective")
    del x, y, plan
