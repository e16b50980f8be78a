"""The plain step's splits per channel at one channel (the reference benchmark's shape, B = 4096,
P = 32, and B = 1024 / 2048): GPU time per step (HIP events around every step) and the latency
mode's GPU step and host round trip, per forced split count (neo_hip_upols_opts.split_workgroups)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "neo-dsp_amd"))
import neo  # noqa: E402

dev = torch.device("cuda:0")
for B, L in ((4096, 131072), (2048, 65536), (1024, 32768)):
    P = neo.num_partitions(L, B)
    ir = torch.rand((1, L), device=dev) * 2 - 1
    x = torch.rand((1, B * 512), device=dev) * 2 - 1
    for S in (0, 1, 2, 4, 8, 16, 32):
        if S > P:
            continue
        conv = neo.UpolsConvolver(1, B, P, options={"split_workgroups": S, "levels": 0})
        conv.set_impulse(ir, normalize=True)
        conv.set_batch(False)
        s = torch.cuda.current_stream()
        for i in range(64):
            conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, x.shape[1], 1, s.cuda_stream)
        torch.cuda.synchronize()
        conv.step_times()
        conv.set_timing(True, every=1)
        for i in range(256):
            conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, x.shape[1], 1, s.cuda_stream)
        torch.cuda.synchronize()
        conv.set_timing(False)
        st = np.array(conv.step_times()) * 1e3
        rt = []
        for i in range(200):
            t0 = time.perf_counter()
            conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, x.shape[1], 1, s.cuda_stream)
            s.synchronize()
            rt.append(time.perf_counter() - t0)
        conv.set_persistent(True)
        prt = []
        for i in range(400):
            t0 = time.perf_counter()
            conv.process_blocks_ptr(x.data_ptr() + 4 * i * B, x.data_ptr() + 4 * i * B, x.shape[1], 1, s.cuda_stream)
            prt.append(time.perf_counter() - t0)
        pst = np.array(conv.persist_step_times())
        conv.set_persistent(False)
        print(json.dumps({"B": B, "P": P, "split_workgroups": S, "step_p50_us": round(float(np.median(st)), 2),
                          "rt_p50_us": round(float(np.median(rt)) * 1e6, 1),
                          "persist_rt_p50_us": round(float(np.median(prt[100:])) * 1e6, 1),
                          "persist_gpu_p50_us": round(float(np.median(pst)), 2)}), flush=True)
        conv.close()
