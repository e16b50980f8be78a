"""Convolver bring-up and teardown (dmem.hip): handle buffers come from per-device chunks the
library keeps mapped, streams from a per-device set of four, so creating and destroying a plugin's
convolvers (extra/plugin/src/dsp/DenseConvolution.cpp:78-108 rebuilds one per channel on every IR
change) costs no device synchronization and no stream creation. Freed memory is reused by later
handles (whose results must not depend on what it held) and the chunks drain back to HIP."""
import ctypes
import time

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu


def _info(lib, dev=0):
    r, u = ctypes.c_int64(), ctypes.c_int64()
    assert lib.neo_hip_memory_info(dev, ctypes.byref(r), ctypes.byref(u)) == 0
    return r.value, u.value


def test_pool_reuse_and_drain(neo_gpu, oracle):
    """64 one-channel C5-shape handles created, stepped (streaming levels primed: level and far
    buffers allocated) and destroyed, twice; the second round's outputs equal the first's bit for
    bit on reused (dirty) memory and match the oracle; in-use bytes return to where they were;
    trim releases every unused chunk."""
    lib = neo_gpu._native.load()
    B, P, nb = 512, 938, 6
    r0, u0 = _info(lib)
    ir = oracle.noise(6100, B * P)[None]
    parts = oracle.uniform_partition(oracle.normalize_impulse(ir), B)
    x = np.stack([oracle.noise(6200, B * nb)])
    ref = oracle.dense_convolve(x, parts)
    outs = []
    times = []
    for rnd in range(2):
        hs = []
        for i in range(64):
            t0 = time.perf_counter()
            c = neo_gpu.UpolsConvolver(1, B, P)
            times.append(time.perf_counter() - t0)
            c.filter(parts)
            c.set_batch(False)
            hs.append(c)
        y = None
        for c in hs:
            y = np.empty_like(x)
            for t in range(nb):
                blk = x[:, t * B:(t + 1) * B].copy()  # a view of a one-row array is contiguous: copy
                c(blk)
                y[:, t * B:(t + 1) * B] = blk
        outs.append(y)
        r1, u1 = _info(lib)
        assert u1 > u0
        for c in hs:
            c.close()
        assert _info(lib)[1] == u0
    assert np.array_equal(outs[0], outs[1])
    assert peak_err(outs[1], ref) <= 1e-5
    assert np.median(times) < 2e-3, f"median create {np.median(times) * 1e3:.2f} ms"
    neo_gpu.memory_trim(0)
    info = neo_gpu.memory_info(0)
    assert info["in_use"] == u0 and info["reserved"] < r1
