"""C-ABI boundary checks that need no GPU: the library loads, exports exactly
the symbols include/neo_hip.h declares, validates arguments before touching a
device, and the Python mirror binds every one of them."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "neo_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"NEO_HIP_API\s+[^;(]*?\b(neo_hip_\w+)\s*\(", txt)))


def test_header_declares_api():
    syms = declared_symbols()
    assert "neo_hip_fft_plan_create" in syms and "neo_hip_upols_process" in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol():
    import neo

    lib = neo._native.LIB_PATH
    assert os.path.exists(lib), "build libneo_hip.so first (make -C neo-dsp_amd)"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (neo_hip_\w+)", out))
    assert set(declared_symbols()) == exported
    # and the Python binding covers them all
    assert set(neo._native.SIGNATURES) == exported
    neo._native.load()


def test_host_validation_without_gpu():
    import neo

    lib = neo._native.load()
    h = ctypes.c_void_p()
    assert lib.neo_hip_fft_plan_create(28, 1, 0, 0, ctypes.byref(h)) == neo._native.NEO_HIP_EINVAL
    assert b"unsupported order" in lib.neo_hip_last_error()
    assert lib.neo_hip_fft_plan_create(4, 0, 0, 0, ctypes.byref(h)) == neo._native.NEO_HIP_EINVAL
    assert lib.neo_hip_upols_create(1, 500, 3, 0, ctypes.byref(h)) == neo._native.NEO_HIP_EINVAL
    assert lib.neo_hip_upols_create(0, 512, 3, 0, ctypes.byref(h)) == neo._native.NEO_HIP_EINVAL
    assert lib.neo_hip_upols_join_background(None, None) == neo._native.NEO_HIP_EINVAL
    assert lib.neo_hip_upols_get_far_form(None, None) == neo._native.NEO_HIP_EINVAL
    assert lib.neo_hip_fft_max_order() == 27
    hdr = open(os.path.join(REPO, "include", "neo_hip.h")).read()
    assert lib.neo_hip_version() == int(re.search(r"#define NEO_HIP_VERSION (\d+)", hdr).group(1))
    assert neo._native.ABI_VERSION == lib.neo_hip_version()
    with pytest.raises(neo._native.NeoHipError):
        neo.fft.FFTPlan(0, 28)


def test_num_partitions_matches_reference_formula(oracle):
    import neo

    for L, B in [(4096, 128), (4095, 128), (480000, 512), (480000, 256), (96000, 512), (1, 64), (64, 64), (65, 64)]:
        assert neo.num_partitions(L, B) == oracle.num_partitions(L, B)
    assert neo.num_partitions(480000, 512) == 938 and neo.num_partitions(480000, 256) == 1875
    assert neo.num_partitions(96000, 512) == 188


def test_python_fft_helpers():
    import neo

    assert neo.fft.next_order(1024) == 10 and neo.fft.next_order(1025) == 11 and neo.fft.next_order(1) == 0
    assert neo.fft.size(12) == 4096
    with pytest.raises(RuntimeError):
        neo.fft._check_size(12)


def test_no_cpu_fallback_without_gpu():
    """The product path fails loudly when no device is present (this container)."""
    import neo

    if neo._native.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        neo.fft.fft(np.zeros(8, np.complex64))
    with pytest.raises(RuntimeError):
        neo.UpolsConvolver(1, 128, 2)


def test_rfftfreq_reference_values():
    """extra/python/test/test.py:65-68 (host index arithmetic, no GPU)."""
    import neo

    assert neo.fft.rfftfreq(2) == pytest.approx([0.0, 0.5])
    assert neo.fft.rfftfreq(2, 1.0 / 20.0) == pytest.approx([0.0, 10.0])
    assert neo.fft.rfftfreq(2, 1.0 / 44100.0) == pytest.approx([0.0, 22050.0])


def test_hot_kernels_do_not_spill():
    """Register spills of the built kernels, read from libneo_hip.so's code objects
    (tools/spill_check.py, no GPU): the streaming step's kernels, the plain step, the offline
    windows, the FFT and the latency-mode kernels spill nothing. Only the flat-load batched-MAC
    fallback (variant 0, used where buffer loads are not available) and the one-window offline
    pass may; a second inlined copy of the slice roles once made k_lvl_slices spill 104 VGPRs
    (-12 % at c5full, profiles/r6_ab_slice_queue.json)."""
    import shutil

    if not shutil.which("/opt/rocm/lib/llvm/bin/llvm-readelf"):
        pytest.skip("llvm tools not available")
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import spill_check

    k = spill_check.kernels(os.path.join(REPO, "neo-dsp_amd", "lib", "libneo_hip.so"))
    assert len(k) > 100
    hot = [n for n in k if any(s in n for s in ("k_lvl_slices", "k_lvl_block", "k_lvl_step", "k_lvl_persist",
                                                  "k_plain_persist", "k_upols_step", "k_off_macILi2", "k_c2c_lds",
                                                  "k_lvf_filter", "k_batch_window", "k_batch_finish"))]
    assert len(hot) > 50
    bad = {n: k[n] for n in hot if k[n]["vgpr_spill"] or k[n]["scratch"]}
    assert not bad, bad
    allowed = ("k_batch_macILi", "k_off_macILi1")
    other = {n: v for n, v in k.items() if (v["vgpr_spill"] or v["scratch"]) and not any(a in n for a in allowed)}
    assert not other, other
