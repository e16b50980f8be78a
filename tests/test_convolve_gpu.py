"""GPU parity of the one-shot convolutions (neo.convolve: fft_convolve / direct_convolve)
against the CPU restatement, the golden fixture and the reference's Python tests."""
import os

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("n,m", [(2, 2), (3, 9), (10, 4), (128, 7), (555, 10), (1000, 333), (70000, 5000),
                                 (1 << 16, 1 << 16)])
def test_fft_convolve_vs_oracle(neo_gpu, oracle, n, m):
    x, p = oracle.noise(n + 1, n), oracle.noise(m + 2, m)
    y = neo_gpu.fft_convolve(x, p)
    assert y.shape == (n + m - 1,)
    assert peak_err(y, oracle.fft_convolve(x, p)) <= 1e-5


@pytest.mark.parametrize("n,m", [(2, 2), (3, 9), (10, 4), (128, 7), (555, 10), (1000, 333), (4000, 3000)])
def test_direct_convolve_bit_exact(neo_gpu, oracle, n, m):
    x, p = oracle.noise(n + 3, n), oracle.noise(m + 4, m)
    assert np.array_equal(neo_gpu.direct_convolve(x, p), oracle.direct_convolve(x, p))


def test_golden_convolve(neo_gpu):
    g = np.load(os.path.join(GOLD, "convolve_5000x777_seed9.npz"))
    assert peak_err(neo_gpu.fft_convolve(g["signal"], g["patch"]), g["fft"]) <= 1e-5
    assert np.array_equal(neo_gpu.direct_convolve(g["signal"], g["patch"]), g["direct"])


@pytest.mark.parametrize("method", ["direct", "fft"])
@pytest.mark.parametrize("signal_size", [2, 3, 4, 5, 6, 7, 8, 9, 10, 128, 555])
@pytest.mark.parametrize("patch_size", [2, 3, 4, 5, 6, 7, 8, 9, 10])
def test_python_convolve_contract(neo_gpu, method, signal_size, patch_size):
    """extra/python/test/test.py:21-39 (float32: the GPU path's dtype)."""
    rng = np.random.default_rng(signal_size * 100 + patch_size)
    signal = rng.random(signal_size).astype(np.float32)
    patch = np.zeros(patch_size, dtype=np.float32)
    patch[0] = 1.0
    convolved = neo_gpu.convolve(signal, patch, method=method)
    assert convolved.shape[0] == signal.shape[0] + patch.shape[0] - 1
    assert convolved[:signal_size] == pytest.approx(signal, abs=1e-6)
    with pytest.raises(RuntimeError):
        neo_gpu.convolve(signal, patch, mode="valid")
    with pytest.raises(RuntimeError):
        neo_gpu.convolve(signal, patch, mode="same")


def test_convolve_edge_cases(neo_gpu):
    assert neo_gpu.fft_convolve(np.zeros(0, np.float32), np.ones(3, np.float32)).shape == (0,)
    assert neo_gpu.fft_convolve(np.ones(4), np.ones(2)).dtype == np.float64  # double overload
    assert neo_gpu.fft_convolve(np.ones(4, np.float32), np.ones(2)).dtype == np.float32  # mixed: converts
    with pytest.raises(RuntimeError):
        neo_gpu.convolve(np.ones((2, 2), np.float32), np.ones(2, np.float32))


@pytest.mark.parametrize("method", ["direct", "fft"])
@pytest.mark.parametrize("signal_size", [2, 3, 4, 5, 6, 7, 8, 9, 10, 128, 555])
@pytest.mark.parametrize("patch_size", [2, 3, 4, 5, 6, 7, 8, 9, 10])
def test_reference_python_convolve_float64(neo_gpu, method, signal_size, patch_size):
    """extra/python/test/test.py:21-39 exactly as written there (dtype float64)."""
    signal = np.random.default_rng(signal_size * 31 + patch_size).random(signal_size).astype(np.float64)
    patch = np.zeros(patch_size, dtype=np.float64)
    patch[0] = 1.0
    convolved = neo_gpu.convolve(signal, patch, method=method)
    assert convolved.dtype == np.float64
    assert convolved.shape[0] == signal.shape[0] + patch.shape[0] - 1
    assert convolved[:signal_size] == pytest.approx(signal)
    with pytest.raises(RuntimeError):
        neo_gpu.convolve(signal, patch, mode="valid")
    with pytest.raises(RuntimeError):
        neo_gpu.convolve(signal, patch, mode="same")


@pytest.mark.parametrize("n,m", [(2, 2), (3, 9), (10, 4), (128, 7), (555, 10), (1000, 333), (70000, 5000)])
def test_convolve_f64_vs_oracle(neo_gpu, oracle, n, m):
    """double overloads: direct bit-identical to the double restatement (same loop order,
    no FMA), fft within 1e-12 peak-normalized."""
    rng = np.random.default_rng(n * 7 + m)
    x, p = rng.random(n) * 2 - 1, rng.random(m) * 2 - 1
    if n * m <= 2_000_000:
        d = neo_gpu.direct_convolve(x, p)
        assert d.dtype == np.float64
        assert np.array_equal(d, oracle.direct_convolve_f64(x, p))
    f = neo_gpu.fft_convolve(x, p)
    assert f.dtype == np.float64
    assert peak_err(f, oracle.fft_convolve_f64(x, p)) <= 1e-12
