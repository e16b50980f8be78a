"""GPU parity of the FFT path (libneo_hip.so via the C-ABI) against the CPU
restatement of c2c_dit2_plan / fallback_rfft_plan and the golden fixtures.

Tolerance (BASELINE.json north_star, float32): peak-normalized max error
max|y - ref| / max|ref| <= 1e-5, plus the reference's own allclose abs 1e-5
(src/neo/algorithm/allclose.hpp:36-39) on round trips."""
import os

import numpy as np
import pytest

from conftest import peak_err

pytestmark = pytest.mark.gpu
TOL = 1e-5
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def cnoise(oracle, seed, shape):
    n = int(np.prod(shape))
    return oracle.noise(seed, 2 * n).view(np.complex64).reshape(shape)


@pytest.mark.parametrize("order", range(0, 15))
@pytest.mark.parametrize("direction", [-1, 1])
def test_c2c_vs_oracle(neo_gpu, oracle, order, direction):
    x = cnoise(oracle, 100 + order, (3, 1 << order))
    ref = oracle.fft(x, direction)
    y = neo_gpu.fft.fft(x) if direction < 0 else neo_gpu.fft.ifft(x, norm="forward")
    assert peak_err(y, ref) <= TOL


@pytest.mark.parametrize("order", [15, 16, 17, 20])
def test_c2c_large_vs_oracle(neo_gpu, oracle, order):
    x = cnoise(oracle, 200 + order, (1 << order,))
    for d in (-1, 1):
        ref = oracle.fft(x, d)
        y = neo_gpu.fft.fft(x) if d < 0 else neo_gpu.fft.ifft(x, norm="forward")
        assert peak_err(y, ref) <= TOL


@pytest.mark.parametrize("order", list(range(2, 15)) + [16, 18])
def test_round_trip(neo_gpu, oracle, order):
    """fft_test.cpp:79-91: fft -> ifft -> scale(1/N) == x within abs 1e-5."""
    x = cnoise(oracle, 300 + order, (1 << order,))
    y = neo_gpu.fft.ifft(neo_gpu.fft.fft(x))
    assert np.abs(y - x).max() <= 1e-5


def test_known_answer(neo_gpu):
    """rfft_test.cpp:170-186: FFT([1,2,3,4]) = [10, -2+2i, -2, -2-2i]; impulse -> ones."""
    y = neo_gpu.fft.fft(np.array([1, 2, 3, 4], np.complex64))
    np.testing.assert_allclose(y, [10, -2 + 2j, -2, -2 - 2j], atol=1e-6)
    for order in range(2, 9):
        imp = np.zeros(1 << order, np.complex64)
        imp[0] = 1
        np.testing.assert_allclose(neo_gpu.fft.fft(imp), np.ones(1 << order), atol=1e-6)


def test_python_api_contract(neo_gpu):
    """extra/python/test/test.py:10-18 and main.cpp:135-139."""
    for n in [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096]:
        assert neo_gpu.fft.fft(np.zeros(n, np.complex64)).shape == (n,)
        imp = np.zeros(n, np.complex64)
        imp[0] = 1
        assert np.allclose(neo_gpu.fft.ifft(neo_gpu.fft.fft(imp.copy())), imp)
    with pytest.raises(RuntimeError):
        neo_gpu.fft.fft(np.zeros(12, np.complex64))
    with pytest.raises(RuntimeError):
        neo_gpu.fft.FFTPlan(0, 28)  # order > max_order throws (fft_test.cpp:62-67)
    x = np.arange(8).astype(np.complex64)
    np.testing.assert_allclose(neo_gpu.fft.fft(x, norm="ortho"), np.fft.fft(x, norm="ortho"), atol=1e-5)
    np.testing.assert_allclose(neo_gpu.fft.fft(x, norm="forward"), np.fft.fft(x, norm="forward"), atol=1e-6)


def test_golden_c2c(neo_gpu):
    g = np.load(os.path.join(GOLD, "c2c_1024_seed1.npz"))
    assert peak_err(neo_gpu.fft.fft(g["x"]), g["fwd"]) <= TOL
    assert peak_err(neo_gpu.fft.ifft(g["fwd"], norm="forward"), g["bwd"]) <= TOL
    g = np.load(os.path.join(GOLD, "c2c_4096x8_seed2.npz"))
    assert peak_err(neo_gpu.fft.fft(g["x"]), g["fwd"]) <= TOL


@pytest.mark.parametrize("order", list(range(0, 15)) + [15, 17])
def test_rfft_irfft_vs_oracle(neo_gpu, oracle, order):
    n = 1 << order
    x = oracle.noise(400 + order, 2 * n).reshape(2, n)
    R = neo_gpu.fft.rfft(x)
    ref = oracle.rfft(x)
    assert R.shape == (2, n // 2 + 1)
    assert peak_err(R, ref) <= TOL
    back = neo_gpu.fft.irfft(R, n, norm="forward")  # unnormalized c2r
    assert peak_err(back, oracle.irfft(ref, n)) <= TOL
    # round trip rfft_test.cpp:40-71
    assert np.abs(back / n - x).max() <= 1e-5


def test_irfft_ignores_dc_nyquist_imag(neo_gpu, oracle):
    """fallback_rfft_plan c2r takes .real() of a Hermitian-filled buffer: Im(DC), Im(Nyq) drop out."""
    n = 256
    X = oracle.rfft(oracle.noise(7, n))
    X2 = X.copy()
    X2[0] += 0.5j
    X2[-1] -= 0.25j
    a = neo_gpu.fft.irfft(X, n, norm="forward")
    b = neo_gpu.fft.irfft(X2, n, norm="forward")
    assert peak_err(b, oracle.irfft(X2, n)) <= TOL
    assert np.abs(a - b).max() <= 1e-5 * np.abs(a).max()


@pytest.mark.parametrize("order", [4, 5, 6, 7, 8])
def test_rfft_deinterleave_cross_check(neo_gpu, oracle, order):
    """rfft_test.cpp:80-126: two reals packed into one c2c, split by rfft_deinterleave,
    equal two rffts (pins bin layout and sign convention against c2c)."""
    n = 1 << order
    a, b = oracle.noise(500, n), oracle.noise(501, n)
    z = neo_gpu.fft.fft((a + 1j * b).astype(np.complex64))
    ca, cb = oracle.rfft_deinterleave(z)
    assert np.abs(ca - neo_gpu.fft.rfft(a)).max() <= 1e-5 * n
    assert np.abs(cb - neo_gpu.fft.rfft(b)).max() <= 1e-5 * n


def test_golden_rfft(neo_gpu):
    for n in (512, 1024):
        g = np.load(os.path.join(GOLD, f"rfft_{n}_seed3.npz"))
        assert peak_err(neo_gpu.fft.rfft(g["x"]), g["r2c"]) <= TOL
        assert peak_err(neo_gpu.fft.irfft(g["r2c"], n, norm="forward"), g["c2r"]) <= TOL


def test_inplace_device(neo_gpu, oracle):
    torch = pytest.importorskip("torch")
    x = cnoise(oracle, 600, (16, 4096))
    t = torch.from_numpy(x).cuda()
    plan = neo_gpu.fft.get_plan(0, 12, 16)
    plan.execute_device(t.data_ptr(), t.data_ptr(), -1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert peak_err(t.cpu().numpy(), oracle.fft(x)) <= TOL


def test_c2_full_shape_properties(neo_gpu, oracle):
    """C2 (4096 x 65536) at full size: spot rows vs the oracle, the round trip, Parseval,
    and linearity hold on every transform (size-independent checks)."""
    torch = pytest.importorskip("torch")
    B, N = 65536, 4096
    g = torch.Generator(device="cuda").manual_seed(2)
    x = (torch.rand((B, N, 2), generator=g, device="cuda") * 2 - 1).contiguous()
    xc = torch.view_as_complex(x)
    y = neo_gpu.fft.fft(xc)
    rows = [0, 1, 4095, 32768, 65535]
    for r in rows:
        ref = oracle.fft(xc[r].cpu().numpy())
        assert peak_err(y[r].cpu().numpy(), ref) <= TOL
    e_x = (xc.abs() ** 2).sum(dim=1).double()
    e_y = (y.abs() ** 2).sum(dim=1).double() / N
    assert torch.max(torch.abs(e_y / e_x - 1)).item() < 1e-5
    back = neo_gpu.fft.ifft(y)
    assert torch.max(torch.abs(back - xc)).item() < 1e-5
    y2 = neo_gpu.fft.fft(xc * 2 + xc.conj())
    lin = y * 2 + neo_gpu.fft.fft(xc.conj())
    assert (torch.max(torch.abs(y2 - lin)) / torch.max(torch.abs(lin))).item() < 1e-5


# ------------------------------------------------------------------ double precision
TOL64 = 1e-12  # complex<double> / double plans: peak-normalized vs the double restatement


@pytest.mark.parametrize("order", list(range(0, 15)) + [15, 17, 20])
@pytest.mark.parametrize("direction", [-1, 1])
def test_c2c_f64_vs_oracle(neo_gpu, oracle, order, direction):
    """fft_plan<complex<double>> (the reference's double instantiation; Python complex128)."""
    rng = np.random.default_rng(700 + order)
    x = (rng.random((2, 1 << order)) * 2 - 1) + 1j * (rng.random((2, 1 << order)) * 2 - 1)
    ref = oracle.fft_f64(x, direction)
    y = neo_gpu.fft.fft(x) if direction < 0 else neo_gpu.fft.ifft(x, norm="forward")
    assert y.dtype == np.complex128
    assert peak_err(y, ref) <= TOL64


def test_python_api_contract_complex128(neo_gpu):
    """extra/python/test/test.py:10-18 with complex=np.complex128, and the pybind11 overload
    rule: complex64 / complex128 keep their precision, other dtypes convert to complex64."""
    for n in [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096]:
        z = neo_gpu.fft.fft(np.zeros(n, np.complex128))
        assert z.shape == (n,) and z.dtype == np.complex128
        imp = np.zeros(n, np.complex128)
        imp[0] = 1
        assert np.allclose(neo_gpu.fft.ifft(neo_gpu.fft.fft(imp.copy())), imp)
    assert neo_gpu.fft.fft(np.zeros(8)).dtype == np.complex64        # float64 real: converted
    assert neo_gpu.fft.fft(np.zeros(8, np.complex64)).dtype == np.complex64
    x = np.arange(8).astype(np.complex128)
    np.testing.assert_allclose(neo_gpu.fft.fft(x, norm="ortho"), np.fft.fft(x, norm="ortho"), atol=1e-13)


@pytest.mark.parametrize("order", list(range(0, 15)) + [15, 17])
def test_rfft_irfft_f64_vs_oracle(neo_gpu, oracle, order):
    n = 1 << order
    x = np.random.default_rng(800 + order).random(n) * 2 - 1
    X = neo_gpu.fft.rfft(x)
    assert X.dtype == np.complex128
    assert peak_err(X, oracle.rfft_f64(x)) <= TOL64
    back = neo_gpu.fft.irfft(X, n, norm="forward")  # unnormalized, like the plan
    assert back.dtype == np.float64
    assert peak_err(back, oracle.irfft_f64(X, n)) <= TOL64


def test_c2c_f64_device_tensor(neo_gpu, oracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(900)
    x = rng.random((4, 4096)) + 1j * rng.random((4, 4096))
    t = torch.from_numpy(x).cuda()
    y = neo_gpu.fft.fft(t)
    torch.cuda.synchronize()
    assert y.dtype == torch.complex128
    assert peak_err(y.cpu().numpy(), oracle.fft_f64(x, -1)) <= TOL64


def test_max_order_round_trips(neo_gpu):
    """The largest plan the reference allows (order 27 = max_order(), c2c_dit2_plan.hpp:58-61):
    size-independent properties at full size — forward then backward gives N·x (c2c and
    real), Parseval, and an impulse transforms to all ones."""
    torch = pytest.importorskip("torch")
    order, n = 27, 1 << 27
    g = torch.Generator(device="cuda").manual_seed(27)
    x = torch.complex(torch.rand(n, generator=g, device="cuda") * 2 - 1,
                      torch.rand(n, generator=g, device="cuda") * 2 - 1)
    plan = neo_gpu.fft.FFTPlan(0, order, 1)
    X = torch.empty_like(x)
    plan.execute_device(x.data_ptr(), X.data_ptr(), -1, torch.cuda.current_stream().cuda_stream)
    y = torch.empty_like(x)
    plan.execute_device(X.data_ptr(), y.data_ptr(), +1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    err = ((y / n - x).abs().max() / x.abs().max()).item()
    assert err <= 1e-5, err
    ex = (x.abs() ** 2).double().sum().item()
    eX = (X.abs() ** 2).double().sum().item() / n
    assert abs(eX - ex) / ex <= 1e-5  # Parseval
    d = torch.zeros_like(x)
    d[0] = 1
    plan.execute_device(d.data_ptr(), X.data_ptr(), -1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (X - 1).abs().max().item() <= 1e-6
    del x, X, y, d
    # real: r2c + c2r of 2^27 reals
    r = torch.rand(n, generator=g, device="cuda") * 2 - 1
    R = torch.empty(n // 2 + 1, dtype=torch.complex64, device="cuda")
    back = torch.empty_like(r)
    neo_gpu.fft.FFTPlan(1, order, 1).execute_device(r.data_ptr(), R.data_ptr(), -1, 0)
    neo_gpu.fft.FFTPlan(2, order, 1).execute_device(R.data_ptr(), back.data_ptr(), +1, 0)
    torch.cuda.synchronize()
    assert ((back / n - r).abs().max() / r.abs().max()).item() <= 1e-5


# ------------------------------------------------------------------ STFT (stft.hpp:40-125)
@pytest.mark.parametrize("length", [2040, 2048])
def test_stft_reference_shapes(neo_gpu, length):
    """stft_test.cpp:15-37: no overlap -> 8 x 129, stft(x, 256) (half overlap) -> 16 x 129."""
    x = np.zeros((1, length), np.float32)
    assert neo_gpu.fft.stft(x, 256, 256, 0).shape == (1, 8, 129)
    assert neo_gpu.fft.stft(x, 256).shape == (1, 16, 129)
    assert neo_gpu.fft.stft(x.astype(np.float64), 256).shape == (1, 16, 129)


@pytest.mark.parametrize("C,L,frame,transform,overlap", [(1, 2040, 256, 256, 128), (3, 5000, 300, 512, 100),
                                                         (2, 100, 64, 64, 0), (1, 48000, 1024, 2048, 512),
                                                         (2, 10, 16, 16, 8)])
@pytest.mark.parametrize("window", ["hann", "rectangular", "custom"])
def test_stft_vs_oracle(neo_gpu, oracle, C, L, frame, transform, overlap, window):
    x = np.stack([oracle.noise(900 + c, L) for c in range(C)])
    N = 1 << (transform - 1).bit_length()
    if window == "hann":
        w, arg = oracle.hann(N), "hann"
    elif window == "rectangular":
        w = np.ones(N, np.float32)
        arg = "rectangular"
    else:
        w = (oracle.noise(77, N) * 0.5 + 1).astype(np.float32)
        arg = w
    got = neo_gpu.fft.stft(x, frame, transform, overlap, window=arg)
    ref = oracle.stft(x, frame, transform, overlap, w)
    assert got.shape == ref.shape
    assert peak_err(got, ref) <= TOL


def test_stft_f64(neo_gpu, oracle):
    rng = np.random.default_rng(5)
    x = rng.random((2, 3000)) * 2 - 1
    got = neo_gpu.fft.stft(x, 256, 512, 64, window="rectangular")
    assert got.dtype == np.complex128
    F = got.shape[1]
    truth = np.empty_like(got)
    for c in range(2):
        for f in range(F):
            seg = x[c, f * 192:f * 192 + 256]
            truth[c, f] = np.fft.rfft(np.pad(seg, (0, 512 - len(seg))))
    assert peak_err(got, truth) <= 1e-12


def test_uniform_partition_is_a_rectangular_stft(neo_gpu, oracle):
    """uniform_partition.hpp:12-26 = stft(frame B, transform 2B, overlap 0, rectangular)."""
    ir = np.stack([oracle.noise(950 + c, 3000) for c in range(2)])
    H = neo_gpu.uniform_partition(ir, 256)
    S = neo_gpu.fft.stft(ir, 256, 512, 0, window="rectangular")
    assert H.shape == S.shape
    assert peak_err(H, S) <= TOL
