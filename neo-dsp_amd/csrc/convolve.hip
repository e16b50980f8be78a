// convolve.hip — one-shot transforms built on the FFT plans: full linear convolution
// (fft_convolve, direct_convolve; the reference's Python `neo.convolve` methods,
// extra/python/src/neo/__init__.py:43-48 -> main.cpp:169-198) and the STFT
// (stft_plan, src/neo/fft/stft.hpp:40-109, the general form of uniform_partition).
//
//   fft_convolve    (src/neo/convolution/fft_convolver.hpp:19-93): zero-pad both inputs
//                   to N = 2^next_order(n+m-1), r2c both (one batched plan), complex
//                   product, c2r, 1/N, keep n+m-1 samples.
//   direct_convolve (src/neo/convolution/direct_convolve.hpp:14-56): one lane per output
//                   sample, the reference's loop order and float accumulation (no FMA),
//                   so results are bit-identical to the reference's scalar loop.
#include "common.hpp"

#include <algorithm>
#include <cmath>
#include <vector>
#include <type_traits>

namespace neo_hip {

// rows [2][N]: row 0 = signal zero-padded, row 1 = patch zero-padded
template<class R>
__global__ void k_pad2(const R* __restrict__ a, int64_t n, const R* __restrict__ b, int64_t m, R* __restrict__ rows,
                       int64_t N)
{
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < 2 * N; i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t r = i / N, k = i - r * N;
        rows[i] = r == 0 ? (k < n ? a[k] : R(0)) : (k < m ? b[k] : R(0));
    }
}

// spectra [2][bins]: row 0 *= row 1 (algorithm/multiply.hpp: out = x * y)
template<class C>
__global__ void k_spectral_multiply(C* __restrict__ spec, int64_t bins)
{
    for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < bins; k += int64_t(gridDim.x) * blockDim.x)
        spec[k] = cmul(spec[k], spec[bins + k]);
}

template<class R>
__global__ void k_scale_copy(const R* __restrict__ in, R* __restrict__ out, int64_t len, R scale)
{
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < len; i += int64_t(gridDim.x) * blockDim.x)
        out[i] = in[i] * scale;
}

// direct_convolve.hpp:14-56: with (a, na) the longer input and (b, nb) the shorter,
// out[k] = sum_{m} a[m] * b[k - m], m ascending, accumulated in R (float or double).
template<class R>
__global__ void k_direct_convolve(const R* __restrict__ a, int64_t na, const R* __restrict__ b, int64_t nb,
                                  R* __restrict__ out)
{
#pragma clang fp contract(off)  // product then sum, two roundings, like the reference (no FMA)
    const int64_t mm = na + nb - 1;
    for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < mm; k += int64_t(gridDim.x) * blockDim.x) {
        int64_t lo, hi;  // m range
        if (k < nb) {
            lo = 0;
            hi = k + 1;
        } else {
            lo = k - nb + 1;  // i in the reference
            hi = std::min(nb + lo, na);
        }
        R acc = R(0);
        for (int64_t mi = lo; mi < hi; ++mi) {
            const R prod = a[mi] * b[k - mi];  // contract(off): not fused with the add
            acc = acc + prod;
        }
        out[k] = acc;
    }
}

// stft_plan::operator() framing (stft.hpp:56-99): frame f of channel c starts at f*hop,
// takes min(L - start, frame) samples, zero-pads to N and multiplies by window[0, N)
// (the reference multiplies the whole zero-padded buffer, :92); rows [C][F][N].
template<class R>
__global__ void k_stft_frames(const R* __restrict__ x, int64_t L, int64_t F, int64_t frame, int64_t hop, int64_t N,
                              const R* __restrict__ window, R* __restrict__ rows, int64_t total)
{
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t n = i % N, cf_ = i / N, f = cf_ % F, c = cf_ / F;
        const int64_t start = f * hop;
        const int64_t cnt = L - start < frame ? L - start : frame;
        const R v = n < cnt ? x[c * L + start + n] : R(0);
        rows[i] = v * window[n];
    }
}

unsigned grid_for(int64_t n) { return unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192))); }

template<class R>
struct device_buffers {
    const R* a = nullptr;
    const R* b = nullptr;
    R* out = nullptr;
    R* tmp_a = nullptr;
    R* tmp_b = nullptr;
    R* tmp_out = nullptr;
    ~device_buffers()
    {
        dfree(tmp_a);  // pooled (dmem.hip): no device-wide wait; the caller joined its stream
        dfree(tmp_b);
        dfree(tmp_out);
    }
    int stage(const R* ha, int64_t n, const R* hb, int64_t m, R* hout, int is_device, hipStream_t s)
    {
        if (is_device) {
            a = ha;
            b = hb;
            out = hout;
            return NEO_HIP_OK;
        }
        if (int rc = dalloc(&tmp_a, size_t(n) * sizeof(R))) return rc;
        if (int rc = dalloc(&tmp_b, size_t(m) * sizeof(R))) return rc;
        if (int rc = dalloc(&tmp_out, size_t(n + m - 1) * sizeof(R))) return rc;
        NEO_HIP_CHECK(hipMemcpyAsync(tmp_a, ha, size_t(n) * sizeof(R), hipMemcpyHostToDevice, s));
        NEO_HIP_CHECK(hipMemcpyAsync(tmp_b, hb, size_t(m) * sizeof(R), hipMemcpyHostToDevice, s));
        a = tmp_a;
        b = tmp_b;
        out = tmp_out;
        return NEO_HIP_OK;
    }
};

template<class R>
int fft_convolve_impl(const R* signal, int64_t n, const R* patch, int64_t m, R* out, int is_device, int device)
{
    using C = std::conditional_t<sizeof(R) == 8, cd, cf>;
    const int f64 = sizeof(R) == 8 ? NEO_HIP_F64 : 0;
    if (n < 0 || m < 0) return fail(NEO_HIP_EINVAL, "negative length");
    if (n == 0 || m == 0) return NEO_HIP_OK;  // fft_convolver.hpp:80-82: empty result
    if (!signal || !patch || !out) return fail(NEO_HIP_EINVAL, "null buffer");
    const int64_t len = n + m - 1;
    int order = 0;
    while ((int64_t(1) << order) < len) ++order;
    if (order > 27) return fail(NEO_HIP_EINVAL, "convolution of %lld samples exceeds the max FFT order 27", (long long)len);
    device_guard g(device);
    if (g.rc) return g.rc;
    const int64_t N = int64_t(1) << order, bins = N / 2 + 1;
    if (is_device)
        if (int rj = null_join()) return rj;  // after its producer (common.hpp: null_join)
    hipStream_t s = nullptr;
    if (int rs = shared_stream(&s)) return rs;  // one of the device's four (dmem.hip)
    int rc = NEO_HIP_OK;
    neo_hip_fft_plan *r2c = nullptr, *c2r = nullptr;
    R* rows = nullptr;
    C* spec = nullptr;
    {
        device_buffers<R> io;
        rc = io.stage(signal, n, patch, m, out, is_device, s);
        if (!rc) rc = neo_hip_fft_plan_create(order, 2, NEO_HIP_R2C | f64, device, &r2c);
        if (!rc) rc = neo_hip_fft_plan_create(order, 1, NEO_HIP_C2R | f64, device, &c2r);
        if (!rc && (dalloc(&rows, size_t(2 * N) * sizeof(R)) || dalloc(&spec, size_t(2 * bins) * sizeof(C))))
            rc = fail(NEO_HIP_ENOMEM, "convolution buffers");
        if (!rc) {
            hipLaunchKernelGGL((k_pad2<R>), dim3(grid_for(2 * N)), dim3(256), 0, s, io.a, n, io.b, m, rows, N);
            rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "pad launch failed");
        }
        if (!rc) rc = neo_hip_fft_execute(r2c, rows, spec, -1, s);
        if (!rc) {
            hipLaunchKernelGGL((k_spectral_multiply<C>), dim3(grid_for(bins)), dim3(256), 0, s, spec, bins);
            rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "multiply launch failed");
        }
        if (!rc) rc = neo_hip_fft_execute(c2r, spec, rows, +1, s);
        if (!rc) {
            hipLaunchKernelGGL((k_scale_copy<R>), dim3(grid_for(len)), dim3(256), 0, s, rows, io.out, len,
                               R(1) / R(N));  // fft_convolver.hpp:66-70
            rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "scale launch failed");
        }
        if (!rc && !is_device &&
            hipMemcpyAsync(out, io.out, size_t(len) * sizeof(R), hipMemcpyDeviceToHost, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    }
    neo_hip_fft_plan_destroy(r2c);
    neo_hip_fft_plan_destroy(c2r);
    dfree(rows);
    dfree(spec);
    return rc;
}

template<class R>
int direct_convolve_impl(const R* signal, int64_t n, const R* patch, int64_t m, R* out, int is_device, int device)
{
    if (n < 0 || m < 0) return fail(NEO_HIP_EINVAL, "negative length");
    if (n == 0 || m == 0) return NEO_HIP_OK;
    if (!signal || !patch || !out) return fail(NEO_HIP_EINVAL, "null buffer");
    device_guard g(device);
    if (g.rc) return g.rc;
    if (is_device)
        if (int rj = null_join()) return rj;  // after its producer (common.hpp: null_join)
    hipStream_t s = nullptr;
    if (int rs = shared_stream(&s)) return rs;  // one of the device's four (dmem.hip)
    int rc = NEO_HIP_OK;
    {
        device_buffers<R> io;
        rc = io.stage(signal, n, patch, m, out, is_device, s);
        if (!rc) {
            const bool sig_long = n >= m;  // direct_convolve.hpp:22 vs :35
            hipLaunchKernelGGL((k_direct_convolve<R>), dim3(grid_for(n + m - 1)), dim3(256), 0, s,
                               sig_long ? io.a : io.b, sig_long ? n : m, sig_long ? io.b : io.a, sig_long ? m : n,
                               io.out);
            rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "direct launch failed");
        }
        if (!rc && !is_device &&
            hipMemcpyAsync(out, io.out, size_t(n + m - 1) * sizeof(R), hipMemcpyDeviceToHost, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
        if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    }
    return rc;
}

// detail::num_sftf_frames (stft.hpp:21-25): idiv(L - frame + overlap, frame - overlap) + 1,
// clamped to one frame where the reference's unsigned arithmetic would underflow
int64_t stft_frames(int64_t L, int64_t frame, int64_t overlap)
{
    const int64_t hop = frame - overlap;
    if (L <= frame) return 1;
    return (L - frame + overlap + hop - 1) / hop + 1;
}

template<class R>
int stft_impl(const R* x, int channels, int64_t length, int frame, int transform, int overlap, const R* window,
              void* out, int is_device, int device)
{
    using C = std::conditional_t<sizeof(R) == 8, cd, cf>;
    const int f64 = sizeof(R) == 8 ? NEO_HIP_F64 : 0;
    if (!x || !out || channels < 1 || length < 1 || frame < 1 || transform < 1 || overlap < 0 || overlap >= frame)
        return fail(NEO_HIP_EINVAL, "bad stft arguments");
    int order = 0;
    while ((int64_t(1) << order) < transform) ++order;  // rfft_plan{from_order, next_order(transform_size)}
    const int64_t N = int64_t(1) << order, bins = N / 2 + 1;
    if (frame > N) return fail(NEO_HIP_EINVAL, "frame_size %d exceeds the transform size %lld", frame, (long long)N);
    if (order > 27) return fail(NEO_HIP_EINVAL, "transform size exceeds max order 27");
    const int64_t F = stft_frames(length, frame, overlap), rows_n = int64_t(channels) * F;
    device_guard g(device);
    if (g.rc) return g.rc;
    if (is_device)
        if (int rj = null_join()) return rj;  // after its producer (common.hpp: null_join)
    hipStream_t s = nullptr;
    if (int rs = shared_stream(&s)) return rs;  // one of the device's four (dmem.hip)
    int rc = NEO_HIP_OK;
    R *d_x = nullptr, *d_w = nullptr, *rows = nullptr;
    C* d_out = static_cast<C*>(out);
    neo_hip_fft_plan* plan = nullptr;
    std::vector<R> hann;
    if (!window) {  // hann_window (windowing.hpp:29-41) over the transform size, in R
        hann.resize(size_t(N));
        const R n1 = R(N - 1), two_pi = R(3.14159265358979323846) * R(2);
        for (int64_t i = 0; i < N; ++i) hann[size_t(i)] = R(0.5) * (R(1) - std::cos(two_pi * R(i) / n1));
    }
    const size_t xbytes = size_t(channels) * size_t(length) * sizeof(R), obytes = size_t(rows_n * bins) * sizeof(C);
    if (dalloc(&rows, size_t(rows_n * N) * sizeof(R)) || dalloc(&d_w, size_t(N) * sizeof(R)) ||
        (!is_device && (dalloc(&d_x, xbytes) || dalloc(&d_out, obytes))))
        rc = fail(NEO_HIP_ENOMEM, "stft buffers");
    const R* xin = is_device ? x : d_x;
    if (!rc && !is_device && hipMemcpyAsync(d_x, x, xbytes, hipMemcpyHostToDevice, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "input copy failed");
    if (!rc && hipMemcpyAsync(d_w, window ? window : hann.data(), size_t(N) * sizeof(R),
                              window && is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "window copy failed");
    if (!rc) {
        const int64_t total = rows_n * N;
        hipLaunchKernelGGL((k_stft_frames<R>), dim3(grid_for(total)), dim3(256), 0, s, xin, length, F, int64_t(frame),
                           int64_t(frame - overlap), N, d_w, rows, total);
        rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "framing launch failed");
    }
    if (!rc) rc = neo_hip_fft_plan_create(order, rows_n, NEO_HIP_R2C | f64, device, &plan);
    if (!rc) rc = neo_hip_fft_execute(plan, rows, d_out, -1, s);
    if (!rc && !is_device && hipMemcpyAsync(out, d_out, obytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    neo_hip_fft_plan_destroy(plan);
    dfree(rows);  // the stream was joined above
    dfree(d_w);
    if (!is_device) {
        dfree(d_x);
        dfree(d_out);
    }
    return rc;
}

}  // namespace neo_hip

using namespace neo_hip;

extern "C" {

NEO_HIP_API int neo_hip_fft_convolve(const float* signal, int64_t n, const float* patch, int64_t m, float* out,
                                     int is_device, int device)
{
    return fft_convolve_impl(signal, n, patch, m, out, is_device, device);
}

NEO_HIP_API int neo_hip_fft_convolve_f64(const double* signal, int64_t n, const double* patch, int64_t m, double* out,
                                         int is_device, int device)
{
    return fft_convolve_impl(signal, n, patch, m, out, is_device, device);
}

NEO_HIP_API int neo_hip_direct_convolve(const float* signal, int64_t n, const float* patch, int64_t m, float* out,
                                        int is_device, int device)
{
    return direct_convolve_impl(signal, n, patch, m, out, is_device, device);
}

NEO_HIP_API int neo_hip_direct_convolve_f64(const double* signal, int64_t n, const double* patch, int64_t m,
                                            double* out, int is_device, int device)
{
    return direct_convolve_impl(signal, n, patch, m, out, is_device, device);
}

NEO_HIP_API int neo_hip_stft_num_frames(int64_t length, int frame_size, int overlap, int64_t* frames)
{
    if (!frames || length < 0 || frame_size < 1 || overlap < 0 || overlap >= frame_size)
        return fail(NEO_HIP_EINVAL, "bad stft arguments");
    *frames = stft_frames(length, frame_size, overlap);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_stft(const float* x, int channels, int64_t length, int frame_size, int transform_size,
                             int overlap, const float* window, void* out, int is_device, int device)
{
    return stft_impl(x, channels, length, frame_size, transform_size, overlap, window, out, is_device, device);
}

NEO_HIP_API int neo_hip_stft_f64(const double* x, int channels, int64_t length, int frame_size, int transform_size,
                                 int overlap, const double* window, void* out, int is_device, int device)
{
    return stft_impl(x, channels, length, frame_size, transform_size, overlap, window, out, is_device, device);
}

}  // extern "C"
