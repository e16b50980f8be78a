// overlap.hip — the standalone overlap stages of neo::convolution on MI355X: overlap_save
// (src/neo/convolution/overlap_save.hpp:19-112) and overlap_add (overlap_add.hpp:23-107) for
// any filter size F, batched over C independent channels. The convolvers fuse this stage into
// their step kernels; these entry points expose it on its own, with the reference's
// operator()(block, callback) split at the callback: forward (window + r2c -> the n/2 + 1 bins
// the callback sees) and inverse (c2r, 1/n, output block).
//
// Transform size n = 2^next_order(B + F - 1) (overlap_save.hpp:53; overlap_add.hpp:43-46 with
// output_size<full>(B, F) = B + F - 1). Per call, as the reference:
//   overlap_save  slide the n-sample window left by B (slide_window_left, :37-49), the block
//                 into window[n - B, n), rfft; inverse: irfft into a separate real buffer, 1/n,
//                 real[n - B, n) -> block (:98-111)
//   overlap_add   block -> window[0, B), window[B, 2B) = 0 (only that "padding": window[2B, n)
//                 keeps the previous irfft output), rfft; inverse: irfft back INTO the window,
//                 1/n, block = window[0, B) + overlap, overlap = window[B, 2B) (:79-106)
#include "common.hpp"

#include <cstring>

namespace neo_hip {
namespace {

// overlap_save window slide, out of place (double-buffered windows): nw = ow[B, n) | block
__global__ __launch_bounds__(256) void k_ols_window(const float* __restrict__ ow, float* __restrict__ nw,
                                                   const float* __restrict__ in, int64_t ld_in, int64_t n, int64_t B,
                                                   int64_t total)
{
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int64_t c = g / n, i = g - c * n;
        nw[g] = i < n - B ? ow[g + B] : in[c * ld_in + (i - (n - B))];
    }
}

// overlap_add window: block -> [0, B), zeros -> [B, min(2B, n)), the rest kept
__global__ __launch_bounds__(256) void k_ola_window(float* __restrict__ w, const float* __restrict__ in,
                                                   int64_t ld_in, int64_t n, int64_t B, int64_t total)
{
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int64_t c = g / n, i = g - c * n;
        if (i < B) w[g] = in[c * ld_in + i];
        else if (i < 2 * B) w[g] = 0.f;
    }
}

// overlap_save output: out = real[n - B, n) * (1/n) (scale.hpp:14-28 multiplies by the float 1/n)
__global__ __launch_bounds__(256) void k_ols_out(const float* __restrict__ real, float* __restrict__ out, int64_t ld_out,
                                                int64_t n, int64_t B, float scale, int64_t total)
{
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int64_t c = g / B, i = g - c * B;
        out[c * ld_out + i] = real[c * n + (n - B) + i] * scale;
    }
}

// overlap_add output over the n samples of each window (thread i < B takes the pair i, i + B):
// window *= 1/n, out = window[0, B) + overlap, overlap = window[B, 2B)
__global__ __launch_bounds__(256) void k_ola_out(float* __restrict__ w, float* __restrict__ ov, float* __restrict__ out,
                                                int64_t ld_out, int64_t n, int64_t B, float scale, int64_t total)
{
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int64_t c = g / n, i = g - c * n;
        float* wc = w + c * n;
        if (i < B) {
            const float a = wc[i] * scale;
            wc[i] = a;
            out[c * ld_out + i] = a + ov[c * B + i];
            if (2 * B <= n) {
                const float b = wc[i + B] * scale;
                wc[i + B] = b;
                ov[c * B + i] = b;
            }
        } else if (i >= 2 * B) {
            wc[i] *= scale;
        }
    }
}

unsigned grid_for(int64_t total) { return unsigned(std::min<int64_t>((total + 255) / 256, 8192)); }

}  // namespace
}  // namespace neo_hip

struct neo_hip_overlap {
    int device = 0, kind = 0, C = 0, order = 0;
    int64_t B = 0, F = 0, n = 0, bins = 0;
    neo_hip_fft_plan* r2c = nullptr;
    neo_hip_fft_plan* c2r = nullptr;
    hipStream_t stream = nullptr;
    float* win[2] = {};        // [C][n] windows (overlap_save: double-buffered slide)
    int cur = 0;               // overlap_save: the current window
    float* real = nullptr;     // [C][n] overlap_save irfft target
    float* ov = nullptr;       // [C][B] overlap_add tail
    neo_hip::cf* spec = nullptr;  // [C][bins] device spectrum (host-memory calls)
    float* io = nullptr;          // [C][B] device block (host-memory calls)
    neo_hip::stream_set used;     // streams the device-memory calls ran on (reset and destroy join them)
};

namespace {
using neo_hip::fail;

void destroy_overlap(neo_hip_overlap* h)
{
    if (!h) return;
    if (h->r2c) neo_hip_fft_plan_destroy(h->r2c);
    if (h->c2r) neo_hip_fft_plan_destroy(h->c2r);
    for (float* w : h->win) neo_hip::dfree(w);  // pooled (dmem.hip): no device-wide wait
    neo_hip::dfree(h->real);
    neo_hip::dfree(h->ov);
    neo_hip::dfree(h->spec);
    neo_hip::dfree(h->io);
    // h->stream is one of the device's shared streams (dmem.hip)
    delete h;
}

int reset_overlap(neo_hip_overlap* h)
{
    const size_t wb = size_t(h->C) * size_t(h->n) * sizeof(float);
    for (float* w : h->win)
        if (w) NEO_HIP_CHECK(hipMemsetAsync(w, 0, wb, h->stream));
    if (h->ov) NEO_HIP_CHECK(hipMemsetAsync(h->ov, 0, size_t(h->C) * size_t(h->B) * sizeof(float), h->stream));
    h->cur = 0;
    NEO_HIP_CHECK(hipStreamSynchronize(h->stream));
    return NEO_HIP_OK;
}

int forward_dev(neo_hip_overlap* h, const float* in, int64_t ld_in, void* spec, hipStream_t s)
{
    const int64_t total = int64_t(h->C) * h->n;
    float* w;
    if (h->kind == 0) {
        w = h->win[h->cur ^ 1];
        hipLaunchKernelGGL(neo_hip::k_ols_window, dim3(neo_hip::grid_for(total)), dim3(256), 0, s, h->win[h->cur], w, in,
                           ld_in, h->n, h->B, total);
        h->cur ^= 1;
    } else {
        w = h->win[0];
        hipLaunchKernelGGL(neo_hip::k_ola_window, dim3(neo_hip::grid_for(total)), dim3(256), 0, s, w, in, ld_in, h->n,
                           h->B, total);
    }
    NEO_HIP_LAUNCH_CHECK();
    return neo_hip_fft_execute(h->r2c, w, spec, -1, s);
}

int inverse_dev(neo_hip_overlap* h, const void* spec, float* out, int64_t ld_out, hipStream_t s)
{
    const float scale = 1.0f / float(h->n);
    if (h->kind == 0) {
        if (int rc = neo_hip_fft_execute(h->c2r, spec, h->real, 1, s)) return rc;
        const int64_t total = int64_t(h->C) * h->B;
        hipLaunchKernelGGL(neo_hip::k_ols_out, dim3(neo_hip::grid_for(total)), dim3(256), 0, s, h->real, out, ld_out,
                           h->n, h->B, scale, total);
    } else {
        if (int rc = neo_hip_fft_execute(h->c2r, spec, h->win[0], 1, s)) return rc;
        const int64_t total = int64_t(h->C) * h->n;
        hipLaunchKernelGGL(neo_hip::k_ola_out, dim3(neo_hip::grid_for(total)), dim3(256), 0, s, h->win[0], h->ov, out,
                           ld_out, h->n, h->B, scale, total);
    }
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}
}  // namespace

extern "C" {

NEO_HIP_API int neo_hip_overlap_create(int kind, int channels, int64_t block, int64_t filter, int device,
                                       neo_hip_overlap** out)
{
    if (!out) return fail(NEO_HIP_EINVAL, "handle pointer is null");
    *out = nullptr;
    if (kind != 0 && kind != 1) return fail(NEO_HIP_EINVAL, "kind must be 0 (overlap_save) or 1 (overlap_add)");
    if (channels < 1) return fail(NEO_HIP_EINVAL, "channels must be >= 1");
    if (block < 1 || (block & (block - 1))) return fail(NEO_HIP_EINVAL, "block must be a power of two, got %lld", (long long)block);
    if (filter < 1) return fail(NEO_HIP_EINVAL, "filter size must be >= 1");
    int order = 0;
    while ((int64_t(1) << order) < block + filter - 1) ++order;  // next_order = log2(bit_ceil)
    if (order > neo_hip_fft_max_order())
        return fail(NEO_HIP_EINVAL, "transform size 2^%d for block %lld + filter %lld exceeds max_order %d", order,
                    (long long)block, (long long)filter, neo_hip_fft_max_order());
    neo_hip::device_guard g(device);
    if (g.rc) return g.rc;
    auto* h = new neo_hip_overlap{};
    (void)hipGetDevice(&h->device);
    h->kind = kind;
    h->C = channels;
    h->B = block;
    h->F = filter;
    h->order = order;
    h->n = int64_t(1) << order;
    h->bins = h->n / 2 + 1;
    const size_t wb = size_t(channels) * size_t(h->n) * sizeof(float);
    int rc = NEO_HIP_OK;
    if (int rs = neo_hip::shared_stream(&h->stream)) rc = rs;
    if (!rc) rc = neo_hip_fft_plan_create(order, channels, NEO_HIP_R2C, h->device, &h->r2c);
    if (!rc) rc = neo_hip_fft_plan_create(order, channels, NEO_HIP_C2R, h->device, &h->c2r);
    if (!rc && (neo_hip::dalloc(&h->win[0], wb) ||
                (kind == 0 && (neo_hip::dalloc(&h->win[1], wb) || neo_hip::dalloc(&h->real, wb))) ||
                (kind == 1 && neo_hip::dalloc(&h->ov, size_t(channels) * size_t(block) * sizeof(float)))))
        rc = fail(NEO_HIP_ENOMEM, "device allocation of the overlap stage failed");
    if (!rc) rc = reset_overlap(h);
    if (rc) {
        destroy_overlap(h);
        return rc;
    }
    *out = h;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_overlap_destroy(neo_hip_overlap* h)
{
    if (!h) return NEO_HIP_OK;
    neo_hip::device_guard g(h->device);
    (void)h->used.join();  // this handle's calls on any stream, not the device
    (void)hipStreamSynchronize(h->stream);
    destroy_overlap(h);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_overlap_info(neo_hip_overlap* h, int64_t* block, int64_t* filter, int64_t* transform_size)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (block) *block = h->B;
    if (filter) *filter = h->F;
    if (transform_size) *transform_size = h->n;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_overlap_reset(neo_hip_overlap* h)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    neo_hip::device_guard g(h->device);
    if (g.rc) return g.rc;
    if (int rc = h->used.join()) return rc;  // this handle's calls on any stream, not the device
    return reset_overlap(h);
}

NEO_HIP_API int neo_hip_overlap_forward(neo_hip_overlap* h, const float* in, int64_t ld_in, void* spectrum,
                                        int is_device, void* stream)
{
    if (!h || !in || !spectrum) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (ld_in < h->B) return fail(NEO_HIP_EINVAL, "leading dimension smaller than the block");
    neo_hip::device_guard g(h->device);
    if (g.rc) return g.rc;
    if (is_device) {
        if (int rc = h->used.note(neo_hip::as_stream(stream))) return rc;
        return forward_dev(h, in, ld_in, spectrum, neo_hip::as_stream(stream));
    }
    hipStream_t s = stream ? neo_hip::as_stream(stream) : h->stream;
    const size_t ib = size_t(h->C) * size_t(h->B) * sizeof(float), sb = size_t(h->C) * size_t(h->bins) * sizeof(neo_hip::cf);
    if ((!h->io && neo_hip::dalloc(&h->io, ib)) || (!h->spec && neo_hip::dalloc(&h->spec, sb)))
        return fail(NEO_HIP_ENOMEM, "overlap stage staging");
    NEO_HIP_CHECK(hipMemcpy2DAsync(h->io, size_t(h->B) * sizeof(float), in, size_t(ld_in) * sizeof(float),
                                   size_t(h->B) * sizeof(float), size_t(h->C), hipMemcpyHostToDevice, s));
    if (int rc = forward_dev(h, h->io, h->B, h->spec, s)) return rc;
    NEO_HIP_CHECK(hipMemcpyAsync(spectrum, h->spec, sb, hipMemcpyDeviceToHost, s));
    NEO_HIP_CHECK(hipStreamSynchronize(s));
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_overlap_inverse(neo_hip_overlap* h, const void* spectrum, float* out, int64_t ld_out,
                                        int is_device, void* stream)
{
    if (!h || !out || !spectrum) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (ld_out < h->B) return fail(NEO_HIP_EINVAL, "leading dimension smaller than the block");
    neo_hip::device_guard g(h->device);
    if (g.rc) return g.rc;
    if (is_device) {
        if (int rc = h->used.note(neo_hip::as_stream(stream))) return rc;
        return inverse_dev(h, spectrum, out, ld_out, neo_hip::as_stream(stream));
    }
    hipStream_t s = stream ? neo_hip::as_stream(stream) : h->stream;
    const size_t ib = size_t(h->C) * size_t(h->B) * sizeof(float), sb = size_t(h->C) * size_t(h->bins) * sizeof(neo_hip::cf);
    if ((!h->io && neo_hip::dalloc(&h->io, ib)) || (!h->spec && neo_hip::dalloc(&h->spec, sb)))
        return fail(NEO_HIP_ENOMEM, "overlap stage staging");
    NEO_HIP_CHECK(hipMemcpyAsync(h->spec, spectrum, sb, hipMemcpyHostToDevice, s));
    if (int rc = inverse_dev(h, h->spec, h->io, h->B, s)) return rc;
    NEO_HIP_CHECK(hipMemcpy2DAsync(out, size_t(ld_out) * sizeof(float), h->io, size_t(h->B) * sizeof(float),
                                   size_t(h->B) * sizeof(float), size_t(h->C), hipMemcpyDeviceToHost, s));
    NEO_HIP_CHECK(hipStreamSynchronize(s));
    return NEO_HIP_OK;
}

}  // extern "C"
