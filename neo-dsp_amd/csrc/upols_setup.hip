// upols_setup.hip — the IR-change path on the GPU: uniform_partition
// (uniform_partition.hpp:12-26 -> stft.hpp:40-109: C·P packed r2c of zero-padded
// partitions) and normalize_impulse (normalize_impulse.hpp:11-33, bit-exact sequential
// float energy), used by neo_hip_upols_set_impulse and exported on their own.
#include "upols_device.hpp"
#include "upols_handle.hpp"

#include <algorithm>

namespace neo_hip {

// uniform_partition (uniform_partition.hpp:12-26 -> stft.hpp:56-99): partition p
// of channel c = rfft_2B(ir[c][pB : pB+B] zero-padded to 2B). Packed output
// [C][P][B] (UPOLS layout) or unpacked [C][P][B+1] (reference layout).
template<int B, bool PACKED>
__global__ __launch_bounds__(256) void k_partition(const float* __restrict__ ir, int64_t L, int P,
                                                   cf* __restrict__ out, const cf* __restrict__ twg, int64_t cstride,
                                                   int64_t pstride)
{
    using K = upols_cfg<B>;
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x;
    const int64_t cp = blockIdx.x;
    const int64_t c = cp / P, p = cp - c * P;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    const bool active = tid < K::T;
    const float* seg = ir + c * L + p * B;
    const int64_t cnt = min(int64_t(B), L - p * B);
    cf v[K::E];
    if (active) {
#pragma unroll
        for (int m = 0; m < K::E; ++m) {
            const int n = tid + m * K::T;  // z[n] = (w[2n], w[2n+1]); w = segment | zeros
            const float a = 2 * n < cnt ? seg[2 * n] : 0.f;
            const float b = 2 * n + 1 < cnt ? seg[2 * n + 1] : 0.f;
            v[m] = {a, b};
        }
    }
    __syncthreads();
    stockham<B, K::E, -1>(v, fft, tw, tid, active);
    if (active) {
#pragma unroll
        for (int m = 0; m < K::E; ++m) fft[lpad(tid + m * K::T)] = v[m];
    }
    __syncthreads();
    if constexpr (PACKED) {
        cf* row = out + c * cstride + p * pstride;  // device layout (see neo_hip_upols)
        for (int k = tid; k < B; k += 256) row[k] = r2c_split<B>(fft, tw + K::TW1, k);
    } else {
        cf* row = out + cp * (B + 1);
        for (int k = tid; k < B; k += 256) {
            const cf x = r2c_split<B>(fft, tw + K::TW1, k);
            if (k == 0) {
                row[0] = {x.x, 0.f};
                row[B] = {x.y, 0.f};
            } else {
                row[k] = x;
            }
        }
    }
}

// filter [C][P][B+1] (reference layout) -> packed [C][P][B]
__global__ void k_pack_filter(const cf* __restrict__ in, cf* __restrict__ out, int B, int64_t rows, int P,
                              int64_t cstride, int64_t pstride)
{
    const int64_t gid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (gid >= rows * B) return;
    const int64_t r = gid / B, k = gid - r * B;
    const int64_t c = r / P, p = r - c * P;
    const cf* src = in + r * (B + 1);
    out[c * cstride + p * pstride + k] = k == 0 ? cf{src[0].x, src[B].x} : src[k];
}

// normalize_energy_factor (normalize_energy.hpp:17-44) with the reference's exact
// rounding: sequential float sum of x*x (multiply, then add; no FMA), then
// 1/sqrt.
// One workgroup per kEnergyGroup channels: all 256 lanes stream a [G][256] tile of the
// impulse with coalesced loads into LDS (double-buffered), then lane g < G folds row g
// into its channel's energy in sample order. Zero padding past L adds +0.0f, which
// leaves the running sum unchanged, so the rounding equals the reference's loop.
constexpr int kEnergyGroup = 16;
constexpr int kEnergyTile = 256;

__global__ __launch_bounds__(256) void k_energy_factor(const float* __restrict__ ir, int64_t L, int C,
                                                       float* __restrict__ factor)
{
#pragma clang fp contract(off)  // x*x then +, two roundings, like the reference (no FMA)
    constexpr int G = kEnergyGroup, T = kEnergyTile, LD = T + 4;  // +4: conflict-free b128 row reads
    __shared__ float tile[2][G * LD];
    const int c0 = int(blockIdx.x) * G, t = int(threadIdx.x);
    const int64_t chunks = (L + T - 1) / T;
    float r[G];
    bool valid = true;
    auto load = [&](int64_t chunk) {
        const int64_t i = chunk * T + t;
        valid = i < L;
        const int64_t ic = valid ? i : L - 1;  // clamped address, no branch around the loads
#pragma unroll
        for (int g = 0; g < G; ++g)  // rows past C repeat channel C-1; their sums are discarded
            r[g] = ir[int64_t(min(c0 + g, C - 1)) * L + ic];
    };
    auto store = [&](int buf) {  // the zero select sits here so the loads stay in flight
#pragma unroll
        for (int g = 0; g < G; ++g) tile[buf][g * LD + t] = valid ? r[g] : 0.0f;
    };
    float e = 0.0f;
    load(0);
    store(0);
    __syncthreads();
    for (int64_t chunk = 0; chunk < chunks; ++chunk) {
        const int buf = int(chunk & 1);
        if (chunk + 1 < chunks) load(chunk + 1);  // in flight while row t is summed
        if (t < G) {
            const float* row = &tile[buf][t * LD];
#pragma unroll 8
            for (int j = 0; j < T; j += 4) {
                const float4 v = *reinterpret_cast<const float4*>(row + j);
                const float s0 = v.x * v.x, s1 = v.y * v.y, s2 = v.z * v.z, s3 = v.w * v.w;
                e = e + s0;
                e = e + s1;
                e = e + s2;
                e = e + s3;
            }
        }
        if (chunk + 1 < chunks) store(buf ^ 1);
        __syncthreads();
    }
    if (t < G && c0 + t < C) factor[c0 + t] = e == 0.0f ? 1.0f : __fdiv_rn(1.0f, __fsqrt_rn(e));
}

// normalize_impulse.hpp:21-30: min factor over channels, then scale everything
__global__ void k_scale_min(float* __restrict__ ir, int64_t n, const float* __restrict__ factor, int C)
{
    __shared__ float fmin_s;
    if (threadIdx.x == 0) {
        float f = factor[0];
        for (int c = 1; c < C; ++c) f = fminf(f, factor[c]);
        fmin_s = f;
    }
    __syncthreads();
    const float f = fmin_s;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
        ir[i] = __fmul_rn(ir[i], f);
}


int upload_tw(cf** d, int B)
{
    std::vector<cf> t = make_twiddle_table(B);
    std::vector<cf> t2 = make_twiddle_table(2 * int64_t(B));
    t.insert(t.end(), t2.begin(), t2.end());
    NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(d), t.size() * sizeof(cf)));
    NEO_HIP_CHECK(hipMemcpy(*d, t.data(), t.size() * sizeof(cf), hipMemcpyHostToDevice));
    return NEO_HIP_OK;
}

// normalize (optional) + partition ir [C][L] (device) into packed or unpacked rows.
int partition_device(const float* d_ir, int C, int64_t L, int B, bool packed, cf* out, const cf* tw, hipStream_t s,
                     int64_t cstride, int64_t pstride)
{
    const int64_t P = partitions_for(L, B);
    const int64_t blocks = int64_t(C) * P;
    if (blocks > 0x7fffffff) return fail(NEO_HIP_EINVAL, "too many partitions");
    if (packed) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_partition<BB, true>), dim3(unsigned(blocks)), dim3(256), 0, s,
                                                 d_ir, L, int(P), out, tw, cstride, pstride))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_partition<BB, false>), dim3(unsigned(blocks)), dim3(256), 0, s,
                                                 d_ir, L, int(P), out, tw, cstride, pstride))
    }
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

int normalize_device(float* d_ir, int C, int64_t L, hipStream_t s)
{
    if (C < 1) return NEO_HIP_OK;
    float* factor = nullptr;
    NEO_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&factor), size_t(C) * sizeof(float), s));
    hipLaunchKernelGGL(k_energy_factor, dim3(unsigned((C + kEnergyGroup - 1) / kEnergyGroup)), dim3(256), 0, s, d_ir, L,
                       C, factor);
    NEO_HIP_LAUNCH_CHECK();
    const int64_t n = int64_t(C) * L;
    const unsigned blocks = unsigned(std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(k_scale_min, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, d_ir, n, factor, C);
    NEO_HIP_LAUNCH_CHECK();
    NEO_HIP_CHECK(hipFreeAsync(factor, s));
    return NEO_HIP_OK;
}

int pack_filter(upols_t* h, const cf* src, hipStream_t s)
{
    const int64_t rows = int64_t(h->C) * h->P, total = rows * h->B;
    hipLaunchKernelGGL(k_pack_filter, dim3(unsigned((total + 255) / 256)), dim3(256), 0, s, src, h->H, h->B, rows,
                       h->P, h->cstride, h->pstride);
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

}  // namespace neo_hip

using namespace neo_hip;

extern "C" {

NEO_HIP_API int neo_hip_num_partitions(int64_t length, int block, int64_t* partitions)
{
    if (!partitions || block < 1 || length < 0) return fail(NEO_HIP_EINVAL, "bad arguments");
    *partitions = partitions_for(length, block);
    return NEO_HIP_OK;
}


NEO_HIP_API int neo_hip_uniform_partition(const float* ir, int channels, int64_t length, int block, void* out,
                                          int is_device, int device)
{
    if (!ir || !out || channels < 1 || length < 1) return fail(NEO_HIP_EINVAL, "bad arguments");
    if (!valid_block(block)) return fail(NEO_HIP_EINVAL, "block must be a power of two in [16, 4096], got %d", block);
    device_guard g(device);
    if (g.rc) return g.rc;
    const int64_t P = partitions_for(length, block);
    const size_t in_bytes = size_t(channels) * size_t(length) * sizeof(float);
    const size_t out_bytes = size_t(channels) * size_t(P) * size_t(block + 1) * sizeof(cf);
    hipStream_t s = nullptr;
    if (is_device)
        if (int rc = null_join()) return rc;  // after its producer (common.hpp: null_join)
    if (int rs = shared_stream(&s)) return rs;  // one of the device's four (dmem.hip)
    cf* tw = nullptr;
    const float* d_ir = ir;
    float* tmp_in = nullptr;
    cf* d_out = static_cast<cf*>(out);
    int rc = shared_tw(&tw, block);
    if (!rc && !is_device) {  // pooled (dmem.hip): no hipMalloc / hipFree, which wait for the device
        if (dalloc(&tmp_in, in_bytes) || dalloc(&d_out, out_bytes))
            rc = fail(NEO_HIP_ENOMEM, "allocation failed");
        else if (hipMemcpyAsync(tmp_in, ir, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy failed");
        d_ir = tmp_in;
    }
    if (!rc) rc = partition_device(d_ir, channels, length, block, false, d_out, tw, s);
    if (!rc && !is_device && hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    if (!is_device) {  // the stream was joined above
        dfree(tmp_in);
        dfree(d_out);
    }
    return rc;
}

NEO_HIP_API int neo_hip_normalize_impulse(float* ir, int channels, int64_t length, int is_device, int device)
{
    if (!ir || channels < 0 || length < 0) return fail(NEO_HIP_EINVAL, "bad arguments");
    if (channels == 0 || length == 0) return NEO_HIP_OK;
    device_guard g(device);
    if (g.rc) return g.rc;
    hipStream_t s = nullptr;
    if (is_device)
        if (int rc = null_join()) return rc;  // after its producer (common.hpp: null_join)
    if (int rs = shared_stream(&s)) return rs;  // one of the device's four (dmem.hip)
    const size_t bytes = size_t(channels) * size_t(length) * sizeof(float);
    float* d = ir;
    int rc = NEO_HIP_OK;
    if (!is_device) {
        if (dalloc(&d, bytes)) rc = fail(NEO_HIP_ENOMEM, "alloc failed");
        else if (hipMemcpyAsync(d, ir, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy failed");
    }
    if (!rc) rc = normalize_device(d, channels, length, s);
    if (!rc && !is_device && hipMemcpyAsync(ir, d, bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    if (!is_device) dfree(d);  // the stream was joined above
    return rc;
}

}  // extern "C"
