// fftbench.hip — variant microbenchmark for the batched 4096-pt c2c kernel (C2).
// Each variant is checked bit-for-bit against the baseline and timed with HIP events.
#include "../../neo-dsp_amd/csrc/fft_device.hpp"
#include "../../include/neo_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <string>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace neo_hip;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int N = 4096, E = 16, T = N / E, TWL = twiddle_len<N>(), LL = lds_len(N);

template<bool NT>
__device__ __forceinline__ cf ld(const cf* p)
{
    if constexpr (NT) {
        cf r;
        r.x = __builtin_nontemporal_load(&p->x);
        r.y = __builtin_nontemporal_load(&p->y);
        return r;
    } else {
        return *p;
    }
}

template<bool NT>
__device__ __forceinline__ void st(cf* p, cf v)
{
    if constexpr (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
    } else {
        *p = v;
    }
}

// V0: one transform per workgroup (the product kernel), optional nontemporal loads / stores
template<bool NTL, bool NTS = NTL>
__global__ __launch_bounds__(256) void k_v0(const cf* __restrict__ in, cf* __restrict__ out, const cf* __restrict__ twg,
                                            int64_t batch)
{
    __shared__ cf smem[LL + TWL];
    cf* tw = smem + LL;
    const int t = threadIdx.x;
    for (int i = t; i < TWL; i += 256) tw[i] = twg[i];
    const int64_t g = blockIdx.x;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) v[m] = ld<NTL>(in + g * N + t + m * T);
    __syncthreads();
    stockham<N, E, -1>(v, smem, tw, t, true);
#pragma unroll
    for (int m = 0; m < E; ++m) st<NTS>(out + g * N + t + m * T, v[m]);
}

// copy kernels with the FFT's access pattern (8 B/lane, t + m*T) and a 16-B/lane variant
template<bool NT>
__global__ __launch_bounds__(256) void k_copy8(const cf* __restrict__ in, cf* __restrict__ out)
{
    const int t = threadIdx.x;
    const int64_t g = blockIdx.x;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) v[m] = ld<NT>(in + g * N + t + m * T);
#pragma unroll
    for (int m = 0; m < E; ++m) st<NT>(out + g * N + t + m * T, v[m]);
}
typedef float f4v __attribute__((ext_vector_type(4)));
template<bool NT>
__global__ __launch_bounds__(256) void k_copy16(const f4v* __restrict__ in, f4v* __restrict__ out)
{
    const int t = threadIdx.x;
    const int64_t g = blockIdx.x;
    f4v v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        if constexpr (NT) v[m] = __builtin_nontemporal_load(in + g * 2048 + t + m * 256);
        else v[m] = in[g * 2048 + t + m * 256];
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        if constexpr (NT) __builtin_nontemporal_store(v[m], out + g * 2048 + t + m * 256);
        else out[g * 2048 + t + m * 256] = v[m];
    }
}

// read-only stream (the MAC kernel's regime: 99.5 % reads): grid-stride float4 sum
template<bool NT>
__global__ __launch_bounds__(256) void k_read16(const f4v* __restrict__ in, int64_t n4, float* __restrict__ sink)
{
    float acc = 0.f;
    const int64_t stride = int64_t(gridDim.x) * 256 * 4;
    for (int64_t i = int64_t(blockIdx.x) * 256 * 4 + threadIdx.x; i < n4; i += stride) {
        f4v v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t j = i + u * 256;
            if constexpr (NT) v[u] = j < n4 ? __builtin_nontemporal_load(in + j) : f4v{0, 0, 0, 0};
            else v[u] = j < n4 ? in[j] : f4v{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 12345.678f) sink[0] = acc;  // keep the loads live
}

// V1: grid-stride over transforms with the next transform prefetched into registers
template<bool NT>
__global__ __launch_bounds__(256) void k_v1(const cf* __restrict__ in, cf* __restrict__ out, const cf* __restrict__ twg,
                                            int64_t batch)
{
    __shared__ cf smem[LL + TWL];
    cf* tw = smem + LL;
    const int t = threadIdx.x;
    for (int i = t; i < TWL; i += 256) tw[i] = twg[i];
    int64_t g = blockIdx.x;
    cf v[E], nx[E];
    if (g < batch) {
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = ld<NT>(in + g * N + t + m * T);
    }
    __syncthreads();
    for (; g < batch; g += gridDim.x) {
        const int64_t gn = g + gridDim.x;
        if (gn < batch) {
#pragma unroll
            for (int m = 0; m < E; ++m) nx[m] = ld<NT>(in + gn * N + t + m * T);
        }
        stockham<N, E, -1>(v, smem, tw, t, true);
#pragma unroll
        for (int m = 0; m < E; ++m) st<NT>(out + g * N + t + m * T, v[m]);
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = nx[m];
    }
}

__global__ void k_fill(cf* x, int64_t n, uint64_t seed)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ull * uint64_t(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = {float(z >> 40) * (2.0f / 16777216.0f) - 1.0f, float((z >> 16) & 0xFFFFFF) * (2.0f / 16777216.0f) - 1.0f};
    }
}

int main(int argc, char** argv)
{
    const int64_t batch = argc > 1 ? std::atoll(argv[1]) : 65536;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const size_t bytes = size_t(batch) * N * sizeof(cf);
    cf *in, *out, *ref, *tw;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&ref, bytes));
    std::vector<cf> t(TWL);
    for (int e = 0; e < 64; ++e) t[e] = {float(std::cos(-2 * M_PI * e / N)), float(std::sin(-2 * M_PI * e / N))};
    for (int h = 0; h < N / 64; ++h)
        t[64 + h] = {float(std::cos(-2 * M_PI * 64 * h / N)), float(std::sin(-2 * M_PI * 64 * h / N))};
    CK(hipMalloc(&tw, TWL * sizeof(cf)));
    CK(hipMemcpy(tw, t.data(), TWL * sizeof(cf), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, in, batch * N, 12345ull);
    hipLaunchKernelGGL(k_v0<false>, dim3(unsigned(batch)), dim3(256), 0, 0, in, ref, tw, batch);
    CK(hipDeviceSynchronize());
    std::vector<cf> h_ref(size_t(N) * 64), h_out(size_t(N) * 64);

    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int dev_cus = 0;
    CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));

    using launch_fn = std::function<void()>;
    std::vector<std::pair<std::string, launch_fn>> vars;
    unsigned nb = unsigned(batch);
    neo_hip_fft_plan* plan = nullptr;
    if (neo_hip_fft_plan_create(12, batch, NEO_HIP_C2C, 0, &plan)) std::printf("plan failed: %s\n", neo_hip_last_error());
    vars.push_back({"product neo_hip_fft_execute", [&] { neo_hip_fft_execute(plan, in, out, -1, nullptr); }});
    vars.push_back({"v0 plain", [&] { hipLaunchKernelGGL(k_v0<false>, dim3(nb), dim3(256), 0, 0, in, out, tw, batch); }});
    vars.push_back({"v0 nt", [&] { hipLaunchKernelGGL(k_v0<true>, dim3(nb), dim3(256), 0, 0, in, out, tw, batch); }});
    vars.push_back({"v0 nt loads", [&] { hipLaunchKernelGGL((k_v0<true, false>), dim3(nb), dim3(256), 0, 0, in, out, tw, batch); }});
    vars.push_back({"v0 nt stores", [&] { hipLaunchKernelGGL((k_v0<false, true>), dim3(nb), dim3(256), 0, 0, in, out, tw, batch); }});
    unsigned g4 = unsigned(std::min<int64_t>(batch, int64_t(4) * dev_cus));
    vars.push_back({"v1 prefetch nt 4/CU", [&] { hipLaunchKernelGGL(k_v1<true>, dim3(g4), dim3(256), 0, 0, in, out, tw, batch); }});
    vars.push_back({"copy 8B nt (bytes ref)", [&] { hipLaunchKernelGGL(k_copy8<true>, dim3(nb), dim3(256), 0, 0, in, out); }});
    vars.push_back({"copy 16B nt (bytes ref)", [&] { hipLaunchKernelGGL(k_copy16<true>, dim3(nb), dim3(256), 0, 0, (const f4v*)in, (f4v*)out); }});
    vars.push_back({"copy 16B (bytes ref)", [&] { hipLaunchKernelGGL(k_copy16<false>, dim3(nb), dim3(256), 0, 0, (const f4v*)in, (f4v*)out); }});
    float* sink;
    CK(hipMalloc(&sink, 4));
    const int64_t n4 = int64_t(bytes / 16);
    for (int wgs : {1024, 2048, 4096}) {
        vars.push_back({"read-only 16B nt " + std::to_string(wgs) + "WG (x0.5)", [&, wgs] {
                            hipLaunchKernelGGL(k_read16<true>, dim3(wgs), dim3(256), 0, 0, (const f4v*)in, n4, sink);
                        }});
        vars.push_back({"read-only 16B " + std::to_string(wgs) + "WG (x0.5)", [&, wgs] {
                            hipLaunchKernelGGL(k_read16<false>, dim3(wgs), dim3(256), 0, 0, (const f4v*)in, n4, sink);
                        }});
    }
    // correctness vs baseline (first/last 64 transforms); copies are skipped
    for (size_t v = 0; v < vars.size(); ++v) {
        if (vars[v].first.rfind("copy", 0) == 0 || vars[v].first.rfind("read", 0) == 0) continue;
        CK(hipMemset(out, 0, bytes));
        vars[v].second();
        CK(hipDeviceSynchronize());
        double md = 0;
        for (int part = 0; part < 2; ++part) {
            size_t off = part == 0 ? 0 : (size_t(batch) - 64) * N;
            CK(hipMemcpy(h_ref.data(), ref + off, h_ref.size() * sizeof(cf), hipMemcpyDeviceToHost));
            CK(hipMemcpy(h_out.data(), out + off, h_out.size() * sizeof(cf), hipMemcpyDeviceToHost));
            for (size_t i = 0; i < h_ref.size(); ++i)
                md = std::max(md, double(std::fabs(h_ref[i].x - h_out[i].x)) + std::fabs(h_ref[i].y - h_out[i].y));
        }
        std::printf("check %-28s max|diff| vs v0 %.2e\n", vars[v].first.c_str(), md);
    }
    // interleaved rounds: one launch of every variant per round (rule 24)
    std::vector<std::vector<float>> ms(vars.size());
    for (int r = 0; r < iters; ++r)
        for (size_t v = 0; v < vars.size(); ++v) {
            CK(hipEventRecord(a, 0));
            vars[v].second();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float t = 0;
            CK(hipEventElapsedTime(&t, a, b));
            if (r > 0) ms[v].push_back(t);  // round 0 = warm-up
        }
    // sustained: 20 back-to-back launches of one variant between two events
    for (size_t v = 0; v < vars.size(); ++v) {
        if (vars[v].first.rfind("read", 0) == 0) continue;
        std::vector<float> bb;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < 20; ++i) vars[v].second();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float t = 0;
            CK(hipEventElapsedTime(&t, a, b));
            bb.push_back(t / 20);
        }
        std::sort(bb.begin(), bb.end());
        std::printf("back-to-back x20 %-28s %.4f ms/launch (best of 3: %.4f)\n", vars[v].first.c_str(), bb[1], bb[0]);
    }
    for (size_t v = 0; v < vars.size(); ++v) {
        auto& m = ms[v];
        std::sort(m.begin(), m.end());
        const float med = m[m.size() / 2];
        std::printf("%-28s med %.4f ms  min %.4f  max %.4f -> %.0f GB/s (%.3f of 8 TB/s)\n", vars[v].first.c_str(), med,
                    m.front(), m.back(), 16.0 * N * batch / (med * 1e6), 16.0 * N * batch / (med * 1e6) / 8000.0);
    }
    return 0;
}
