// pmc_calib.hip — FETCH_SIZE / WRITE_SIZE calibration (MI355X_MICROARCH.md §HBM: gfx950 reports
// 1/2 of the bytes for 16-B-per-lane coalesced reads; other widths are uncalibrated) on the access
// forms the UPOLS step roles use: 4-, 8- and 16-B lanes, plain / nontemporal global loads and
// buffer loads, 8-B stores, and the roles' 16-column row segments (128 B of a row per 16 lanes,
// rows 4 KB apart). Every kernel reads a 1 GiB buffer once (past the 256 MiB Infinity Cache) or
// writes it once; run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE) in separate passes and
// divide the counter (KiB) by the known bytes (tools/pmc_calib/summary.py).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = size_t(1) << 30;
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

template<typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ p, size_t n, float* sink)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const T v = p[i];
        s += reinterpret_cast<const float*>(&v)[0];
    }
    if (s == 1234.5f) sink[0] = s;  // keeps the loads
}

template<typename T>
__global__ __launch_bounds__(256) void k_read_nt(const T* __restrict__ p, size_t n, float* sink)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        const T v = __builtin_nontemporal_load(p + i);
        s += reinterpret_cast<const float*>(&v)[0];
    }
    if (s == 1234.5f) sink[0] = s;
}

// buffer loads, 8 B per lane, aux 2 (the roles' buf_ld), one 256-lane workgroup per 128 KB chunk
__global__ __launch_bounds__(256) void k_read_buf8(const char* p, size_t bytes, float* sink)
{
    float s = 0.f;
    constexpr int kChunk = 1 << 17;
    for (size_t c = blockIdx.x; c * kChunk < bytes; c += gridDim.x) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p) + c * kChunk, 0, kChunk, 0x00020000);
        for (int o = threadIdx.x * 8; o < kChunk; o += 256 * 8) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 2);
            s += __uint_as_float(v[0]);
        }
    }
    if (s == 1234.5f) sink[0] = s;
}

// the roles' row segments: a lane reads 8 B of column (t & 15) of a 16-column group; the lanes of a
// wave take 4 consecutive column groups of one row (512 B), rows of 4096 B, every row once
__global__ __launch_bounds__(256) void k_read_rows16(const v2f* __restrict__ p, size_t n, float* sink)
{
    float s = 0.f;
    const size_t rows = n / 512;  // 512 v2f per 4 KB row
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    for (size_t r = blockIdx.x * size_t(4) + w; r < rows; r += size_t(gridDim.x) * 4) {
        const v2f* row = p + r * 512;
#pragma unroll
        for (int g = 0; g < 8; ++g) s += __builtin_nontemporal_load(row + g * 64 + l)[0];
    }
    if (s == 1234.5f) sink[0] = s;
}

template<typename T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        T v{};
        reinterpret_cast<float*>(&v)[0] = float(i);
        p[i] = v;
    }
}

#define CK(x)                                                                     \
    do {                                                                          \
        if ((x) != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(x));    \
            return 1;                                                             \
        }                                                                         \
    } while (0)

int main()
{
    char* buf = nullptr;
    float* sink = nullptr;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 0, kBytes));
    const dim3 grid(4096), blk(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((k_read<float>), grid, blk, 0, 0, (const float*)buf, kBytes / 4, sink);
        hipLaunchKernelGGL((k_read<v2f>), grid, blk, 0, 0, (const v2f*)buf, kBytes / 8, sink);
        hipLaunchKernelGGL((k_read<v4f>), grid, blk, 0, 0, (const v4f*)buf, kBytes / 16, sink);
        hipLaunchKernelGGL((k_read_nt<v2f>), grid, blk, 0, 0, (const v2f*)buf, kBytes / 8, sink);
        hipLaunchKernelGGL((k_read_nt<v4f>), grid, blk, 0, 0, (const v4f*)buf, kBytes / 16, sink);
        hipLaunchKernelGGL(k_read_buf8, grid, blk, 0, 0, (const char*)buf, kBytes, sink);
        hipLaunchKernelGGL(k_read_rows16, grid, blk, 0, 0, (const v2f*)buf, kBytes / 8, sink);
        hipLaunchKernelGGL((k_write<v2f>), grid, blk, 0, 0, (v2f*)buf, kBytes / 8);
        hipLaunchKernelGGL((k_write<v4f>), grid, blk, 0, 0, (v4f*)buf, kBytes / 16);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"bytes_per_kernel\": %zu}\n", kBytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
