// valubench — f32 FMA issue rate on gfx950: packed (v_pk_fma_f32) vs scalar (v_fma_f32)
// chains, independent accumulators, registers only. Prints TFLOP/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2v __attribute__((ext_vector_type(2)));

template<int NA, int W>
__global__ __launch_bounds__(256, W) void k_pk(float* out, int iters, float s)
{
    f2v a[NA];
    f2v x = {s * threadIdx.x, s + threadIdx.x}, h = {s, -s};
#pragma unroll
    for (int i = 0; i < NA; ++i) a[i] = {float(i), float(i + 1)};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NA; ++i) a[i] = __builtin_elementwise_fma(h, x, a[i]);
        x = x.yx;
    }
    f2v t = a[0];
#pragma unroll
    for (int i = 1; i < NA; ++i) t += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

template<int NA, int W>
__global__ __launch_bounds__(256, W) void k_sc(float* out, int iters, float s)
{
    float a[2 * NA];
    float x = s * threadIdx.x, h = s;
#pragma unroll
    for (int i = 0; i < 2 * NA; ++i) a[i] = float(i);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 2 * NA; ++i) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(h), "v"(x));
        x = x + 1.0f;
    }
    float t = 0;
#pragma unroll
    for (int i = 0; i < 2 * NA; ++i) t += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template<class F>
static void run(const char* name, F kern, int grid, int iters, int fma_per_iter, float* d)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, iters, 1.0001f);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, d, iters, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * double(grid) * 256 * iters * fma_per_iter * reps;
    printf("%-28s %8.3f ms  %7.1f TFLOP/s\n", name, ms / reps, flop / (ms * 1e-3) / 1e12);
}

int main()
{
    const int grid = 256 * 8 * 4, iters = 4096;
    float* d;
    hipMalloc(&d, size_t(grid) * 256 * sizeof(float));
    run("pk_fma 16 acc, 2 w/simd", k_pk<16, 2>, grid, iters, 32, d);
    run("pk_fma 32 acc, 2 w/simd", k_pk<32, 2>, grid, iters, 64, d);
    run("pk_fma 16 acc, 4 w/simd", k_pk<16, 4>, grid, iters, 32, d);
    run("pk_fma 8 acc, 8 w/simd", k_pk<8, 8>, grid, iters, 16, d);
    run("fma 32 acc, 2 w/simd", k_sc<16, 2>, grid, iters, 32, d);
    run("fma 32 acc, 4 w/simd", k_sc<16, 4>, grid, iters, 32, d);
    hipFree(d);
    return 0;
}
