// fft_device.hpp — CDNA4 (gfx950) device building blocks for neo's FFT hot path.
//
// Self-sorting Stockham FFT of a power-of-two size N held by T = N/E lanes,
// E elements per lane, exchanged through LDS between passes. Pass radix R is E
// while it divides the remaining length, then the remainder; a lane performs
// E/R butterflies per pass. Lane t always owns elements t + m*T (m < E) on
// entry and on exit, so global loads/stores are coalesced at both ends and the
// output is in natural order (no bit-reverse pass, unlike the reference's
// c2c_dit2_plan, src/neo/fft/reference/c2c_dit2_plan.hpp:81-95, whose result
// is the same unnormalized DFT: X[k] = sum_n x[n] e^{dir*2*pi*i*n*k/N},
// direction::forward = -1, src/neo/fft/direction.hpp:8-12).
//
// Twiddles come from a two-level table (lo: e & 63, hi: e >> 6) computed on the
// host in double precision and staged in LDS, so one twiddle costs two LDS reads
// and one complex multiply with ~1.5 ulp error (the reference computes angles in
// float, src/neo/fft/twiddle.hpp:17-29).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace neo_hip {

struct alignas(8) cf {  // complex float, interleaved {re, im} = std::complex<float> layout
    float x, y;
};
struct alignas(16) cd {  // complex double, = std::complex<double> layout (the f64 plans)
    double x, y;
};
template<class C>
using real_of = decltype(C::x);

// Streaming (nontemporal) global accesses: HBM-streamed data that no later
// kernel re-reads from cache (measured: 4096-pt batched FFT 0.856 -> 0.739 ms).
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ cf ld_nt(const cf* p)
{
    const f2v v = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p));
    return {v.x, v.y};
}
__device__ __forceinline__ void st_nt(cf* p, cf a)
{
    f2v v;
    v.x = a.x;
    v.y = a.y;
    __builtin_nontemporal_store(v, reinterpret_cast<f2v*>(p));
}
__device__ __forceinline__ cd ld_nt(const cd* p)
{
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return {v.x, v.y};
}
__device__ __forceinline__ void st_nt(cd* p, cd a)
{
    d2v v;
    v.x = a.x;
    v.y = a.y;
    __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(p));
}
__device__ __forceinline__ float4 ld4_nt(const float4* p)
{
    const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st4_nt(float4* p, float4 a)
{
    f4v v;
    v.x = a.x;
    v.y = a.y;
    v.z = a.z;
    v.w = a.w;
    __builtin_nontemporal_store(v, reinterpret_cast<f4v*>(p));
}
template<bool NT>
__device__ __forceinline__ float4 ld4(const float4* p)
{
    if constexpr (NT) return ld4_nt(p);
    else return *p;
}

template<class C>
__device__ __forceinline__ C cadd(C a, C b) { return {a.x + b.x, a.y + b.y}; }
template<class C>
__device__ __forceinline__ C csub(C a, C b) { return {a.x - b.x, a.y - b.y}; }
template<class C>
__device__ __forceinline__ C cmul(C a, C b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
template<class C>
__device__ __forceinline__ C cconj(C a) { return {a.x, -a.y}; }
template<class C>
__device__ __forceinline__ C cscale(C a, real_of<C> s) { return {a.x * s, a.y * s}; }

// cos/sin(2*pi*k/16), k = 0..15, rounded to float
__device__ constexpr float kCos16[16] = {
    1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
    0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
    -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f,
    0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f};
__device__ constexpr float kSin16[16] = {
    0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f,
    1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
    0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
    -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};

__device__ constexpr double kCos16d[16] = {
    1.0, 0.92387953251128674, 0.70710678118654752, 0.38268343236508977,
    0.0, -0.38268343236508977, -0.70710678118654752, -0.92387953251128674,
    -1.0, -0.92387953251128674, -0.70710678118654752, -0.38268343236508977,
    0.0, 0.38268343236508977, 0.70710678118654752, 0.92387953251128674};
__device__ constexpr double kSin16d[16] = {
    0.0, 0.38268343236508977, 0.70710678118654752, 0.92387953251128674,
    1.0, 0.92387953251128674, 0.70710678118654752, 0.38268343236508977,
    0.0, -0.38268343236508977, -0.70710678118654752, -0.92387953251128674,
    -1.0, -0.92387953251128674, -0.70710678118654752, -0.38268343236508977};

// a * exp(DIR * 2*pi*i * k / 16); k is a compile-time constant after unrolling,
// so the trivial rotations fold into swaps/negations.
template<int DIR, class C>
__device__ __forceinline__ C rot16(C a, int k)
{
    k &= 15;
    if (k == 0) return a;
    if (k == 8) return {-a.x, -a.y};
    if (k == 4) return DIR < 0 ? C{a.y, -a.x} : C{-a.y, a.x};
    if (k == 12) return DIR < 0 ? C{-a.y, a.x} : C{a.y, -a.x};
    using R = real_of<C>;
    R c, s;
    if constexpr (sizeof(R) == 8) {
        c = kCos16d[k];
        s = DIR < 0 ? -kSin16d[k] : kSin16d[k];
    } else {
        c = kCos16[k];
        s = DIR < 0 ? -kSin16[k] : kSin16[k];
    }
    return {a.x * c - a.y * s, a.x * s + a.y * c};
}

__host__ __device__ constexpr int ilog2(int n) { return n <= 1 ? 0 : 1 + ilog2(n / 2); }

__host__ __device__ constexpr int bitrev_c(int v, int bits)
{
    int r = 0;
    for (int i = 0; i < bits; ++i) r |= ((v >> i) & 1) << (bits - 1 - i);
    return r;
}

// In-register R-point DFT (R | 16), natural order in and out.
// Radix-2 DIF network, then a compile-time bit-reverse permutation.
template<int R, int DIR, class C>
__device__ __forceinline__ void dft(C (&v)[R])
{
    if constexpr (R == 1) {
        return;
    } else {
#pragma unroll
        for (int half = R / 2; half >= 1; half /= 2) {
#pragma unroll
            for (int blk = 0; blk < R; blk += 2 * half) {
#pragma unroll
                for (int j = 0; j < half; ++j) {
                    const C a = v[blk + j], b = v[blk + j + half];
                    v[blk + j] = cadd(a, b);
                    // twiddle W_{2half}^j = W_16^{j * 16 / (2 half)}
                    v[blk + j + half] = rot16<DIR>(csub(a, b), j * (16 / (2 * half)));
                }
            }
        }
        C t[R];
#pragma unroll
        for (int k = 0; k < R; ++k) t[k] = v[bitrev_c(k, ilog2(R))];
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = t[k];
    }
}

// LDS padding: one complex every 16 breaks the power-of-two write strides of
// the first Stockham passes (stride-R b64 writes would hit one bank otherwise).
__device__ __forceinline__ int lpad(int a) { return a + (a >> 4); }
__host__ __device__ constexpr int lds_len(int n) { return n + n / 16 + 1; }

// Twiddle table for an FFT of size N, W = exp(-2*pi*i/N) (forward); DIR=+1 conjugates.
// N <= kTwFull: one entry per exponent, tw[e] = W^e (64 entries at least, e mod N); one LDS
// read per twiddle in the block steps' B-point transforms. Larger N: two levels,
// tw[0..63] = W^e (e < 64), tw[64..64+N/64) = W^(64*h), a read pair and a complex multiply.
constexpr int kTwFull = 512;

template<int N, int DIR, class C>
__device__ __forceinline__ C twiddle(const C* tw, int e)
{
    C w;
    if constexpr (N <= kTwFull) {
        w = tw[e];
    } else {
        w = cmul(tw[64 + (e >> 6)], tw[e & 63]);
    }
    if constexpr (DIR > 0) w.y = -w.y;
    return w;
}

template<int N>
__host__ __device__ constexpr int twiddle_len()
{
    return N <= 64 ? 64 : (N <= kTwFull ? N : 64 + N / 64);
}

// Radix chosen for the pass that starts with sub-transform length Ns.
template<int N, int E, int Ns>
__host__ __device__ constexpr int pass_radix()
{
    return ((N / Ns) % E == 0) ? E : (N / Ns);
}

// Stockham passes from sub-length Ns upward. v[m] = element t + m*T on entry
// (T = N/E); on exit v[m] = X[t + m*T]. `lds` holds lds_len(N) complex and is
// reused by every pass; all threads of the block must call (barriers inside).
// Wave-level LDS ordering for transforms run by ONE wave (WS = true in stockham): a
// wave's LDS accesses execute in order, so a compiler-level barrier plus wavefront-scope
// fences replaces the workgroup barrier, and the other waves of the workgroup need not
// take part.
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template<int N, int E, int DIR, int Ns = 1, bool WS = false, class C>
__device__ __forceinline__ void stockham(C (&v)[E], C* lds, const C* tw, int t, bool active)
{
    if constexpr (N == 1 || Ns >= N) {
        return;
    } else {
        constexpr int R = pass_radix<N, E, Ns>();
        constexpr int NB = E / R;  // butterflies per lane this pass
        constexpr int T = N / E;
        constexpr bool last = (Ns * R == N);
        if (active) {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int j = t + b * T;
                C w[R];
#pragma unroll
                for (int r = 0; r < R; ++r) w[r] = v[b + r * NB];
                const int jm = j & (Ns - 1);
                if constexpr (Ns > 1) {
#pragma unroll
                    for (int r = 1; r < R; ++r) w[r] = cmul(w[r], twiddle<N, DIR>(tw, r * jm * (N / (Ns * R))));
                }
                dft<R, DIR>(w);
                if constexpr (last) {
#pragma unroll
                    for (int r = 0; r < R; ++r) v[b + r * NB] = w[r];
                } else {
                    const int base = (j / Ns) * Ns * R + jm;
#pragma unroll
                    for (int r = 0; r < R; ++r) lds[lpad(base + r * Ns)] = w[r];
                }
            }
        }
        if constexpr (!last) {
            if constexpr (WS) wave_sync(); else __syncthreads();
            if (active) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = lds[lpad(t + m * T)];
            }
            if constexpr (WS) wave_sync(); else __syncthreads();
            stockham<N, E, DIR, Ns * R, WS>(v, lds, tw, t, active);
        }
    }
}

}  // namespace neo_hip
