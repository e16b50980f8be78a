// upols_device.hpp — device building blocks shared by the UPOLS kernels
// (upols.hip: single-block step / finish / v2 piece; upols_batch.hip: batched passes;
// upols_setup.hip: partitioning): per-B geometry, the packed-bin MAC, the overlap
// window r2c and the c2r tail (overlap_save.hpp:84-112, overlap_add.hpp:76-106).
#pragma once

#include "common.hpp"
#include "fft_device_real.hpp"

// elements per lane of the per-channel tail transforms (c2r of k_upols_finish /
// k_batch_finish): 4 per lane puts B/4 lanes to work (C5 finish 6.3 -> 4.9 us, batch 61 -> 29 us)
#ifndef NEO_FINISH_E
#define NEO_FINISH_E(B) ((B) / 4 <= 256 ? ((B) >= 4 ? 4 : (B)) : (B) / 256)
#endif
#define NEO_BATCH_FINISH_E(B) NEO_FINISH_E(B)

namespace neo_hip {

__host__ __device__ constexpr int upols_e(int b) { return b >= 16 ? 16 : b; }

template<int B>
struct upols_cfg {
    static constexpr int E = upols_e(B);                 // FFT elements per lane
    static constexpr int T = B / E;                      // FFT lanes
    static constexpr int Q = B / 2;                      // float4 (2 bins) per row
    static constexpr int QT = Q < 256 ? Q : 256;         // lanes per row group
    static constexpr int RPI = 256 / QT;                 // rows in flight per iteration
    static constexpr int VPT = Q / QT;                   // float4 per lane per row
    static constexpr int U = VPT >= 4 ? 1 : 4 / VPT;     // row unroll
    static constexpr int TW1 = twiddle_len<B>();
    static constexpr int TW2 = twiddle_len<2 * B>();
    static constexpr int LL = lds_len(B);
};

// Twiddle table staged global -> registers -> LDS: the loads issue together with the
// window loads that follow, instead of a load / wait / ds_write round trip per iteration
// ahead of them (a copy loop with a runtime trip count is not hoisted by the compiler).
template<int N, int LANES>
struct tw_regs {
    static constexpr int R = (N + LANES - 1) / LANES;
    cf v[R];
    __device__ __forceinline__ void load(const cf* __restrict__ g, int t)
    {
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (t + LANES * i < N) v[i] = g[t + LANES * i];
    }
    __device__ __forceinline__ void store(cf* l, int t) const
    {
#pragma unroll
        for (int i = 0; i < R; ++i)
            if (t + LANES * i < N) l[t + LANES * i] = v[i];
    }
};

struct acc4 {  // 4 partial products per bin keep the packed bin 0 exact
    float rr, ii, ri, ir;
};

__device__ __forceinline__ void mac2(acc4& a0, acc4& a1, float4 h, float4 x)
{
    a0.rr = fmaf(h.x, x.x, a0.rr);
    a0.ii = fmaf(h.y, x.y, a0.ii);
    a0.ri = fmaf(h.x, x.y, a0.ri);
    a0.ir = fmaf(h.y, x.x, a0.ir);
    a1.rr = fmaf(h.z, x.z, a1.rr);
    a1.ii = fmaf(h.w, x.w, a1.ii);
    a1.ri = fmaf(h.z, x.w, a1.ri);
    a1.ir = fmaf(h.w, x.z, a1.ir);
}

// acc4 -> packed complex bin: bin 0 = {DC, Nyquist} (products of real values),
// other bins = the complex product sum.
__device__ __forceinline__ cf finish(const acc4& a, bool bin0)
{
    return bin0 ? cf{a.rr, a.ii} : cf{a.rr - a.ii, a.ri + a.ir};
}

// Load the overlap-save window [prev | in] of channel c as the packed complex
// sequence z[n] = w[2n] + i w[2n+1] (lane t owns n = t + m*T), forward FFT, and
// leave the natural-order spectrum Z in `fft` (lpad'ed).
// E = 8 elements per lane keeps this fused r2c from raising the kernel's register
// count (the MAC loop itself needs ~60 VGPRs; occupancy is what streams HBM).
// OLS window = [previous block | new block] (overlap_save.hpp:90-95);
// OLA window = [new block | zeros]          (overlap_add.hpp:84-86).
// WT: the input block read at system scope (a persistent kernel: the caller may have rewritten it
// since this CU last read there); OLS: the previous block written here, from registers
__device__ __forceinline__ cf ld_in_cf(const cf* p, bool wt)
{
    if (wt)
        return __builtin_bit_cast(cf, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_SYSTEM));
    return *p;
}
template<bool WT>
__device__ __forceinline__ float4 ld4_in(const float4* p)
{
    if constexpr (WT) {
        const cf a = ld_in_cf(reinterpret_cast<const cf*>(p), true), b = ld_in_cf(reinterpret_cast<const cf*>(p) + 1, true);
        return make_float4(a.x, a.y, b.x, b.y);
    } else {
        return *p;
    }
}

template<int B, bool OLA, int E = (B / 8 <= 256 ? 8 : B / 256), bool WT = false>
__device__ __forceinline__ void window_fft(const float* prev_c, const float* in_c, cf* fft, cf* tw1, int tid,
                                           const cf* __restrict__ twg = nullptr)
{
    constexpr int T = B / E;
    static_assert(T <= 256 && B % E == 0, "window FFT must fit one 256-lane workgroup");
    using K = upols_cfg<B>;
    const bool active = tid < T;
    tw_regs<K::TW1 + K::TW2, 256> twr;  // twg: stage the twiddles here, loads issued with the window's
    if (twg) twr.load(twg, tid);
    cf v[E];
    if (active) {
        const cf* pz = reinterpret_cast<const cf*>(prev_c);
        const cf* iz = reinterpret_cast<const cf*>(in_c);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int n = tid + m * T;
            if constexpr (OLA) v[m] = n < B / 2 ? ld_in_cf(iz + n, WT) : cf{0.f, 0.f};
            else v[m] = n < B / 2 ? pz[n] : ld_in_cf(iz + n - B / 2, WT);
        }
    }
    if (twg) twr.store(tw1, tid);
    if constexpr (WT && !OLA) {
        // the window's second half becomes the next call's first half, stored from registers (a
        // second system-scope read of the input would be another trip to memory): after every
        // lane's loads of the first half have landed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (active) {
            cf* pw = const_cast<cf*>(reinterpret_cast<const cf*>(prev_c));
#pragma unroll
            for (int m = E / 2; m < E; ++m) pw[tid + m * T - B / 2] = v[m];
        }
    }
    __syncthreads();  // twiddles staged (here or by the caller)
    stockham<B, E, -1>(v, fft, tw1, tid, active);
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) fft[lpad(tid + m * T)] = v[m];
    }
    __syncthreads();
}

// c2r of the packed spectrum X (LDS), scaled by 1/2B (fallback_rfft_plan.hpp:38-55):
//   OLS: out = window samples [B, 2B)                       (overlap_save.hpp:104-111)
//   OLA: out = samples [0, B) + overlap; overlap = [B, 2B)  (overlap_add.hpp:92-106)
// E = 4 keeps the fused kernel inside its 64-VGPR budget (T = B/E <= 256 lanes).
// WS = true: run by one wave (T <= 64 lanes), no workgroup barriers.
// JOINED = true: X already holds the joined c2r input Z[k] (c2r_join applied by the caller).
// WT = true: the output block is stored write-through at system scope (the latency mode hands it
// to the host after s_waitcnt alone, no L2 write-back on its path)
__device__ __forceinline__ void st_out(cf* p, cf v, bool wt)
{
    if (wt) __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *p = v;
}

template<int B, bool OLA, int E = (B / 4 <= 256 ? 4 : B / 256), bool WS = false, bool JOINED = false, bool WT = false>
__device__ __forceinline__ void c2r_tail(const cf* X, cf* fft, const cf* tw, float* out_c, float* ovl_c, int tid)
{
    using K = upols_cfg<B>;
    constexpr int T = B / E;
    static_assert(T <= (WS ? 64 : 256) && B % E == 0, "c2r must fit one 256-lane workgroup (one wave for WS)");
    const bool active = tid < T;
    cf v[E];
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = tid + m * T;
            if constexpr (JOINED) {
                v[m] = X[k];
            } else {
                const cf x0 = X[0];
                v[m] = k == 0 ? c2r_join<B>(cf{x0.x, 0.f}, cf{x0.y, 0.f}, tw + K::TW1, 0)
                              : c2r_join<B>(X[k], X[B - k], tw + K::TW1, k);
            }
        }
    }
    stockham<B, E, +1, 1, WS>(v, fft, tw, tid, active);
    if (active) {
        const float scale = 1.0f / float(2 * B);  // overlap_save.hpp:107-108 / overlap_add.hpp:98
        cf* o = reinterpret_cast<cf*>(out_c);
        if constexpr (OLA) {
            cf* ov = reinterpret_cast<cf*>(ovl_c);
            // the same lane reads overlap[n] (m < E/2) before writing it (m >= E/2: n - B/2)
#pragma unroll
            for (int m = 0; m < E / 2; ++m) {
                const int n = tid + m * T;
                const cf old = ov[n];
                st_out(o + n, cf{v[m].x * scale + old.x, v[m].y * scale + old.y}, WT);
            }
#pragma unroll
            for (int m = E / 2; m < E; ++m) {
                const int n = tid + m * T;
                ov[n - B / 2] = {v[m].x * scale, v[m].y * scale};
            }
        } else {
#pragma unroll
            for (int m = E / 2; m < E; ++m) {  // window samples [B, 2B): z[n], n >= B/2
                const int n = tid + m * T;
                st_out(o + n - B / 2, cf{v[m].x * scale, v[m].y * scale}, WT);
            }
        }
    }
}

}  // namespace neo_hip
