// upols_far.hip — two-level lookahead: the far partitions of a 128-block window by a
// transform along the partition axis (opt-in, NEO_HIP_FAR=1; DESIGN.md §5 "Far field").
//
// Per bin k the UPOLS output spectrum is a convolution along the block axis,
//   Y[t][k] = sum_p H[p][k] X[t - p][k]      (uniform_partitioned_convolver.hpp:47-65,
//                                              fdl_index.hpp:23-36: partition p meets FDL row w - p)
// For the T2 = 128 blocks t0 + j of a level-2 window, the partitions p >= T2 only meet FDL
// rows written before t0. Cut them into segments q >= 1 of T2 partitions; segment q is a
// T2-tap FIR over the 2 T2 rows S_q[i] = X[t0 - (q+1) T2 + i], and its outputs for j < T2 are
// samples T2 .. 2T2-1 of the 256-point circular convolution of S_q with the zero-padded
// segment (no wrap reaches them). So, per channel and bin,
//   FF[j] = IDFT256( sum_q DFT256(S_q) . DFT256(h_q) )[T2 + j] / 256,
// 2 (Q - 1) * 256 complex MACs per bin per window instead of 128 * (P - 128): the far field
// becomes a stream of the segment spectra (precomputed at filter set) and the FDL, read once
// per 128 blocks. The level-1 lookahead pass then walks partitions < T2 only, and each block
// step adds FF[j] to its slabs.
//
// Packed bin 0 holds two real sequences (DC, Nyquist), so its partition-axis convolution is
// two real convolutions: with Z = DFT(x_dc + i x_ny) and G = DFT(h_dc + i h_ny), the packed
// result's spectrum is Z[f] A[f] + conj(Z[-f]) Bv[f], A = (Hdc + Hny) / 2, Bv = (Hdc - Hny) / 2,
// Hdc = (G[f] + conj(G[-f])) / 2, Hny = (G[f] - conj(G[-f])) / 2i. A takes bin 0's slot of the
// segment spectra, Bv a side array.
#include "fft_device.hpp"
#include "upols_handle.hpp"

namespace neo_hip {

#ifndef NEO_FAR_WAVES
#define NEO_FAR_WAVES 2  // A/B builds: waves per SIMD the far MAC is register-capped for
#endif
#ifndef NEO_FAR_PLAIN
#define NEO_FAR_PLAIN 0  // A/B builds: 1 = default-policy loads in the far MAC
#endif
__device__ __forceinline__ cf far_ld(const cf* p)
{
    if constexpr (NEO_FAR_PLAIN) return *p;
    else return ld_nt(p);
}

constexpr int kFarN = 2 * kFarT;  // partition-axis transform length
constexpr int kFarL = 256;        // lanes per workgroup: 16 row groups x 16 bin pairs (32 bins)

// 256-point transform of two bins' columns held by lane (a, cp): on entry v[n2] = x[a + 16 n2],
// on exit v[k1] = X[16 k1 + a] (four-step: 16-point DFTs in registers, twiddle, LDS transpose)
template<int DIR>
__device__ __forceinline__ void col_fft(cf (&v)[16], cf* lds, const cf* tw, int a, int cp)
{
    dft<16, DIR>(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], twiddle<kFarN, DIR>(tw, a * k));
#pragma unroll
    for (int k = 0; k < 16; ++k) lds[(k * 16 + a) * 16 + cp] = v[k];
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 16; ++n) v[n] = lds[(a * 16 + n) * 16 + cp];
    __syncthreads();
    dft<16, DIR>(v);
}

// bin 0's partner values v(-f) for f = 16 k1 + a, through LDS (uniform per workgroup)
__device__ __forceinline__ void mirror0(const cf (&v)[16], cf (&m)[16], cf* z, int a, int cp)
{
    if (cp == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) z[16 * k + a] = v[k];
    }
    __syncthreads();
    if (cp == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) m[k] = z[(kFarN - (16 * k + a)) & (kFarN - 1)];
    }
    __syncthreads();
}

// Segment spectra (grid C x (Q-1) x B/32): hf[c][q-1][f][k] = DFT256(H[c][q T2 + r][k], r < T2),
// bin 0 -> A, hf0[c][q-1][f] = Bv.
__global__ __launch_bounds__(kFarL) void k_far_filter(const cf* __restrict__ H, cf* __restrict__ hf,
                                                      cf* __restrict__ hf0, const cf* __restrict__ twg, int B, int P,
                                                      int Q1, int64_t cstride, int64_t pstride)
{
    __shared__ cf lds[2][16 * 16 * 16];
    __shared__ cf z[kFarN];
    __shared__ cf tw[kFarN];
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int ng = B / 32, bg = blockIdx.x % ng, cq = blockIdx.x / ng, q = cq % Q1 + 1, c = cq / Q1;
    const int kb = bg * 32 + 2 * cp;
    tw[t] = twg[t];
    __syncthreads();
    cf v0[16], v1[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
        const int r = a + 16 * n2, p = q * kFarT + r;
        float4 x = {0.f, 0.f, 0.f, 0.f};
        if (r < kFarT && p < P) x = *reinterpret_cast<const float4*>(H + int64_t(c) * cstride + int64_t(p) * pstride + kb);
        v0[n2] = {x.x, x.y};
        v1[n2] = {x.z, x.w};
    }
    col_fft<-1>(v0, lds[0], tw, a, cp);
    col_fft<-1>(v1, lds[1], tw, a, cp);
    const bool b0 = bg == 0;
    cf g0[16];
    if (b0) mirror0(v0, g0, z, a, cp);
    cf* dst = hf + (int64_t(c) * Q1 + (q - 1)) * kFarN * B;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int f = 16 * k + a;
        cf o0 = v0[k];
        if (b0 && cp == 0) {
            const cf g = v0[k], gm = cconj(g0[k]);
            const cf hdc = cscale(cadd(g, gm), 0.5f);
            const cf d = cscale(csub(g, gm), 0.5f);
            const cf hny = {d.y, -d.x};  // d / i
            o0 = cscale(cadd(hdc, hny), 0.5f);
            hf0[(int64_t(c) * Q1 + (q - 1)) * kFarN + f] = cscale(csub(hdc, hny), 0.5f);
        }
        *reinterpret_cast<float4*>(dst + int64_t(f) * B + kb) = make_float4(o0.x, o0.y, v1[k].x, v1[k].y);
    }
}

// Far field of one level-2 window (grid C x B/16, one bin per lane): FF[c][j][k] for j < T2,
// from the FDL rows before write position w (rows older than P - 1 blocks meet only zero
// filter taps and read 0). Segment q + 1's rows 128..255 are segment q's rows 0..127, so each
// lane keeps them in registers: the FDL is read once per window (a 2-bin-per-lane first
// version held 300 registers, ran at 1 wave/SIMD and took 2.0 ms at C5).
__global__ __launch_bounds__(kFarL) __attribute__((amdgpu_waves_per_eu(NEO_FAR_WAVES))) void k_far_mac(const cf* __restrict__ fdl, const cf* __restrict__ hf,
                                                   const cf* __restrict__ hf0, cf* __restrict__ ff,
                                                   const cf* __restrict__ twg, int B, int P, int Q1, int ring, int w,
                                                   int64_t cstride, int64_t pstride)
{
    __shared__ cf lds[16 * 16 * 16];
    __shared__ cf z[kFarN];
    __shared__ cf z0[kFarN];  // bin 0's Bv coefficients of the current segment
    __shared__ cf tw[kFarN];
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int ng = B / 16, bg = blockIdx.x % ng, c = blockIdx.x / ng;
    const int kb = bg * 16 + cp;
    const bool b0 = bg == 0;  // uniform per workgroup: bin 0 (packed DC / Nyquist) is lane cp == 0's
    tw[t] = twg[t];
    __syncthreads();
    const cf* F = fdl + int64_t(c) * cstride + kb;
    // FDL row n2 (< 16) of segment q, zero where it is older than P - 1 blocks
    auto row = [&](int q, int n2) {
        const int d = (q + 1) * kFarT - (a + 16 * n2);  // blocks before t0 (>= 1)
        if (d >= P) return cf{0.f, 0.f};
        const int r = w - d < 0 ? w - d + ring : w - d;
        return far_ld(F + int64_t(r) * pstride);
    };
    cf acc[16], v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        acc[k] = cf{0.f, 0.f};
        v[k] = row(1, k);
    }
    for (int q = 1; q <= Q1; ++q) {
        // issue this segment's spectra and the next segment's new rows before the transform
        // (the barriers inside it wait on LDS only, so the loads stay in flight)
        const cf* hq = hf + (int64_t(c) * Q1 + (q - 1)) * kFarN * B + kb;
        cf h[16], nx[8];
#pragma unroll
        for (int k = 0; k < 16; ++k) h[k] = far_ld(hq + int64_t(16 * k + a) * B);
#pragma unroll
        for (int n2 = 0; n2 < 8; ++n2) nx[n2] = q < Q1 ? row(q + 1, n2) : cf{0.f, 0.f};
        const cf b0v = b0 ? hf0[(int64_t(c) * Q1 + (q - 1)) * kFarN + t] : cf{0.f, 0.f};
        cf keep[8];
#pragma unroll
        for (int n2 = 0; n2 < 8; ++n2) keep[n2] = v[n2];
        col_fft<-1>(v, lds, tw, a, cp);
        if (b0) {
            if (cp == 0) {
#pragma unroll
                for (int k = 0; k < 16; ++k) z[16 * k + a] = v[k];
            }
            z0[t] = b0v;  // the previous segment's reads of z / z0 ended before col_fft's barriers
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int f = 16 * k + a;
            acc[k] = cadd(acc[k], cmul(v[k], h[k]));
            if (b0 && cp == 0)
                acc[k] = cadd(acc[k], cmul(cconj(z[(kFarN - f) & (kFarN - 1)]), z0[f]));
        }
#pragma unroll
        for (int n2 = 0; n2 < 8; ++n2) {  // segment q + 1's rows 128.. are this segment's rows 0..127
            v[n2] = nx[n2];
            v[n2 + 8] = keep[n2];
        }
    }
    // inverse along f: acc[k1] sits at f = a + 16 k1, the layout col_fft takes
    col_fft<1>(acc, lds, tw, a, cp);
    constexpr float s = 1.0f / kFarN;
    cf* o = ff + int64_t(c) * kFarT * B + kb;
#pragma unroll
    for (int m = 8; m < 16; ++m) {  // n = 16 m + a >= T2: output block j = n - T2
        const int j = 16 * (m - 8) + a;
        o[int64_t(j) * B] = cscale(acc[m], s);
    }
}

bool far_usable(const upols_t* h)
{
    return h->far && h->ahead && h->akern == 2 && h->B >= 32 && h->B <= 1024 && h->P > kFarT &&
           batch_blocks(h) == kMaxBatch && kFarT % kMaxBatch == 0;
}

int far_filter(upols_t* h, hipStream_t s)
{
    h->fwin = -1;
    if (!h->far || h->B < 32 || h->P <= kFarT) return NEO_HIP_OK;
    const int Q1 = (h->P + kFarT - 1) / kFarT - 1;
    if (!h->hf) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->hf), size_t(h->C) * Q1 * kFarN * h->B * sizeof(cf)));
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->hf0), size_t(h->C) * Q1 * kFarN * sizeof(cf)));
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->ff), size_t(h->C) * kFarT * h->B * sizeof(cf)));
        const auto t = make_twiddle_table(kFarN);
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->twf), t.size() * sizeof(cf)));
        NEO_HIP_CHECK(hipMemcpy(h->twf, t.data(), t.size() * sizeof(cf), hipMemcpyHostToDevice));
    }
    const unsigned grid = unsigned(h->C) * unsigned(Q1) * unsigned(h->B / 32);
    hipLaunchKernelGGL(k_far_filter, dim3(grid), dim3(kFarL), 0, s, h->H, h->hf, h->hf0, h->twf, h->B, h->P, Q1,
                       h->cstride, h->pstride);
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

int far_window(upols_t* h, hipStream_t s)
{
    const int Q1 = (h->P + kFarT - 1) / kFarT - 1;
    const unsigned grid = unsigned(h->C) * unsigned(h->B / 16);
    hipLaunchKernelGGL(k_far_mac, dim3(grid), dim3(kFarL), 0, s, h->fdl, h->hf, h->hf0, h->ff, h->twf, h->B, h->P, Q1,
                       h->ring, h->wpos, h->cstride, h->pstride);
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

}  // namespace neo_hip
