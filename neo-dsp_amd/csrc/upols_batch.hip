// upols_batch.hip — batched passes for process_blocks / process_samples / dense_convolve:
// T consecutive blocks of every channel share ONE pass over the filter and the FDL
// (window r2c + insert, MAC with a sliding FDL window in registers, per-block finish,
// OLA overlap chain). Same results as T single-block steps up to summation order.
// (The streaming one-block-per-call step is upols_levels.hip.)
#include "upols_device.hpp"
#include "upols_handle.hpp"

#include <algorithm>
#include <vector>

#include <type_traits>
#include <utility>

namespace neo_hip {

// Block j of a batch (write position w) is inserted as FDL row (w + j) mod R and uses
// rows (w + j - p) mod R, so partition p of all T blocks reads one H row and T rows of
// the FDL of which T - 1 were already read for p - 1: a workgroup that walks p in order
// keeps a sliding window of T FDL rows in registers and streams one H row and one new
// FDL row per partition. HBM bytes per pass stay ~16·P·B per channel (the single-block
// figure) while the pass produces T blocks: T× the work per byte.
template<int B, int NB>
struct batch_cfg {
    static constexpr int Q = B / NB;               // vectors (NB bins each) per row
    static constexpr int L = Q < 256 ? Q : 256;    // lanes per MAC workgroup
    static constexpr int VPT = 1;                  // vectors per lane
    static constexpr int G = Q / L;                // workgroups per row (bin chunks): several
                                                   // small workgroups per CU run out of phase
};
template<int NB>
using bvec = std::conditional_t<NB == 2, f4v, f2v>;  // NB interleaved complex bins

// Window r2c of block j (grid C x T): [x_{j-1} | x_j] (OLS, x_{-1} = prev) or [x_j | 0]
// (OLA), inserted as FDL row (w + j) mod R.
template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_batch_window(const float* __restrict__ in, int64_t ld_in,
                                                      const float* __restrict__ prev, cf* __restrict__ fdl,
                                                      const cf* __restrict__ twg, int T, int ring, int w,
                                                      int64_t cstride, int64_t pstride)
{
    using K = upols_cfg<B>;
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x / T, j = blockIdx.x - c * T;
    const float* in_c = in + int64_t(c) * ld_in + int64_t(j) * B;
    const float* prev_c = j == 0 ? prev + int64_t(c) * B : in_c - B;
    window_fft<B, OLA>(prev_c, in_c, fft, tw, tid, twg);
    const int r = w + j < ring ? w + j : w + j - ring;
    cf* row = fdl + int64_t(c) * cstride + int64_t(r) * pstride;
    for (int k = tid; k < B; k += 256) row[k] = r2c_split<B>(fft, tw + K::TW1, k);
}

// Per bin two packed pairs d = (sum hr*xr, sum hi*xi) and x = (sum hr*xi, sum hi*xr): each
// is one v_pk_fma_f32 per partition (x with the operand halves swapped), and the packed
// bin 0 stays exact: bin 0 -> d (DC, Nyquist), other bins -> {d.x - d.y, x.x + x.y}.
struct acc3 {
    f2v d, x;
};

// Row loads of the batched MAC. BUF = false: flat global loads (64-bit address per lane
// and row). BUF = true: buffer loads over a per-channel descriptor, the lane's byte
// offset fixed in a VGPR and the row offset in an SGPR (no per-row address VALU).
// HNT: filter rows nontemporal (true) or with the default policy, so that the first rows of
// each channel stay resident in the Infinity Cache across passes (false).
template<class V, bool BUF, bool HNT = true>
struct row_src {
    const V* Hv;
    const V* Fv;
    int64_t psv;                   // row stride in vectors
    __amdgpu_buffer_rsrc_t Hr, Fr;
    int prow;                      // row stride in bytes
    // FDL row entering the sliding window at partition pn (write position w)
    __device__ __forceinline__ int frow(int w, int pn, int ring) const
    {
        const int r = w - pn;
        return r < 0 ? r + ring : r;
    }
    __device__ __forceinline__ V h(int p, int lane) const
    {
        if constexpr (BUF) {
            // (a per-row cacheable/nontemporal select here cost 54 spilled VGPRs at 256: the policy
            // is a template argument and the partition loop runs in two ranges instead)
            const auto u = __builtin_amdgcn_raw_buffer_load_b64(Hr, lane * int(sizeof(V)), p * prow, HNT ? 2 : 0);
            return __builtin_bit_cast(V, u);
        } else {
            if constexpr (HNT) return __builtin_nontemporal_load(Hv + int64_t(p) * psv + lane);
            else return Hv[int64_t(p) * psv + lane];
        }
    }
    __device__ __forceinline__ V f(int r, int lane) const
    {
        if constexpr (BUF) {
            auto u = __builtin_amdgcn_raw_buffer_load_b64(Fr, lane * int(sizeof(V)), r * prow, 2 /* nt */);
            return __builtin_bit_cast(V, u);
        } else {
            return __builtin_nontemporal_load(Fv + int64_t(r) * psv + lane);
        }
    }
};

// Step U of a T-step chunk (p = pb + U; U is a template argument so every slot index
// is static and the arrays stay in registers): take H row p and FDL row (w - p) from
// prefetch slot U mod D (loaded D steps earlier) into window slot (T - U) mod T, issue
// the loads for p + D, then MAC all T blocks; block j reads window slot (j - U) mod T.
// D bounds the loads in flight per lane (and so the registers they hold).
//   A2 = false: four partial products per bin in two packed pairs (acc3 d and x).
//   A2 = true:  one packed pair per bin, the complex product itself: (re, im) +=
//     (hr, hr)(xr, xi) + (-hi, hi)(xi, xr) -- two v_pk_fma_f32 as before, half the
//     accumulator registers. The lane holding the packed bin 0 (DC, Nyquist: two real
//     products) takes the operands (hr, hi) and (0, 0) instead, so its pair sums
//     (hr xr, hi xi) = (DC, Nyquist) exactly as the four-product form does.
template<int T, int NB, int VPT, int L, int D, bool A2, int U, class SRC>
__device__ __forceinline__ void batch_step(acc3 (&a)[T][NB * VPT], bvec<NB> (&f)[T][VPT], bvec<NB> (&ph)[D][VPT],
                                           bvec<NB> (&pf)[D][VPT], const SRC& src, int tid, int ring, int w, int p)
{
    constexpr int slot = U % D;
    bvec<NB> hv[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        f[(T - U) % T][v] = pf[slot][v];
        hv[v] = ph[slot][v];
    }
    const int pn = p + D < ring ? p + D : ring - 1;  // stay inside the allocated rows
    {
        const int r = src.frow(w, pn, ring);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[slot][v] = src.f(r, tid + v * L);
            ph[slot][v] = src.h(pn, tid + v * L);
        }
    }
    if constexpr (A2) {
        f2v h1[VPT][NB], h2[VPT][NB];
#pragma unroll
        for (int v = 0; v < VPT; ++v)
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const float hr = hv[v][2 * b], hi = hv[v][2 * b + 1];
                const bool z = b == 0 && tid + v * L == 0;  // packed bin 0
                const float s = z ? 0.0f : hi;
                h1[v][b] = {hr, z ? hi : hr};
                h2[v][b] = {-s, s};
            }
        // two sweeps over the blocks, so consecutive FMAs never chain on one accumulator
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < T; ++j)
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    const bvec<NB> x = f[(j - U + T) % T][v];
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        acc3& A = a[j][v * NB + b];
                        const f2v xb = {x[2 * b], x[2 * b + 1]};
                        A.d = k == 0 ? __builtin_elementwise_fma(h1[v][b], xb, A.d)
                                     : __builtin_elementwise_fma(h2[v][b], xb.yx, A.d);
                    }
                }
    } else {
#pragma unroll
        for (int j = 0; j < T; ++j)
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                const bvec<NB> x = f[(j - U + T) % T][v], h = hv[v];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    acc3& A = a[j][v * NB + b];
                    const f2v hb = {h[2 * b], h[2 * b + 1]}, xb = {x[2 * b], x[2 * b + 1]};
                    A.d = __builtin_elementwise_fma(hb, xb, A.d);
                    A.x = __builtin_elementwise_fma(hb, xb.yx, A.x);
                }
            }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep each step's loads D steps ahead, not all hoisted
}

template<int T, int NB, int VPT, int L, int D, bool A2, class SRC, int... U>
__device__ __forceinline__ void batch_chunk(acc3 (&a)[T][NB * VPT], bvec<NB> (&f)[T][VPT], bvec<NB> (&ph)[D][VPT],
                                            bvec<NB> (&pf)[D][VPT], const SRC& src, int tid, int ring, int w, int pb,
                                            std::integer_sequence<int, U...>)
{
    (batch_step<T, NB, VPT, L, D, A2, U>(a, f, ph, pf, src, tid, ring, w, pb + U), ...);
}

// MAC pass for T blocks (grid C x S, batch_cfg<B, NB>::L lanes, NB bins per lane-vector):
// workgroup (c, s) walks partitions [p0, p1) and writes T partial spectra to
// part[c][s][j][B].
// Variants: accumulator form, prefetch depth D (divides T, so slots line up across chunks)
// and the waves per SIMD the register budget is sized for. Variant 3 is the one for the
// B = 256 / 512 passes (A/B on MI355X, C5 / C4 per pass: variant 0 0.45 / 0.40 ms, complex
// accumulators at D = 4 and 3 waves/SIMD slower, at D = 8 0.405 / 0.400, with buffer loads
// (3) 0.367-0.393 / 0.369-0.384; an LDS-DMA row ring 0.383 / 0.388); variant 0 (flat loads,
// any B and T) serves the rest.
template<int V>
struct bmac_var;
template<>
struct bmac_var<0> {  // four partial products per bin (acc3), D = 4, 256 VGPRs
    static constexpr bool A2 = false, BUF = false;
    static constexpr int D = 4, W = 2;
};
template<>
struct bmac_var<3> {  // complex accumulators, D = 8, buffer loads (row offsets in SGPRs), 256 VGPRs
    static constexpr bool A2 = true, BUF = true;
    static constexpr int D = 8, W = 2;
};

template<int B, int T, int NB, int VAR, int D0 = bmac_var<VAR>::D, int D = (T < D0 ? T : D0)>
__global__ __launch_bounds__((batch_cfg<B, NB>::L), bmac_var<VAR>::W) void k_batch_mac(const cf* __restrict__ H,
                                                                   const cf* __restrict__ fdl, cf* __restrict__ part,
                                                                   int P, int ring, int S, int rows, int w,
                                                                   int64_t cstride, int64_t pstride, int pc)
{
    using K = batch_cfg<B, NB>;
    using V = bvec<NB>;
    constexpr int VPT = K::VPT, L = K::L;
    constexpr int G = K::G;
    const int cs = blockIdx.x / G, gch = blockIdx.x - cs * G;
    const int tid = gch * L + threadIdx.x;  // vector index within the row (bin chunk gch)
    const int c = cs / S, s = cs - c * S;
    const int p0 = s * rows, p1 = min(P, p0 + rows);
    const int64_t psv = pstride / NB;  // row stride in vectors
    const V* Hv = reinterpret_cast<const V*>(H + int64_t(c) * cstride);
    const V* Fv = reinterpret_cast<const V*>(fdl + int64_t(c) * cstride);
    constexpr bool BUF = bmac_var<VAR>::BUF;
    const int span = BUF ? int(((ring - 1) * pstride + B) * int64_t(sizeof(cf))) : 0;  // < 2 GiB (host check)
    const row_src<V, BUF> src{Hv, Fv, psv, __builtin_amdgcn_make_buffer_rsrc(const_cast<V*>(Hv), 0, span, 0x00020000),
                              __builtin_amdgcn_make_buffer_rsrc(const_cast<V*>(Fv), 0, span, 0x00020000),
                              int(pstride * int64_t(sizeof(cf)))};
    // filter rows p < pc with the default (cacheable) policy: the same rows every pass, kept
    // in the Infinity Cache; the nontemporal stream of the rest does not evict them
    const row_src<V, BUF, false> src_c{src.Hv, src.Fv, src.psv, src.Hr, src.Fr, src.prow};

    acc3 a[T][NB * VPT];
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
        for (int v = 0; v < NB * VPT; ++v) a[j][v] = {f2v(0.0f), f2v(0.0f)};
    V f[T][VPT];
#pragma unroll
    for (int sl = 1; sl < T; ++sl) {  // rows block sl needs at p0 (entered at partition p0 - sl)
        int r = w + sl - p0;
        r = r < 0 ? r + ring : (r >= ring ? r - ring : r);
#pragma unroll
        for (int v = 0; v < VPT; ++v) f[sl][v] = src.f(r, tid + v * L);
    }
    V ph[D][VPT], pf[D][VPT];
#pragma unroll
    for (int d = 0; d < D; ++d) {  // prefetch partitions p0 .. p0 + D - 1
        const int p = p0 + d < ring ? p0 + d : ring - 1;  // past P: zero filter rows
        const int r = src.frow(w, p, ring);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[d][v] = src.f(r, tid + v * L);
            ph[d][v] = BUF && p < pc ? src_c.h(p, tid + v * L) : src.h(p, tid + v * L);
        }
    }
    // splits hold a multiple of T partitions; the last split's final chunk runs past P into
    // the ring's spare filter rows, which are zero (so those steps add nothing). Chunks
    // starting below pc load filter rows cacheable, the rest nontemporally.
    // Two workgroups share a CU (blockIdx i and i + grid/2, the dispatch order) and the SQ
    // favours the older one's waves, which finish ~30 % early and leave one wave per SIMD for
    // the rest of the pass; they trade issue priority in slices of 2^11 s_memrealtime ticks
    // (100 MHz: 20 us; same-box A/B: pass 2-10 % shorter; 2^13 ties, 2^9 and uneven shares
    // lose; locking the two together with a barrier per chunk was 30 % slower: both then
    // stall on memory at the same time).
    const int half = blockIdx.x >= gridDim.x / 2;
    auto share = [&]() {
        const bool mine_old = ((__builtin_amdgcn_s_memrealtime() >> 11) & 1) == 0;
        if (half ? !mine_old : mine_old) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
    };
    int pb = p0;
    for (; BUF && pb < p1 && pb < pc; pb += T) {  // (flat-load variants: all nontemporal, no spills)
        share();
        batch_chunk<T, NB, VPT, L, D, bmac_var<VAR>::A2>(a, f, ph, pf, src_c, tid, ring, w, pb,
                                                          std::make_integer_sequence<int, T>{});
    }
    for (; pb < p1; pb += T) {
        share();
        batch_chunk<T, NB, VPT, L, D, bmac_var<VAR>::A2>(a, f, ph, pf, src, tid, ring, w, pb,
                                                          std::make_integer_sequence<int, T>{});
    }
    __builtin_amdgcn_s_setprio(0);

    cf* slab = part + (int64_t(c) * S + s) * T * B;
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            V o;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const acc3& A = a[j][v * NB + b];
                const bool bin0 = tid + v * L == 0 && b == 0;
                if constexpr (bmac_var<VAR>::A2) {
                    o[2 * b] = A.d.x;
                    o[2 * b + 1] = A.d.y;
                } else {
                    o[2 * b] = bin0 ? A.d.x : A.d.x - A.d.y;
                    o[2 * b + 1] = bin0 ? A.d.y : A.x.x + A.x.y;
                }
            }
            *reinterpret_cast<V*>(slab + int64_t(j) * B + (tid + v * L) * NB) = o;
        }
}

// Sum the S slabs of block j in order, c2r, 1/2B (grid C x T, 256 lanes).
//   OLS: out_j = window samples [B, 2B); workgroup j = T-1 first saves x_{T-1} as the
//        next batch's previous block (before out_j, which may alias it, is written).
//   OLA: out_j = samples [0, B) (overlap added by k_batch_ola), tail_j = [B, 2B).
template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_batch_finish(const cf* __restrict__ part, int S, int T,
                                                      const float* __restrict__ in, int64_t ld_in,
                                                      float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
                                                      float* __restrict__ tail, const cf* __restrict__ twg)
{
    using K = upols_cfg<B>;
    constexpr int E = NEO_BATCH_FINISH_E(B), TT = B / E;  // more lanes in the c2r than the 16-element form
    __shared__ __attribute__((aligned(16))) cf X[B];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x / T, j = blockIdx.x - c * T;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    if (!OLA && j == T - 1) {
        const float4* x4 = reinterpret_cast<const float4*>(in + int64_t(c) * ld_in + int64_t(j) * B);
        float4* p4 = reinterpret_cast<float4*>(prev + int64_t(c) * B);
        for (int i = tid; i < B / 4; i += 256) p4[i] = x4[i];
    }
    const float4* s4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * T * B + int64_t(j) * B);
    const int64_t sstride = int64_t(T) * K::Q;  // float4 between consecutive slabs of one block
    for (int q = tid; q < K::Q; q += 256) {
        float4 sum = s4[q];
        for (int t = 1; t < S; ++t) {
            const float4 r = s4[t * sstride + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        reinterpret_cast<float4*>(X)[q] = sum;
    }
    __syncthreads();
    const bool active = tid < TT;
    cf v[E];
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = tid + m * TT;
            const cf x0 = X[0];
            v[m] = k == 0 ? c2r_join<B>(cf{x0.x, 0.f}, cf{x0.y, 0.f}, tw + K::TW1, 0)
                          : c2r_join<B>(X[k], X[B - k], tw + K::TW1, k);
        }
    }
    stockham<B, E, +1>(v, fft, tw, tid, active);
    if (active) {
        const float scale = 1.0f / float(2 * B);
        cf* o = reinterpret_cast<cf*>(out + int64_t(c) * ld_out + int64_t(j) * B);
        if constexpr (OLA) {
            cf* tl = reinterpret_cast<cf*>(tail + (int64_t(c) * T + j) * B);
#pragma unroll
            for (int m = 0; m < E / 2; ++m) o[tid + m * TT] = {v[m].x * scale, v[m].y * scale};
#pragma unroll
            for (int m = E / 2; m < E; ++m) tl[tid + m * TT - B / 2] = {v[m].x * scale, v[m].y * scale};
        } else {
#pragma unroll
            for (int m = E / 2; m < E; ++m) o[tid + m * TT - B / 2] = {v[m].x * scale, v[m].y * scale};
        }
    }
}

// OLA overlap for a batch (grid C): out_j += tail_{j-1} (out_0 += overlap), overlap = tail_{T-1}
template<int B>
__global__ __launch_bounds__(256) void k_batch_ola(float* __restrict__ out, int64_t ld_out,
                                                   const float* __restrict__ tail, float* __restrict__ ovl, int T)
{
    const int c = blockIdx.x;
    float* o = out + int64_t(c) * ld_out;
    const float* tl = tail + int64_t(c) * T * B;
    float* ov = ovl + int64_t(c) * B;
    for (int i = threadIdx.x; i < B; i += 256) {
        float carry = ov[i];
        for (int j = 0; j < T; ++j) {
            o[int64_t(j) * B + i] += carry;
            carry = tl[int64_t(j) * B + i];
        }
        ov[i] = carry;
    }
}
// ---------------------------------------------------------------------------------------
// host side

// one k_batch_mac launch: T blocks at write position h->wpos into the slabs part_b
// [C][Sb][T][B], splits of rows_b partitions over [0, P)
template<int BB, int NB>
int launch_batch_mac(const upols_t* h, int T, hipStream_t s)
{
    constexpr int L = batch_cfg<BB, NB>::L;
    const unsigned grid = unsigned(h->C) * unsigned(h->Sb) * unsigned(batch_cfg<BB, NB>::G);
#define NEO_BATCH_T(TT)                                                                                          \
    case TT:                                                                                                     \
        if constexpr (batch_t(BB, NB, TT) == TT) {                                                               \
            if constexpr ((TT == 32 || TT == 16 || TT == 8) && NB == 1 && (BB == 256 || BB == 512)) {            \
                if (h->bufload) {                                                                                \
                    hipLaunchKernelGGL((k_batch_mac<BB, TT, NB, 3>), dim3(grid), dim3(L), 0, s, h->H, h->fdl,    \
                                       h->part_b, h->P, h->ring, h->Sb, h->rows_b, h->wpos, h->cstride,          \
                                       h->pstride, h->pcb);                                                      \
                    break;                                                                                       \
                }                                                                                                \
            }                                                                                                    \
            hipLaunchKernelGGL((k_batch_mac<BB, TT, NB, 0>), dim3(grid), dim3(L), 0, s, h->H, h->fdl, h->part_b,  \
                               h->P, h->ring, h->Sb, h->rows_b, h->wpos, h->cstride, h->pstride, h->pcb);        \
            break;                                                                                               \
        }                                                                                                        \
        return fail(NEO_HIP_EINVAL, "batch of %d blocks not available at block %d", TT, BB);
    switch (T) {
        NEO_BATCH_T(2)
        NEO_BATCH_T(4)
        NEO_BATCH_T(8)
        NEO_BATCH_T(16)
        NEO_BATCH_T(32)
        default: return fail(NEO_HIP_EINVAL, "batch of %d blocks not available", T);
    }
#undef NEO_BATCH_T
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

static int batch_buffers(upols_t* h)
{
    if (!h->part_b) {
        if (int rc = dalloc(&h->part_b, size_t(h->C) * h->Sb * kMaxBatch * h->B * sizeof(cf))) return rc;
        if (h->ola && dalloc(&h->tail, size_t(h->C) * kMaxBatch * h->B * sizeof(float))) {
            dfree(h->part_b);
            h->part_b = nullptr;
            return fail(NEO_HIP_ENOMEM, "batched OLA tail allocation failed");
        }
    }
    return NEO_HIP_OK;
}

int launch_batch(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int T, hipStream_t s)
{
    const int B = h->B;
    int rc0 = batch_buffers(h);
    if (rc0) return rc0;
    const unsigned gCT = unsigned(h->C) * unsigned(T);
    if (int rc = lvl_join(h, s)) return rc;  // step-group slices still reading the FDL ring
    h->lv_n = -1;  // a streaming step after this re-primes its level windows
    h->fdl_zero = false;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, true>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, false>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    }
    NEO_HIP_LAUNCH_CHECK();
    upols_t::ev_group* ev = nullptr;
    int rc = timing_begin(h, 2, &ev);
    if (!rc) rc = timing_mark(ev, 0, s);
    if (rc) return rc;
    if (h->bNB == 2) {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s)))
    } else {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s)))
    }
    if (rc) return rc;
    if ((rc = timing_mark(ev, 1, s))) return rc;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_finish<BB, true>), dim3(gCT), dim3(256), 0, s, h->part_b,
                                                 h->Sb, T, in, ld_in, out, ld_out, h->prev, h->tail, h->tw))
        NEO_HIP_LAUNCH_CHECK();
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_ola<BB>), dim3(unsigned(h->C)), dim3(256), 0, s, out, ld_out,
                                                 h->tail, h->prev, T))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_finish<BB, false>), dim3(gCT), dim3(256), 0, s, h->part_b,
                                                 h->Sb, T, in, ld_in, out, ld_out, h->prev, h->tail, h->tw))
    }
    NEO_HIP_LAUNCH_CHECK();
    h->wpos = (h->wpos + T) % h->ring;
    return NEO_HIP_OK;
}

// Offline windows (k_off_mac, upols_levels.hip): wp windows of 128 blocks -- the window r2c of
// every block into FDL rows w .. w + 128 wp - 1, the partition-axis transforms of every segment,
// the per-block finish (one slab: k_off_mac's output spectra), OLA's overlap chain. The ring
// holds >= 128 (nseg + kOffMaxWP) rows (create), so the new rows overwrite none the pass reads.
int launch_offline(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int wp, hipStream_t s)
{
    const int B = h->B, T = kFarT * wp;
    if (!h->off_y) {
        const size_t rows = size_t(h->C) * kFarT * kOffMaxWP * B;
        if (int rc = dalloc(&h->off_y, rows * sizeof(cf))) return rc;
        if (dalloc(&h->off_hf, off_hf_bytes(h)) ||
            (h->ola && dalloc(&h->off_tail, rows * sizeof(float)))) {
            dfree(h->off_y);
            dfree(h->off_hf);
            h->off_y = nullptr;
            h->off_hf = nullptr;
            return fail(NEO_HIP_ENOMEM, "offline window buffers");
        }
        h->off_dirty = true;
    }
    const unsigned gCT = unsigned(h->C) * unsigned(T);
    if (int rc = lvl_join(h, s)) return rc;  // step-group slices still reading the FDL ring
    h->lv_n = -1;  // a streaming step after this re-primes its level windows
    h->fdl_zero = false;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, true>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, false>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    }
    NEO_HIP_LAUNCH_CHECK();
    upols_t::ev_group* ev = nullptr;
    int rc = timing_begin(h, 2, &ev);
    if (!rc) rc = timing_mark(ev, 0, s);
    if (!rc) rc = launch_off_mac(h, wp, s);
    if (!rc) rc = timing_mark(ev, 1, s);
    if (rc) return rc;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_finish<BB, true>), dim3(gCT), dim3(256), 0, s, h->off_y, 1, T,
                                                 in, ld_in, out, ld_out, h->prev, h->off_tail, h->tw))
        NEO_HIP_LAUNCH_CHECK();
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_ola<BB>), dim3(unsigned(h->C)), dim3(256), 0, s, out, ld_out,
                                                 h->off_tail, h->prev, T))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_finish<BB, false>), dim3(gCT), dim3(256), 0, s, h->off_y, 1,
                                                 T, in, ld_in, out, ld_out, h->prev, nullptr, h->tw))
    }
    NEO_HIP_LAUNCH_CHECK();
    h->wpos = (h->wpos + T) % h->ring;
    return NEO_HIP_OK;
}

}  // namespace neo_hip
