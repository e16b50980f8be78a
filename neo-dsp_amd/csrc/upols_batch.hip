// upols_batch.hip — batched passes for process_blocks / process_samples / dense_convolve:
// T consecutive blocks of every channel share ONE pass over the filter and the FDL
// (window r2c + insert, MAC with a sliding FDL window in registers, per-block finish,
// OLA overlap chain). Same results as T single-block steps up to summation order.
#include "upols_device.hpp"
#include "upols_handle.hpp"

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
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    const float* in_c = in + int64_t(c) * ld_in + int64_t(j) * B;
    const float* prev_c = j == 0 ? prev + int64_t(c) * B : in_c - B;
    window_fft<B, OLA>(prev_c, in_c, fft, tw, tid);
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

// Step U of a T-step chunk (p = pb + U; U is a template argument so every slot index
// is static and the arrays stay in registers): take H row p and FDL row (w - p) from
// prefetch slot U mod D (loaded D steps earlier) into window slot (T - U) mod T, issue
// the loads for p + D, then MAC all T blocks; block j reads window slot (j - U) mod T.
// D bounds the loads in flight per lane (and so the registers they hold).
template<int T, int NB, int VPT, int L, int D, int U>
__device__ __forceinline__ void batch_step(acc3 (&a)[T][NB * VPT], bvec<NB> (&f)[T][VPT], bvec<NB> (&ph)[D][VPT],
                                           bvec<NB> (&pf)[D][VPT], const bvec<NB>* Hv, const bvec<NB>* Fv,
                                           int64_t psv, int tid, int ring, int w, int p, int p1)
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
        int r = w - pn;
        r = r < 0 ? r + ring : r;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[slot][v] = __builtin_nontemporal_load(Fv + int64_t(r) * psv + tid + v * L);
            ph[slot][v] = __builtin_nontemporal_load(Hv + int64_t(pn) * psv + tid + v * L);
        }
    }
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
    __builtin_amdgcn_sched_barrier(0);  // keep each step's loads D steps ahead, not all hoisted
}

template<int T, int NB, int VPT, int L, int D, int... U>
__device__ __forceinline__ void batch_chunk(acc3 (&a)[T][NB * VPT], bvec<NB> (&f)[T][VPT], bvec<NB> (&ph)[D][VPT],
                                            bvec<NB> (&pf)[D][VPT], const bvec<NB>* Hv, const bvec<NB>* Fv,
                                            int64_t psv, int tid, int ring, int w, int pb, int p1,
                                            std::integer_sequence<int, U...>)
{
    (batch_step<T, NB, VPT, L, D, U>(a, f, ph, pf, Hv, Fv, psv, tid, ring, w, pb + U, p1), ...);
}

// MAC pass for T blocks (grid C x S, batch_cfg<B, NB>::L lanes, NB bins per lane-vector):
// workgroup (c, s) walks partitions [p0, p1) and writes T partial spectra to
// part[c][s][j][B].
#ifndef NEO_BATCH_D
#define NEO_BATCH_D 4
#endif
template<int B, int T, int NB, int D = (T < NEO_BATCH_D ? T : NEO_BATCH_D)>  // D divides T: slots line up across chunks
__global__ __launch_bounds__((batch_cfg<B, NB>::L), 2) void k_batch_mac(const cf* __restrict__ H,
                                                                   const cf* __restrict__ fdl, cf* __restrict__ part,
                                                                   int P, int ring, int S, int rows, int w,
                                                                   int64_t cstride, int64_t pstride, int ahead)
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

    acc3 a[T][NB * VPT];
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
        for (int v = 0; v < NB * VPT; ++v) a[j][v] = {f2v(0.0f), f2v(0.0f)};
    // ahead (streaming lookahead, see k_upols_ahead): blocks 0..T-1 are not in the FDL yet,
    // so rows w .. w+T-1 (the prologue window and the first row entering it) count as zero
    // and block j collects partitions p > j only
    const bool future = ahead && p0 == 0;
    V f[T][VPT];
#pragma unroll
    for (int sl = 1; sl < T; ++sl) {  // rows block sl needs at p0
        int r = w + sl - p0;
        r = r < 0 ? r + ring : (r >= ring ? r - ring : r);
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            f[sl][v] = future ? V{} : __builtin_nontemporal_load(Fv + int64_t(r) * psv + tid + v * L);
    }
    V ph[D][VPT], pf[D][VPT];
#pragma unroll
    for (int d = 0; d < D; ++d) {  // prefetch partitions p0 .. p0 + D - 1
        const int p = p0 + d < ring ? p0 + d : ring - 1;  // past P: zero filter rows
        int r = w - p;
        r = r < 0 ? r + ring : r;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[d][v] = future && d == 0 ? V{} : __builtin_nontemporal_load(Fv + int64_t(r) * psv + tid + v * L);
            ph[d][v] = __builtin_nontemporal_load(Hv + int64_t(p) * psv + tid + v * L);
        }
    }
    // splits hold a multiple of T partitions; the last split's final chunk runs past P into
    // the ring's spare filter rows, which are zero (so those steps add nothing)
    for (int pb = p0; pb < p1; pb += T)
        batch_chunk<T, NB, VPT, L, D>(a, f, ph, pf, Hv, Fv, psv, tid, ring, w, pb, p1,
                                      std::make_integer_sequence<int, T>{});

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
                o[2 * b] = bin0 ? A.d.x : A.d.x - A.d.y;
                o[2 * b + 1] = bin0 ? A.d.y : A.x.x + A.x.y;
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

// Streaming lookahead: one block step of a T-block window (block j = 0..T-1 of the window
// that started at FDL row w0 = w - j; grid C, 256 lanes). At j = 0 a k_batch_mac pass with
// `ahead` already accumulated, for every block of the window, the partitions whose FDL rows
// existed then (p > j for block j) into the slabs part[c][s][j]. This step completes block j
// with the rest, p = 0..j, whose rows are the window's own blocks:
//   X = rfft(window) -> FDL row w;  Y = sum_s slab[s][j] + H0 X + sum_{p=1..j} H_p FDL[w - p]
//   out = irfft(Y) / 2B (OLS: last B samples; OLA: first B + overlap)
// The same products as a single-block step, in a different summation order; per block the
// HBM traffic is the slabs and j <= T-1 row pairs instead of all P partitions.
template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_upols_ahead(const float* __restrict__ in, int64_t ld_in,
                                                     float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
                                                     const cf* __restrict__ H, cf* __restrict__ fdl,
                                                     const cf* __restrict__ part, int S, int T, int j,
                                                     const cf* __restrict__ twg, int ring, int w, int64_t cstride,
                                                     int64_t pstride)
{
    using K = upols_cfg<B>;
    __shared__ __attribute__((aligned(16))) cf X[B];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    const float* in_c = in + int64_t(c) * ld_in;
    float* prev_c = prev + int64_t(c) * B;
    window_fft<B, OLA>(prev_c, in_c, fft, tw, tid);
    const int64_t crow = int64_t(c) * cstride;
    cf* row = fdl + crow + int64_t(w) * pstride;
    for (int k = tid; k < B; k += 256) {
        const cf x = r2c_split<B>(fft, tw + K::TW1, k);
        X[k] = x;
        row[k] = x;
    }
    if constexpr (!OLA) {  // the window's second half becomes the next call's first half
        for (int i = tid; i < B / 4; i += 256)
            reinterpret_cast<float4*>(prev_c)[i] = reinterpret_cast<const float4*>(in_c)[i];
    }
    __syncthreads();
    const int64_t ps4 = pstride / 2;
    const float4* H4 = reinterpret_cast<const float4*>(H + crow);
    const float4* F4 = reinterpret_cast<const float4*>(fdl + crow);
    const float4* S4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * T * B + int64_t(j) * B);
    const int64_t ss4 = int64_t(T) * K::Q;  // float4 between the slabs of one block
    for (int q = tid; q < K::Q; q += 256) {  // lane-private bins 2q, 2q + 1
        acc4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
        mac2(a0, a1, H4[q], reinterpret_cast<const float4*>(X)[q]);
        int p = 1;
        for (; p + 3 <= j; p += 4) {  // four row pairs in flight
            float4 hv[4], xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = w - p - u < 0 ? w - p - u + ring : w - p - u;
                hv[u] = H4[int64_t(p + u) * ps4 + q];
                xv[u] = F4[int64_t(r) * ps4 + q];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) mac2(a0, a1, hv[u], xv[u]);
        }
        for (; p <= j; ++p) {
            const int r = w - p < 0 ? w - p + ring : w - p;
            mac2(a0, a1, H4[int64_t(p) * ps4 + q], F4[int64_t(r) * ps4 + q]);
        }
        float4 sum = S4[q];
        for (int t = 1; t < S; ++t) {
            const float4 r = S4[t * ss4 + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        const cf b0 = finish(a0, q == 0), b1 = finish(a1, false);
        reinterpret_cast<float4*>(X)[q] = make_float4(sum.x + b0.x, sum.y + b0.y, sum.z + b1.x, sum.w + b1.y);
    }
    __syncthreads();
    c2r_tail<B, OLA>(X, fft, tw, out + int64_t(c) * ld_out, prev_c, tid);
}

// dispatch k_batch_mac over (B, NB, T) for the valid combinations
template<int BB, int NB>
int launch_batch_mac(const upols_t* h, int T, hipStream_t s, int ahead)
{
    constexpr int L = batch_cfg<BB, NB>::L;
    const unsigned grid = unsigned(h->C) * unsigned(h->Sb) * unsigned(batch_cfg<BB, NB>::G);
#define NEO_BATCH_T(TT)                                                                                          \
    case TT:                                                                                                     \
        if constexpr (batch_t(BB, NB, TT) == TT) {                                                               \
            hipLaunchKernelGGL((k_batch_mac<BB, TT, NB>), dim3(grid), dim3(L), 0, s, h->H, h->fdl, h->part_b, h->P, \
                               h->ring, h->Sb, h->rows_b, h->wpos, h->cstride, h->pstride, ahead);               \
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

// T consecutive blocks: window r2c + insert (C x T), one MAC pass (C x Sb), per-block
// finish (C x T), OLA overlap chain (C).
static int batch_buffers(upols_t* h)
{
    if (!h->part_b) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->part_b),
                                size_t(h->C) * h->Sb * kMaxBatch * h->B * sizeof(cf)));
        if (h->ola)
            NEO_HIP_CHECK(
                hipMalloc(reinterpret_cast<void**>(&h->tail), size_t(h->C) * kMaxBatch * h->B * sizeof(float)));
    }
    return NEO_HIP_OK;
}

// timing events (neo_hip_upols_set_timing) around every n-th MAC launch
static int mac_event(upols_t* h, bool timed, bool second, std::pair<hipEvent_t, hipEvent_t>& ev, hipStream_t s)
{
    if (!timed) return NEO_HIP_OK;
    if (!second) {
        if (h->events_used == h->events.size()) {
            NEO_HIP_CHECK(hipEventCreate(&ev.first));
            NEO_HIP_CHECK(hipEventCreate(&ev.second));
            h->events.push_back(ev);
        }
        ev = h->events[h->events_used];
        NEO_HIP_CHECK(hipEventRecord(ev.first, s));
    } else {
        NEO_HIP_CHECK(hipEventRecord(ev.second, s));
        ++h->events_used;
    }
    return NEO_HIP_OK;
}

// One streaming block step in lookahead mode: at the first block of each T-block window a
// k_batch_mac pass (ahead) over the filter and the FDL; then k_upols_ahead for the block.
int launch_ahead(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s)
{
    const int B = h->B, T = batch_blocks(h);
    int rc = batch_buffers(h);
    if (rc) return rc;
    if (h->phase == 0) {
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        const bool timed = h->timing && h->tick++ % h->timing == 0;
        if ((rc = mac_event(h, timed, false, ev, s))) return rc;
        if (h->bNB == 2) {
            NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s, 1)))
        } else {
            NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s, 1)))
        }
        if (rc) return rc;
        if ((rc = mac_event(h, timed, true, ev, s))) return rc;
    }
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_upols_ahead<BB, true>), dim3(unsigned(h->C)), dim3(256), 0, s, in,
                                                 ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T,
                                                 h->phase, h->tw, h->ring, h->wpos, h->cstride, h->pstride))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_upols_ahead<BB, false>), dim3(unsigned(h->C)), dim3(256), 0, s, in,
                                                 ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T,
                                                 h->phase, h->tw, h->ring, h->wpos, h->cstride, h->pstride))
    }
    NEO_HIP_LAUNCH_CHECK();
    h->wpos = h->wpos + 1 >= h->ring ? 0 : h->wpos + 1;
    h->phase = h->phase + 1 >= T ? 0 : h->phase + 1;
    return NEO_HIP_OK;
}

int launch_batch(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int T, hipStream_t s)
{
    const int B = h->B;
    int rc0 = batch_buffers(h);
    if (rc0) return rc0;
    const unsigned gCT = unsigned(h->C) * unsigned(T);
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, true>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    } else {
        NEO_UPOLS_DISPATCH(B, hipLaunchKernelGGL((k_batch_window<BB, false>), dim3(gCT), dim3(256), 0, s, in, ld_in,
                                                 h->prev, h->fdl, h->tw, T, h->ring, h->wpos, h->cstride, h->pstride))
    }
    NEO_HIP_LAUNCH_CHECK();
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    const bool timed = h->timing && h->tick++ % h->timing == 0;
    int rc = mac_event(h, timed, false, ev, s);
    if (rc) return rc;
    if (h->bNB == 2) {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s, 0)))
    } else {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s, 0)))
    }
    if (rc) return rc;
    if ((rc = mac_event(h, timed, true, ev, s))) return rc;
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


}  // namespace neo_hip
