// upols_batch.hip — batched passes for process_blocks / process_samples / dense_convolve:
// T consecutive blocks of every channel share ONE pass over the filter and the FDL
// (window r2c + insert, MAC with a sliding FDL window in registers, per-block finish,
// OLA overlap chain). Same results as T single-block steps up to summation order.
// Also the streaming lookahead built on the same pass (one block per call): the window
// pass at the first block of every T-block window (k_batch_mac, ahead), the sub-window
// passes, and the per-block steps k_upols_ahead / k_upols_ahead2 / k_upols_ahead3.
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
    int emax, rz;                  // FDL rows entering past partition emax read row rz (zero: an H spare row / out of range)
    // FDL row entering the sliding window at partition pn (write position w)
    __device__ __forceinline__ int frow(int w, int pn, int ring) const
    {
        const int r = w - pn;
        return pn > emax ? rz : (r < 0 ? r + ring : r);
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
// Variants (h->bvar, NEO_HIP_BATCH_VAR): accumulator form, prefetch depth D (divides T, so
// slots line up across chunks) and the waves per SIMD the register budget is sized for.
template<int V>
struct bmac_var;
template<>
struct bmac_var<0> {  // four partial products per bin (acc3), D = 4, 256 VGPRs
    static constexpr bool A2 = false, BUF = false;
    static constexpr int D = 4, W = 2;
};
template<>
struct bmac_var<1> {  // complex accumulators, D = 4, <= 168 VGPRs (3 waves/SIMD)
    static constexpr bool A2 = true, BUF = false;
    static constexpr int D = 4, W = 3;
};
template<>
struct bmac_var<2> {  // complex accumulators, D = 8, 256 VGPRs
    static constexpr bool A2 = true, BUF = false;
    static constexpr int D = 8, W = 2;
};
template<>
struct bmac_var<3> {  // as 2 with buffer loads (row offsets in SGPRs)
    static constexpr bool A2 = true, BUF = true;
    static constexpr int D = 8, W = 2;
};
#ifdef NEO_AHEAD_PROBE
// diagnostic build only (make probe): s_memrealtime stamps of channel 0's phases;
// k_batch_mac: s_memtime + s_memrealtime at entry and exit of workgroup 0 (clock)
__device__ unsigned long long g_probe[16];
__device__ unsigned long long g_wgspan[4096][2];  // k_batch_mac (T = 32): per-workgroup entry / exit, s_memrealtime
#define NEO_PROBE(i, cond)                                                                     \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        if (c == 0 && (cond)) g_probe[i] = __builtin_amdgcn_s_memrealtime();                   \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
#define NEO_CLOCK_STAMP(i)                                                                     \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                             \
            g_probe[i] = __builtin_amdgcn_s_memtime();                                         \
            g_probe[i + 1] = __builtin_amdgcn_s_memrealtime();                                 \
        }                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                             \
            g_wgspan[blockIdx.x][(i) == 10 ? 0 : 1] = __builtin_amdgcn_s_memrealtime();        \
        __builtin_amdgcn_sched_barrier(0);                                                     \
    } while (0)
#else
#define NEO_CLOCK_STAMP(i) (void)0
#define NEO_PROBE(i, cond) (void)0
#endif

template<int B, int T, int NB, int VAR, int D0 = bmac_var<VAR>::D, int D = (T < D0 ? T : D0)>
__global__ __launch_bounds__((batch_cfg<B, NB>::L), bmac_var<VAR>::W) void k_batch_mac(const cf* __restrict__ H,
                                                                   const cf* __restrict__ fdl, cf* __restrict__ part,
                                                                   int P, int ring, int S, int rows, int w,
                                                                   int64_t cstride, int64_t pstride, int ahead,
                                                                   int emax, int rz, int pc, int prio)
{
    if constexpr (T == 32) NEO_CLOCK_STAMP(10);
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
                              int(pstride * int64_t(sizeof(cf))), emax, rz};
    // filter rows p < pc with the default (cacheable) policy: the same rows every pass, kept
    // in the Infinity Cache; the nontemporal stream of the rest does not evict them
    const row_src<V, BUF, false> src_c{src.Hv, src.Fv, src.psv, src.Hr, src.Fr, src.prow, emax, rz};

    acc3 a[T][NB * VPT];
#pragma unroll
    for (int j = 0; j < T; ++j)
#pragma unroll
        for (int v = 0; v < NB * VPT; ++v) a[j][v] = {f2v(0.0f), f2v(0.0f)};
    // ahead (streaming lookahead, see k_upols_ahead): blocks 0..T-1 are not in the FDL yet,
    // so rows w .. w+T-1 (the prologue window and the first row entering it) count as zero
    // and block j collects partitions p > j only
    const bool future = (ahead & 1) && p0 == 0;
    const bool nts = (ahead & 2) != 0;  // slabs stored nontemporally (they are read once, next steps)
    V f[T][VPT];
#pragma unroll
    for (int sl = 1; sl < T; ++sl) {  // rows block sl needs at p0 (entered at partition p0 - sl)
        int r = w + sl - p0;
        r = r < 0 ? r + ring : (r >= ring ? r - ring : r);
        r = p0 - sl > emax ? rz : r;
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            f[sl][v] = future ? V{} : src.f(r, tid + v * L);
    }
    V ph[D][VPT], pf[D][VPT];
#pragma unroll
    for (int d = 0; d < D; ++d) {  // prefetch partitions p0 .. p0 + D - 1
        const int p = p0 + d < ring ? p0 + d : ring - 1;  // past P: zero filter rows
        const int r = src.frow(w, p, ring);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[d][v] = future && d == 0 ? V{} : src.f(r, tid + v * L);
            ph[d][v] = BUF && p < pc ? src_c.h(p, tid + v * L) : src.h(p, tid + v * L);
        }
    }
    // splits hold a multiple of T partitions; the last split's final chunk runs past P into
    // the ring's spare filter rows, which are zero (so those steps add nothing). Chunks
    // starting below pc load filter rows cacheable, the rest nontemporally.
    // prio: two workgroups share a CU (blockIdx i and i + grid/2, the dispatch order) and the
    // SQ favours the older one's waves, which finish ~30 % early and leave one wave per SIMD
    // for the rest of the pass; with prio they trade issue priority in slices of 2^prio
    // s_memrealtime ticks (100 MHz; 11 = 20 us). (Locking the two together with a barrier per chunk instead —
    // one 8-wave workgroup per CU — was 30 % slower: both stall on memory at the same time.)
    const int half = blockIdx.x >= gridDim.x / 2;
    // prio = shift + 32 * m: m = 0 alternates slices 1:1; m = 1 gives the younger workgroup
    // 2 slices of 3, m = 2 3 slices of 5
    auto share = [&]() {
        if (prio) {
            const unsigned sh = prio & 31, m = unsigned(prio) >> 5;
            const unsigned long long t = __builtin_amdgcn_s_memrealtime() >> sh;
            const unsigned period = m == 0 ? 2 : (m == 1 ? 3 : 5), older = m == 2 ? 2 : 1;
            const bool mine_old = t % period < older;  // slices held by the older workgroup
            const bool hi = half ? !mine_old : mine_old;
            if (hi) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(0);
        }
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
    if (prio) __builtin_amdgcn_s_setprio(0);

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
            if (nts) __builtin_nontemporal_store(o, reinterpret_cast<V*>(slab + int64_t(j) * B + (tid + v * L) * NB));
            else *reinterpret_cast<V*>(slab + int64_t(j) * B + (tid + v * L) * NB) = o;
        }
    if constexpr (T == 32) NEO_CLOCK_STAMP(12);
}

// k_batch_mac with the row stream through an LDS-DMA ring (B = 256 / 512, T = 32, one
// complex bin per lane): each wave owns 64 bins and a private ring of D slots of 1 KB;
// one buffer_load_dwordx4 ... lds per partition fills a slot (lanes 0-31: the H row's 64
// bins, lanes 32-63: the FDL row's), issued D partitions ahead, so D KB per wave are in
// flight without holding registers. H and the FDL share one allocation, so one buffer
// descriptor per channel covers both; a lane's byte offset is its bin plus its row times
// the row pitch. The wave reads back only its own slots (counted vmcnt, no barrier); the
// accumulators and the sliding window of T FDL values stay in registers (complex
// accumulators, bmac_var<2>'s arithmetic). Prefetches past the last consumed partition
// may read junk rows or out of range (buffer loads return 0 there); they are never used.
template<int D, int W>
struct lds_var {
    static constexpr int depth = D, waves = W;
};
template<int V>
using lds_var_t = std::conditional_t<V == 4, lds_var<8, 3>, lds_var<16, 2>>;  // (8, 4 waves): 1200 spilled VGPRs

template<int N>
__device__ __forceinline__ void wait_vm()  // s_waitcnt vmcnt(N), other counters untouched
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// H and FDL values of this lane's bin from ring slot OFF (bytes; the FDL half 512 B
// further). Inline asm: the compiler would otherwise wait for every LDS-DMA in flight
// before an LDS read it cannot tell apart from their destinations.
template<int OFF>
__device__ __forceinline__ void ring_read(unsigned lane_addr, f2v& h, f2v& x)
{
    asm volatile("ds_read_b64 %0, %2 offset:%3\n\tds_read_b64 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(h), "=v"(x)
                 : "v"(lane_addr), "i"(OFF), "i"(OFF + 512)
                 : "memory");
}

struct lds_src {
    __amdgpu_buffer_rsrc_t rs;  // channel's H rows ... FDL rows
    int voff;                   // next DMA's byte offset: H lanes row p, FDL lanes row (w - p) mod R
    int delta;                  // per partition: +row (H lanes), -row (FDL lanes)
    int wrap;                   // FDL lanes: + R rows when w - p drops below 0 (H lanes: 0)
    unsigned wring;             // wave's ring (LDS byte address, wave-uniform)
    unsigned lane_addr;         // wring + 8 * lane
};

// DMA partition p into ring slot `slot`; q.voff holds p's offsets and then moves to p + 1
// (one add per partition; the FDL lanes wrap once, when p passes w)
__device__ __forceinline__ void lds_fill(lds_src& q, int slot, int p, int w)
{
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q.rs, (__attribute__((address_space(3))) void*)(uintptr_t)(q.wring + slot * 1024),
                                             16, q.voff, 0, 0, 2 /* nt */);
    q.voff += q.delta + (p == w ? q.wrap : 0);
}

template<int T, int D, int U>
__device__ __forceinline__ void lds_step(acc3 (&a)[T], f2v (&f)[T], lds_src& q, int w, int p, bool zero, bool bin0)
{
    constexpr int slot = U % D;
    wait_vm<D - 1>();  // the DMA of partition p (D - 1 newer ones stay in flight)
    f2v hv, xv;
    ring_read<slot * 1024>(q.lane_addr, hv, xv);
    if (zero) xv = f2v(0.0f);
    f[(T - U) % T] = xv;
    lds_fill(q, slot, p + D, w);  // refill the slot with partition p + D
    const float s = bin0 ? 0.0f : hv.y;
    const f2v h1 = {hv.x, bin0 ? hv.y : hv.x}, h2 = {-s, s};
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const f2v x = f[(j - U + T) % T];
            a[j].d = k == 0 ? __builtin_elementwise_fma(h1, x, a[j].d) : __builtin_elementwise_fma(h2, x.yx, a[j].d);
        }
    __builtin_amdgcn_sched_barrier(0);
}

template<int T, int D, int... U>
__device__ __forceinline__ void lds_chunk(acc3 (&a)[T], f2v (&f)[T], lds_src& q, int w, int pb, bool zero0, bool bin0,
                                          std::integer_sequence<int, U...>)
{
    (lds_step<T, D, U>(a, f, q, w, pb + U, U == 0 && zero0, bin0), ...);
}

template<int B, int T, int VAR>
__global__ __launch_bounds__(256, lds_var_t<VAR>::waves) void k_batch_mac_lds(
    const cf* __restrict__ H, const cf* __restrict__ fdl, cf* __restrict__ part, int P, int ring, int S, int rows, int w,
    int64_t cstride, int64_t pstride, int ahead)
{
    constexpr int D = lds_var_t<VAR>::depth, G = B / 256;
    static_assert(B == 256 || B == 512, "one bin per lane, 64 bins per wave");
    __shared__ __attribute__((aligned(1024))) char lring[4 * D * 1024];
    const int cs = blockIdx.x / G, gch = blockIdx.x - cs * G;
    const int tid = gch * 256 + threadIdx.x;  // bin
    const int c = cs / S, s = cs - c * S;
    const int p0 = s * rows, p1 = min(P, p0 + rows);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
    const cf* Hc = H + int64_t(c) * cstride;
    const cf* Fc = fdl + int64_t(c) * cstride;
    const int foff = int((fdl - H) * int64_t(sizeof(cf)));  // FDL of a channel, bytes past its H (host-checked < 2 GiB)
    const int rowbytes = int(pstride * int64_t(sizeof(cf)));
    const bool hl = lane < 32;  // lanes 0-31 fetch the H half of a slot, 32-63 the FDL half
    lds_src q;
    q.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<cf*>(Hc), 0, foff + ring * rowbytes, 0x00020000);
    {
        int r0 = w - p0;
        r0 = r0 < 0 ? r0 + ring : r0;
        q.voff = (hl ? p0 * rowbytes : foff + r0 * rowbytes) + (gch * 256 + wv * 64 + 2 * (lane & 31)) * int(sizeof(cf));
    }
    q.delta = hl ? rowbytes : -rowbytes;
    q.wrap = hl ? 0 : ring * rowbytes;
    q.wring = unsigned(reinterpret_cast<uintptr_t>(lring)) + unsigned(wv * D * 1024);
    q.lane_addr = q.wring + 8u * unsigned(lane);
    const bool bin0 = tid == 0;

    acc3 a[T];
#pragma unroll
    for (int j = 0; j < T; ++j) a[j] = {f2v(0.0f), f2v(0.0f)};
    const bool future = ahead && p0 == 0;  // see k_batch_mac
    f2v f[T];
#pragma unroll
    for (int sl = 1; sl < T; ++sl) {
        int r = w + sl - p0;
        r = r < 0 ? r + ring : (r >= ring ? r - ring : r);
        f[sl] = future ? f2v(0.0f) : __builtin_nontemporal_load(reinterpret_cast<const f2v*>(Fc + int64_t(r) * pstride + tid));
    }
    wait_vm<0>();
#pragma unroll
    for (int d = 0; d < D; ++d) lds_fill(q, d, p0 + d, w);  // partitions p0 .. p0 + D - 1
    for (int pb = p0; pb < p1; pb += T)
        lds_chunk<T, D>(a, f, q, w, pb, future && pb == p0, bin0, std::make_integer_sequence<int, T>{});
    wait_vm<0>();  // no DMA outstanding at exit

    cf* slab = part + (int64_t(c) * S + s) * T * B;
#pragma unroll
    for (int j = 0; j < T; ++j) *reinterpret_cast<f2v*>(slab + int64_t(j) * B + tid) = a[j].d;
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
    const float* in_c = in + int64_t(c) * ld_in;
    float* prev_c = prev + int64_t(c) * B;
    window_fft<B, OLA>(prev_c, in_c, fft, tw, tid, twg);
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

// k_upols_ahead with the work spread over one workgroup of 64 + NG*Q lanes per channel.
// Sub-windows (ssub > 0): at the first block of each sw-block sub-window after the
// first, a small k_batch_mac pass (T = sw, FDL rows limited to the
// window's own) accumulates for the sub-window's blocks the partitions whose rows are the
// window's blocks before it; a block step then adds that slab and runs only the
// partitions 1..jr (jr = its position in the sub-window) itself. Per 32-block window the
// rows a block step reads drop from 496 to 112 row pairs per channel.
// (Q = B/2 float4 per row): wave 0 runs the window r2c alone (wave-synchronous, no
// workgroup barriers) while NG groups of Q lanes sum the slabs and MAC the partitions
// p = 1..j (group g takes p = 1 + g, 1 + g + NG, ...; up to KC row pairs in flight per
// lane); after one barrier group 0 adds H0 X and the groups' partials, and after a second
// wave 0 runs the c2r. The serial chain per block is one window transform, one burst of
// row loads (overlapped with it) and one inverse transform; the per-channel MAC no longer
// walks j partitions four at a time.

// lookahead sub-window length sw (blocks) is per handle: h->subw, 8 or 16

template<int B>
struct ahead_cfg {
    static constexpr int Q = B / 2;                                  // float4 (2 bins) per row
#ifdef NEO_AHEAD_NG
    static constexpr int NG0 = Q >= 768 ? 1 : (768 / Q > 6 ? 6 : 768 / Q);
    static constexpr int NG = NEO_AHEAD_NG < NG0 ? NEO_AHEAD_NG : NG0;  // (A/B builds)
#else
    static constexpr int NG = Q >= 768 ? 1 : (768 / Q > 6 ? 6 : 768 / Q);  // MAC groups
#endif
    static constexpr int EW = B >= 512 ? B / 64 : 8;                 // transform elements per lane
    static constexpr int TW = B / EW;                                // transform lanes (<= 64)
    static constexpr int NT = 64 + NG * Q;                           // workgroup size
    static constexpr int KC = 8;                                     // row pairs in flight per lane
};

template<int B, bool OLA>
__global__ __launch_bounds__(ahead_cfg<B>::NT) void k_upols_ahead2(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, const cf* __restrict__ part, int S, int T, int j,
    const cf* __restrict__ twg, int ring, int w, int64_t cstride, int64_t pstride, const cf* __restrict__ sub, int ssub,
    int jr, int sw, const cf* __restrict__ far, int fj)
{
    using K = upols_cfg<B>;
    using A = ahead_cfg<B>;
    constexpr int Q = A::Q, NG = A::NG, EW = A::EW, TW = A::TW, KC = A::KC;
    static_assert(TW <= 64 && A::NT <= 1024 && EW % 2 == 0, "ahead2 geometry");
    __shared__ __attribute__((aligned(16))) cf X[B];
    __shared__ __attribute__((aligned(16))) float4 acc[NG][Q];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x;
    const int64_t crow = int64_t(c) * cstride;
    const float* in_c = in + int64_t(c) * ld_in;
    float* prev_c = prev + int64_t(c) * B;
    const int64_t ps4 = pstride / 2;
    const float4* H4 = reinterpret_cast<const float4*>(H + crow);
    // group 0 lane i owns the mirror pair of bins (k0, k1) = (i, B - i), (0, B/2) for i = 0:
    // the r2c split, H0 X and the c2r join all pair bin k with bin B - k
    const int i0 = tid - 64, k0 = i0, k1 = i0 == 0 ? B / 2 : B - i0;
    cf h0a = {0.f, 0.f}, h0b = h0a;
    if (tid >= 64 && tid < 64 + Q) {
        h0a = H[crow + k0];
        h0b = H[crow + k1];
    }
    NEO_PROBE(0, tid == 0);
    NEO_PROBE(8, tid == 64);
    if (tid < 64) {  // wave 0: window r2c, FDL row w, previous block
        tw_regs<K::TW1 + K::TW2, 64> twr;
        twr.load(twg, tid);
        cf v[EW];
        if (tid < TW) {
            const cf* pz = reinterpret_cast<const cf*>(prev_c);
            const cf* iz = reinterpret_cast<const cf*>(in_c);
#pragma unroll
            for (int m = 0; m < EW; ++m) {
                const int n = tid + m * TW;
                if constexpr (OLA) v[m] = n < B / 2 ? iz[n] : cf{0.f, 0.f};
                else v[m] = n < B / 2 ? pz[n] : iz[n - B / 2];
            }
            if constexpr (!OLA) {
                // the window's second half (this block, v[EW/2..EW-1]) becomes the next call's
                // first half, stored from registers (a re-load cost a ~1 us round trip). Lanes
                // read prev_c[n] in load m - EW/2 of the same wave, which has completed (loads
                // return in order) by the time the store of load m's value issues.
                cf* pw = reinterpret_cast<cf*>(prev_c);
#pragma unroll
                for (int m = EW / 2; m < EW; ++m) pw[tid + m * TW - B / 2] = v[m];
            }
        }
        twr.store(tw, tid);
        wave_sync();
        NEO_PROBE(1, tid == 0);
        stockham<B, EW, -1, 1, true>(v, fft, tw, tid, tid < TW);
        NEO_PROBE(2, tid == 0);
        if (tid < TW) {
#pragma unroll
            for (int m = 0; m < EW; ++m) fft[lpad(tid + m * TW)] = v[m];
        }
    } else {  // MAC groups: slabs + partitions 1..j
        const int u = tid - 64, g = u / Q, q = u - g * Q;
        const float4* F4 = reinterpret_cast<const float4*>(fdl + crow);
        const float4* S4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * T * B + int64_t(j) * B);
        const int64_t ss4 = int64_t(T) * K::Q;  // float4 between the slabs of one block
        float4 sum = {0.f, 0.f, 0.f, 0.f};
        for (int s = g; s < S; s += NG) {
            const float4 r = S4[s * ss4 + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        for (int s = NG - 1 - g; s < ssub; s += NG) {  // sub-window pass slabs (the window's earlier rows)
            const float4 r = reinterpret_cast<const float4*>(sub + ((int64_t(c) * ssub + s) * sw + jr) * B)[q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        if (far && g == NG - 1) {  // two-level lookahead: the far partitions (upols_far.hip)
            const float4 r = reinterpret_cast<const float4*>(far + (int64_t(c) * kFarT + fj) * B)[q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        acc4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
        for (int pb = 1 + g; pb <= jr; pb += NG * KC) {
            float4 hv[KC], xv[KC];
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const int p = pb + k * NG;
                if (p <= jr) {
                    const int r = w - p < 0 ? w - p + ring : w - p;
                    hv[k] = H4[int64_t(p) * ps4 + q];
                    xv[k] = F4[int64_t(r) * ps4 + q];
                }
            }
#pragma unroll
            for (int k = 0; k < KC; ++k)
                if (pb + k * NG <= jr) mac2(a0, a1, hv[k], xv[k]);
        }
        const cf b0 = finish(a0, q == 0), b1 = finish(a1, false);
        acc[g][q] = make_float4(sum.x + b0.x, sum.y + b0.y, sum.z + b1.x, sum.w + b1.y);
        NEO_PROBE(9, tid == 64);
    }
    NEO_PROBE(3, tid == 0);
    __syncthreads();
    NEO_PROBE(4, tid == 0);
    if (tid >= 64 && tid < 64 + Q) {
        // group 0, bin pair (k0, k1): r2c split of the window transform, FDL row w, Y = the
        // groups' partial sums + H0 X, then the c2r join -- 2 bins per lane over Q lanes
        // instead of B/64 per lane in wave 0, between the two barriers
        // one twiddle lookup serves all four: w(B - k) = -conj(w(k)) (w(B/2) = -i for the k0 = 0
        // lane), the inverse twiddles are the conjugates
        const cf wa = k0 == 0 ? cf{1.f, 0.f} : twiddle<2 * B, -1>(tw + K::TW1, k0);
        const cf wb = k0 == 0 ? cf{0.f, -1.f} : cf{-wa.x, wa.y};
        const cf xa = r2c_split_w<B>(fft, wa, k0), xb = r2c_split_w<B>(fft, wb, k1);
        cf* row = fdl + crow + int64_t(w) * pstride;
        row[k0] = xa;
        row[k1] = xb;
        const cf* accb = reinterpret_cast<const cf*>(&acc[0][0]);  // acc[g] as B bins
        cf ya = accb[k0], yb = accb[k1];
#pragma unroll
        for (int g = 1; g < NG; ++g) {
            const cf ra = accb[g * B + k0], rb = accb[g * B + k1];
            ya.x += ra.x; ya.y += ra.y; yb.x += rb.x; yb.y += rb.y;
        }
        if (k0 == 0) {  // packed {DC, Nyquist}: two real products
            ya.x += h0a.x * xa.x;
            ya.y += h0a.y * xa.y;
        } else {
            ya.x += h0a.x * xa.x - h0a.y * xa.y;
            ya.y += h0a.x * xa.y + h0a.y * xa.x;
        }
        yb.x += h0b.x * xb.x - h0b.y * xb.y;
        yb.y += h0b.x * xb.y + h0b.y * xb.x;
        X[k0] = k0 == 0 ? c2r_join_w<B>(cf{ya.x, 0.f}, cf{ya.y, 0.f}, cf{1.f, 0.f}, 0)
                        : c2r_join_w<B>(ya, yb, cf{wa.x, -wa.y}, k0);
        X[k1] = c2r_join_w<B>(yb, k0 == 0 ? yb : ya, cf{wb.x, -wb.y}, k1);
    }
    __syncthreads();
    NEO_PROBE(5, tid == 0);
    if (tid < 64) c2r_tail<B, OLA, EW, true, true>(X, fft, tw, out + int64_t(c) * ld_out, prev_c, tid);
    NEO_PROBE(6, tid == 0);
}

// ---------------------------------------------------------------------------------------
// Direct-head lookahead block step (OLS, B = 256 / 512): the output no longer waits for the
// window transform. Partition 0's contribution H0 X is the linear convolution of the window
// with the time-domain head h0 (irfft(H0) / 2B; the first B taps, its second half zero for
// a zero-padded partition), y0[n] = sum_k h0[k] x[n - k] for the output samples n in
// [B, 2B) -- the same products the overlap-save irfft of H0 X evaluates, summed directly.
// The rest of block j's spectrum (window-pass slabs, sub-window slab, partitions 1..jr) does
// not depend on this block's input at all. So, one workgroup per channel, by wave role:
//   wave 0        window load -> LDS (for the convolution), previous block from registers,
//                 r2c, FDL row w insert (for later blocks; off the output path)
//   MAC waves     slabs + partitions 1..jr -> rest spectrum R in LDS
//   c2r wave      waits for R, irfft(R) / 2B -> z in LDS
//   conv waves    taps into LDS, wait for the window, B/4 taps each over all B outputs
//                 (8 outputs per lane, two packed accumulator sets: even taps on output
//                 pairs (2i, 2i+1), odd taps on (2i+1, 2i+2), one float4 of the window per
//                 four taps), partial sums in LDS; then out = sum of the four partials + z
// Roles hand over through LDS counters (release / acquire at workgroup scope); all waves of
// a workgroup are resident together, so the waits always end.
template<int B>
struct ahead3_cfg {
    static constexpr int Q = B / 2;                    // float4 (2 bins) per row
    static constexpr int MW = Q / 64;                  // MAC waves
    static constexpr int CW = B >= 512 ? 8 : 4;        // convolution waves (taps split CW ways)
    static constexpr int R = 8;                        // outputs per convolution lane
    static constexpr int CL = B / R;                   // convolution lanes (<= 64)
    static constexpr int KW = B / CW;                  // taps per convolution wave
    static constexpr int EW = B >= 512 ? B / 64 : 8;   // transform elements per lane
    static constexpr int TW = B / EW;                  // transform lanes (<= 64)
    static constexpr int NT = 64 * (1 + MW + 1 + CW);  // workgroup size
    static constexpr int XPAD = 8;                     // zero floats before the window (prefetch underrun)
};

__device__ __forceinline__ void lds_signal(int* cnt)  // all lanes of a wave, after its LDS writes
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void lds_wait(int* cnt, int n)
{
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < n) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template<int B>
__global__ __launch_bounds__(ahead3_cfg<B>::NT) void k_upols_ahead3(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, const cf* __restrict__ part, int S, int T, int j,
    const cf* __restrict__ twg, int ring, int w, int64_t cstride, int64_t pstride, const cf* __restrict__ sub, int ssub,
    int jr, int sw, const float* __restrict__ h0t, const cf* __restrict__ far, int fj)
{
    using K = upols_cfg<B>;
    using A = ahead3_cfg<B>;
    constexpr int MW = A::MW, CW = A::CW, EW = A::EW, TW = A::TW, KW = A::KW, XP = A::XPAD;
    static_assert(TW <= 64 && A::CL <= 64 && A::NT <= 1024 && EW % 2 == 0 && KW % 4 == 0, "ahead3 geometry");
    __shared__ cf tw_f[K::TW1 + K::TW2];
    __shared__ cf fft_f[K::LL];
    __shared__ cf tw_c[K::TW1 + K::TW2];
    __shared__ cf fft_c[K::LL];
    __shared__ __attribute__((aligned(16))) cf Rs[B];                 // rest spectrum (packed)
    __shared__ __attribute__((aligned(16))) float xw[XP + 2 * B + 8];  // window, XP zeros in front
    __shared__ __attribute__((aligned(16))) float hh[B];               // head taps
    __shared__ __attribute__((aligned(16))) float Pc[CW][B];           // convolution partials
    __shared__ __attribute__((aligned(16))) float zs[B];               // irfft(R) / 2B, samples [B, 2B)
    __shared__ int cnt[5];                                             // window, R, partials, z, joined R
    const int tid = threadIdx.x, c = blockIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t crow = int64_t(c) * cstride;
    const float* in_c = in + int64_t(c) * ld_in;
    float* prev_c = prev + int64_t(c) * B;
    NEO_PROBE(0, tid == 0);
    if (tid < 5) cnt[tid] = 0;
    if (tid < XP) xw[tid] = 0.f;
    if (tid < 8) xw[XP + 2 * B + tid] = 0.f;
    __syncthreads();
    if (wave == 0) {  // window -> LDS + registers, previous block, r2c, FDL row w
        tw_regs<K::TW1 + K::TW2, 64> twr;
        twr.load(twg, lane);
        cf v[EW];
        if (lane < TW) {
            const cf* pz = reinterpret_cast<const cf*>(prev_c);
            const cf* iz = reinterpret_cast<const cf*>(in_c);
#pragma unroll
            for (int m = 0; m < EW; ++m) {
                const int n = lane + m * TW;
                v[m] = n < B / 2 ? pz[n] : iz[n - B / 2];
            }
            cf* xc = reinterpret_cast<cf*>(xw + XP);
#pragma unroll
            for (int m = 0; m < EW; ++m) xc[lane + m * TW] = v[m];
            cf* pw = reinterpret_cast<cf*>(prev_c);  // this block becomes the next call's first half
#pragma unroll
            for (int m = EW / 2; m < EW; ++m) pw[lane + m * TW - B / 2] = v[m];
        }
        twr.store(tw_f, lane);
        lds_signal(&cnt[0]);
        NEO_PROBE(1, tid == 0);
        wave_sync();
        stockham<B, EW, -1, 1, true>(v, fft_f, tw_f, lane, lane < TW);
        NEO_PROBE(2, tid == 0);
        if (lane < TW) {
#pragma unroll
            for (int m = 0; m < EW; ++m) fft_f[lpad(lane + m * TW)] = v[m];
        }
        wave_sync();
        cf* row = fdl + crow + int64_t(w) * pstride;
        constexpr int NK = B / 64;
        cf xs[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) xs[i] = r2c_split<B>(fft_f, tw_f + K::TW1, lane + 64 * i);
#pragma unroll
        for (int i = 0; i < NK; ++i) row[lane + 64 * i] = xs[i];
        NEO_PROBE(3, tid == 0);
    } else if (wave <= MW) {  // rest spectrum: slabs + sub-window slabs + partitions 1..jr
        const int q = tid - 64;
        const int64_t ps4 = pstride / 2;
        const float4* H4 = reinterpret_cast<const float4*>(H + crow);
        const float4* F4 = reinterpret_cast<const float4*>(fdl + crow);
        const float4* S4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * T * B + int64_t(j) * B);
        const int64_t ss4 = int64_t(T) * K::Q;
        float4 sum = {0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < S; ++t) {
            const float4 r = S4[t * ss4 + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        for (int t = 0; t < ssub; ++t) {
            const float4 r = reinterpret_cast<const float4*>(sub + ((int64_t(c) * ssub + t) * sw + jr) * B)[q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        if (far) {  // two-level lookahead: the far partitions (upols_far.hip)
            const float4 r = reinterpret_cast<const float4*>(far + (int64_t(c) * kFarT + fj) * B)[q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        acc4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
        for (int pb = 1; pb <= jr; pb += 8) {  // up to 8 row pairs in flight
            float4 hv[8], xv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (pb + k <= jr) {
                    const int p = pb + k, r = w - p < 0 ? w - p + ring : w - p;
                    hv[k] = H4[int64_t(p) * ps4 + q];
                    xv[k] = F4[int64_t(r) * ps4 + q];
                }
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (pb + k <= jr) mac2(a0, a1, hv[k], xv[k]);
        }
        const cf b0 = finish(a0, q == 0), b1 = finish(a1, false);
        reinterpret_cast<float4*>(Rs)[q] = make_float4(sum.x + b0.x, sum.y + b0.y, sum.z + b1.x, sum.w + b1.y);
        lds_signal(&cnt[1]);
        // c2r join on mirror pairs (k, B - k), in place: lane q owns (q, B - q), (0, B/2) for q = 0
        lds_wait(&cnt[1], MW);
        lds_wait(&cnt[0], 1);  // wave 0's twiddle table
        {
            const int k0 = q, k1 = q == 0 ? B / 2 : B - q;
            const cf wa = k0 == 0 ? cf{1.f, 0.f} : twiddle<2 * B, -1>(tw_f + K::TW1, k0);
            const cf wb = k0 == 0 ? cf{0.f, -1.f} : cf{-wa.x, wa.y};
            const cf ya = Rs[k0], yb = Rs[k1];
            Rs[k0] = k0 == 0 ? c2r_join_w<B>(cf{ya.x, 0.f}, cf{ya.y, 0.f}, cf{1.f, 0.f}, 0)
                             : c2r_join_w<B>(ya, yb, cf{wa.x, -wa.y}, k0);
            Rs[k1] = c2r_join_w<B>(yb, k0 == 0 ? yb : ya, cf{wb.x, -wb.y}, k1);
        }
        lds_signal(&cnt[4]);
        NEO_PROBE(4, tid == 64);
    } else if (wave == MW + 1) {  // irfft(R) / 2B -> zs
        for (int i = lane; i < K::TW1 + K::TW2; i += 64) tw_c[i] = twg[i];
        lds_wait(&cnt[4], MW);  // the joined rest spectrum
        NEO_PROBE(5, lane == 0);
        cf v[EW];
        if (lane < TW) {
#pragma unroll
            for (int m = 0; m < EW; ++m) v[m] = Rs[lane + m * TW];
        }
        stockham<B, EW, +1, 1, true>(v, fft_c, tw_c, lane, lane < TW);
        if (lane < TW) {
            const float scale = 1.0f / float(2 * B);  // overlap_save.hpp:107-108
            cf* zc = reinterpret_cast<cf*>(zs);
#pragma unroll
            for (int m = EW / 2; m < EW; ++m) zc[lane + m * TW - B / 2] = {v[m].x * scale, v[m].y * scale};
        }
        lds_signal(&cnt[3]);
        NEO_PROBE(6, lane == 0);
    } else {  // convolution with the head taps
        const int cw = wave - MW - 2;
        const int ka = cw * KW;
        for (int i = lane * 4; i < KW; i += 256)
            *reinterpret_cast<float4*>(hh + ka + i) = *reinterpret_cast<const float4*>(h0t + int64_t(c) * B + ka + i);
        lds_wait(&cnt[0], 1);  // the window (wave 0); the taps are this wave's own writes
        NEO_PROBE(7, lane == 0 && cw == 0);
        f2v ya[4] = {}, yb[4] = {};  // even taps on output pairs (2i, 2i+1); odd taps on (2i+1, 2i+2)
        float y0o = 0.f;              // odd taps of output 0
        const int n0 = B + A::R * lane;
        if (lane < A::CL) {
            const float* x = xw + XP;
            int b = n0 - ka;  // window floats [b - 4, b + 8) cover four taps from ka
            float4 Fm = *reinterpret_cast<const float4*>(x + b - 4);
            float4 F0 = *reinterpret_cast<const float4*>(x + b);
            float4 F1 = *reinterpret_cast<const float4*>(x + b + 4);
#pragma unroll 4
            for (int kc = ka; kc < ka + KW; kc += 4) {
                const float4 hq = *reinterpret_cast<const float4*>(hh + kc);
                const float4 Fn = *reinterpret_cast<const float4*>(x + b - 8);  // next chunk (zeros before the window)
                const f2v s0[4] = {{F0.x, F0.y}, {F0.z, F0.w}, {F1.x, F1.y}, {F1.z, F1.w}};  // x[b .. b+7]
                const f2v s1[4] = {{Fm.z, Fm.w}, {F0.x, F0.y}, {F0.z, F0.w}, {F1.x, F1.y}};  // x[b-2 .. b+5]
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    ya[i] = __builtin_elementwise_fma(f2v{hq.x, hq.x}, s0[i], ya[i]);  // tap kc
                    yb[i] = __builtin_elementwise_fma(f2v{hq.y, hq.y}, s0[i], yb[i]);  // tap kc + 1
                    ya[i] = __builtin_elementwise_fma(f2v{hq.z, hq.z}, s1[i], ya[i]);  // tap kc + 2
                    yb[i] = __builtin_elementwise_fma(f2v{hq.w, hq.w}, s1[i], yb[i]);  // tap kc + 3
                }
                y0o = __builtin_fmaf(hq.y, Fm.w, y0o);  // x[n0 - kc - 1]
                y0o = __builtin_fmaf(hq.w, Fm.y, y0o);  // x[n0 - kc - 3]
                F1 = F0;
                F0 = Fm;
                Fm = Fn;
                b -= 4;
            }
            // y[2i] = ya[i].x + yb[i-1].y (i > 0) or + y0o; y[2i+1] = ya[i].y + yb[i].x
            float* pc = Pc[cw] + (n0 - B);
            const float4 o0 = {ya[0].x + y0o, ya[0].y + yb[0].x, ya[1].x + yb[0].y, ya[1].y + yb[1].x};
            const float4 o1 = {ya[2].x + yb[1].y, ya[2].y + yb[2].x, ya[3].x + yb[2].y, ya[3].y + yb[3].x};
            reinterpret_cast<float4*>(pc)[0] = o0;
            reinterpret_cast<float4*>(pc)[1] = o1;
        }
        lds_signal(&cnt[2]);
        NEO_PROBE(8, lane == 0 && cw == 0);
        lds_wait(&cnt[2], CW);
        lds_wait(&cnt[3], 1);
        NEO_PROBE(9, lane == 0 && cw == 0);
        float* out_c = out + int64_t(c) * ld_out;
        for (int m = cw * (B / CW) + lane * 4; m < (cw + 1) * (B / CW); m += 256) {
            float4 r = *reinterpret_cast<const float4*>(zs + m);
#pragma unroll
            for (int t = 0; t < CW; ++t) {
                const float4 u = *reinterpret_cast<const float4*>(Pc[t] + m);
                r.x += u.x; r.y += u.y; r.z += u.z; r.w += u.w;
            }
            *reinterpret_cast<float4*>(out_c + m) = r;
        }
        NEO_PROBE(10, lane == 0 && cw == 0);
    }
}

// Time-domain head taps for k_upols_ahead3 (grid C, 256 lanes): irfft(H0) / 2B of each
// channel's packed partition 0; taps [0, B) -> h0t, the second half's magnitude relative to
// the first (zero-padded partitions: rounding only) -> tail[c].
template<int B>
__global__ __launch_bounds__(256) void k_head_taps(const cf* __restrict__ H, int64_t cstride, const cf* __restrict__ twg,
                                                   float* __restrict__ h0t, float* __restrict__ tail)
{
    using K = upols_cfg<B>;
    constexpr int E = K::E, T = B / E;
    __shared__ cf X[B];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    __shared__ float red[2][256];
    const int tid = threadIdx.x, c = blockIdx.x;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    for (int k = tid; k < B; k += 256) X[k] = H[int64_t(c) * cstride + k];
    __syncthreads();
    cf v[E];
    const bool active = tid < T;
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = tid + m * T;
            v[m] = k == 0 ? c2r_join<B>(cf{X[0].x, 0.f}, cf{X[0].y, 0.f}, tw + K::TW1, 0)
                          : c2r_join<B>(X[k], X[B - k], tw + K::TW1, k);
        }
    }
    stockham<B, E, +1>(v, fft, tw, tid, active);
    float head = 0.f, tl = 0.f;
    if (active) {
        const float scale = 1.0f / float(2 * B);
        cf* o = reinterpret_cast<cf*>(h0t + int64_t(c) * B);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const cf z = {v[m].x * scale, v[m].y * scale};
            const float a = fmaxf(fabsf(z.x), fabsf(z.y));
            if (m < E / 2) {
                o[tid + m * T] = z;
                head = fmaxf(head, a);
            } else {
                tl = fmaxf(tl, a);
            }
        }
    }
    red[0][tid] = head;
    red[1][tid] = tl;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            red[0][tid] = fmaxf(red[0][tid], red[0][tid + st]);
            red[1][tid] = fmaxf(red[1][tid], red[1][tid + st]);
        }
        __syncthreads();
    }
    if (tid == 0) tail[c] = red[1][0] > 1e-6f * red[0][0] ? 1.f : 0.f;
}

int update_head(upols_t* h, hipStream_t s)
{
    h->direct_ok = false;
    if (h->ola || h->v2 || (h->B != 256 && h->B != 512)) return NEO_HIP_OK;
    if (!h->h0t) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->h0t), size_t(h->C) * h->B * sizeof(float)));
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->h0tail), size_t(h->C) * sizeof(float)));
    }
    if (h->B == 256)
        hipLaunchKernelGGL((k_head_taps<256>), dim3(unsigned(h->C)), dim3(256), 0, s, h->H, h->cstride, h->tw, h->h0t,
                           h->h0tail);
    else
        hipLaunchKernelGGL((k_head_taps<512>), dim3(unsigned(h->C)), dim3(256), 0, s, h->H, h->cstride, h->tw, h->h0t,
                           h->h0tail);
    NEO_HIP_LAUNCH_CHECK();
    std::vector<float> t(size_t(h->C));
    NEO_HIP_CHECK(hipMemcpyAsync(t.data(), h->h0tail, t.size() * sizeof(float), hipMemcpyDeviceToHost, s));
    NEO_HIP_CHECK(hipStreamSynchronize(s));
    // a head with a non-zero second half (a filter not from zero-padded partitions) keeps the
    // transform path for partition 0
    h->direct_ok = std::all_of(t.begin(), t.end(), [](float v) { return v == 0.f; });
    return NEO_HIP_OK;
}

// one k_batch_mac launch: T blocks at write position h->wpos into slabs `part` [C][S][T][B],
// splits of `rows` partitions over [0, P); FDL rows entering past partition `emax` count as
// zero (the lookahead's sub-window passes take only the rows of the current window)
struct mac_pass {
    cf* part;
    int P, S, rows, emax, pc;  // pc: filter rows per channel loaded cacheable
};

static mac_pass full_pass(const upols_t* h) { return {h->part_b, h->P, h->Sb, h->rows_b, 0x7fffffff, h->pcb}; }

// zero FDL row for entering rows past emax, as a row index relative to a channel's FDL base:
// H's first spare row of the same channel (H rows P .. ring-1 are zero; H and FDL share one
// allocation, FDL = H + nrows * B), negative, so buffer loads also see it out of range (0)
static int zero_row(const upols_t* h)
{
    const int64_t fdl_rows = int64_t(h->C) * h->ring * h->B / h->pstride;  // FDL offset in rows
    return int(h->P - fdl_rows);
}

// dispatch k_batch_mac over (B, NB, T) for the valid combinations
template<int BB, int NB>
int launch_batch_mac(const upols_t* h, int T, hipStream_t s, int ahead, const mac_pass& mp)
{
    constexpr int L = batch_cfg<BB, NB>::L;
    const unsigned grid = unsigned(h->C) * unsigned(mp.S) * unsigned(batch_cfg<BB, NB>::G);
    const int rz = zero_row(h);
    const bool lds_ok = mp.emax == 0x7fffffff;  // the LDS-DMA variants take whole passes only
#define NEO_BATCH_T(TT)                                                                                          \
    case TT:                                                                                                     \
        if constexpr (batch_t(BB, NB, TT) == TT) {                                                               \
            if constexpr (TT == 32 && NB == 1 && (BB == 256 || BB == 512)) {                                     \
                if (h->bvar >= 4 && lds_ok) {                                                                    \
                    hipLaunchKernelGGL(h->bvar == 4 ? (k_batch_mac_lds<BB, TT, 4>) : (k_batch_mac_lds<BB, TT, 5>),   \
                                       dim3(grid), dim3(L), 0, s, h->H, h->fdl, mp.part, mp.P, h->ring, mp.S,   \
                                       mp.rows, h->wpos, h->cstride, h->pstride, ahead);                         \
                    break;                                                                                       \
                }                                                                                                \
                if (h->bvar != 0) {                                                                              \
                    hipLaunchKernelGGL(h->bvar == 1   ? (k_batch_mac<BB, TT, NB, 1>)                            \
                                       : h->bvar == 2 ? (k_batch_mac<BB, TT, NB, 2>)                            \
                                                      : (k_batch_mac<BB, TT, NB, 3>),                           \
                                       dim3(grid), dim3(L), 0, s, h->H, h->fdl, mp.part, mp.P, h->ring, mp.S,   \
                                       mp.rows, h->wpos, h->cstride, h->pstride, ahead, mp.emax, rz, mp.pc, h->bprio); \
                    break;                                                                                       \
                }                                                                                                \
            }                                                                                                    \
            if constexpr ((TT == 8 || TT == 16) && NB == 1 && (BB == 256 || BB == 512)) {                       \
                if (h->b8var == 3) { /* 8-block passes (sub-windows, leftovers): buffer loads, D = 8 */          \
                    hipLaunchKernelGGL((k_batch_mac<BB, TT, NB, 3>), dim3(grid), dim3(L), 0, s, h->H, h->fdl,    \
                                       mp.part, mp.P, h->ring, mp.S, mp.rows, h->wpos, h->cstride, h->pstride,   \
                                       ahead, mp.emax, rz, mp.pc, h->bprio);                                     \
                    break;                                                                                       \
                }                                                                                                \
            }                                                                                                    \
            hipLaunchKernelGGL((k_batch_mac<BB, TT, NB, 0>), dim3(grid), dim3(L), 0, s, h->H, h->fdl, mp.part,    \
                               mp.P, h->ring, mp.S, mp.rows, h->wpos, h->cstride, h->pstride, ahead, mp.emax, rz,   \
                               mp.pc, h->bprio);                                                                \
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
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->part_b),
                                size_t(h->C) * h->Sb * kMaxBatch * h->B * sizeof(cf)));
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->part_s), size_t(h->C) * kMaxBatch * h->B * sizeof(cf)));
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
    // two-level lookahead: partitions >= kFarT once per kFarT blocks (upols_far.hip), the
    // level-1 pass over partitions < kFarT only
    const bool far = far_usable(h);
    if (far && h->phase == 0) {
        if (h->fwin <= 0) {
            if ((rc = far_window(h, s))) return rc;
            h->fwin = 0;
            h->fbase = 0;
        } else {
            h->fbase += T;
        }
        h->fwin = (h->fwin + 1) % (kFarT / T);
    }
    const cf* farp = far ? h->ff : nullptr;
    const int fj = far ? h->fbase + h->phase : 0;
    if (h->phase == 0) {
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        const bool timed = h->timing && h->tick++ % h->timing == 0;
        if ((rc = mac_event(h, timed, false, ev, s))) return rc;
        mac_pass mp = full_pass(h);
        if (far) {  // partitions [0, kFarT) in splits of whole 32-partition chunks; splits past it store zeros
            mp.P = kFarT;
            mp.rows = std::max(kMaxBatch, (kFarT / h->Sb + kMaxBatch - 1) / kMaxBatch * kMaxBatch);
            mp.pc = std::min(mp.pc, kFarT);
        }
        if (h->bNB == 2) {
            NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s, 1 | (h->snt ? 2 : 0), mp)))
        } else {
            NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s, 1 | (h->snt ? 2 : 0), mp)))
        }
        if (rc) return rc;
        if ((rc = mac_event(h, timed, true, ev, s))) return rc;
    }
    if (h->akern == 2 && B <= 1024) {
        // sub-windows (sw blocks): at the first block of each after the first, one pass over the
        // window's rows so far; the block step then walks its sub-window's rows only
        const int sw = h->subw;
        const bool sub = h->asub && T % sw == 0 && T > sw;
        const int jr = sub ? h->phase % sw : h->phase;
        // (ssplit: one split per sw partitions, each walks one chunk)
        const int ssub = sub && h->phase >= sw ? (h->ssplit ? h->phase / sw + 1 : 1) : 0;
        if (ssub && jr == 0) {
            const int srows = (h->phase + sw) / ssub;
            const mac_pass mp{h->part_s, h->phase + sw, ssub, srows, h->phase, h->P};
            NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, sw, s, 1 | (h->snt ? 2 : 0), mp)))
            if (rc) return rc;
        }
        const cf* subp = h->part_s;
        const bool direct = sub && h->direct_ok && !h->ola && (B == 256 ? h->adirect >= 1 : B == 512 && h->adirect == 2);
        if (direct) {
            if (B == 256)
                hipLaunchKernelGGL((k_upols_ahead3<256>), dim3(unsigned(h->C)), dim3(ahead3_cfg<256>::NT), 0, s, in,
                                   ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T, h->phase, h->tw,
                                   h->ring, h->wpos, h->cstride, h->pstride, subp, ssub, jr, sw, h->h0t, farp, fj);
            else
                hipLaunchKernelGGL((k_upols_ahead3<512>), dim3(unsigned(h->C)), dim3(ahead3_cfg<512>::NT), 0, s, in,
                                   ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T, h->phase, h->tw,
                                   h->ring, h->wpos, h->cstride, h->pstride, subp, ssub, jr, sw, h->h0t, farp, fj);
        } else if (h->ola) {
            NEO_UPOLS_DISPATCH(B, if constexpr (BB <= 1024) hipLaunchKernelGGL(
                                      (k_upols_ahead2<BB, true>), dim3(unsigned(h->C)), dim3(ahead_cfg<BB>::NT), 0, s, in,
                                      ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T, h->phase, h->tw,
                                      h->ring, h->wpos, h->cstride, h->pstride, subp, ssub, jr, sw, farp, fj))
        } else {
            NEO_UPOLS_DISPATCH(B, if constexpr (BB <= 1024) hipLaunchKernelGGL(
                                      (k_upols_ahead2<BB, false>), dim3(unsigned(h->C)), dim3(ahead_cfg<BB>::NT), 0, s, in,
                                      ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part_b, h->Sb, T, h->phase, h->tw,
                                      h->ring, h->wpos, h->cstride, h->pstride, subp, ssub, jr, sw, farp, fj))
        }
    } else if (h->ola) {
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
    h->fwin = -1;  // the far window restarts at the next lookahead window
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
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s, 0, full_pass(h))))
    } else {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s, 0, full_pass(h))))
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

#ifdef NEO_AHEAD_PROBE
// diagnostic build only: copy channel 0's k_upols_ahead2 phase stamps (s_memrealtime, 100 MHz)
extern "C" __attribute__((visibility("default"))) int neo_hip_debug_probe(unsigned long long* dst)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(neo_hip::g_probe), sizeof(neo_hip::g_probe)) == hipSuccess ? 0 : -1;
}
extern "C" __attribute__((visibility("default"))) int neo_hip_debug_wgspan(unsigned long long* dst)
{
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(neo_hip::g_wgspan), sizeof(neo_hip::g_wgspan)) == hipSuccess ? 0 : -1;
}
#endif
