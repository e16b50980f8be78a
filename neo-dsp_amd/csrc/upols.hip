// upols.hip — multichannel uniformly-partitioned overlap-save convolution on MI355X.
//
// Replaces C instances of neo's upols_convolver<complex<float>>
// (src/neo/convolution/dense_convolver.hpp:19-20) stepped by dense_convolve /
// DenseConvolution (extra/plugin/src/dsp/DenseConvolution.hpp:39-70). One block
// step for all channels is ONE kernel, k_upols_step, grid C x S:
//
//   - workgroup (c, s) accumulates filter partitions p in [p0, p1) of channel c:
//       acc[k] += H[c][p][k] * FDL[c][(w - p) mod R][k]
//     (fdl_index.hpp:23-36 ring order; dense_filter.hpp:30-35 / multiply_add MAC),
//     streaming 16 B per bin per partition from HBM — the roofline part;
//   - split s == 0 first runs the overlap-save r2c of [previous block | new block]
//     (overlap_save.hpp:90-103) as a packed B-point complex FFT in LDS, inserts it as
//     FDL row w (dense_fdl.hpp:27-30) and uses it for p = 0 straight from LDS;
//   - the last split of a channel to finish sums the S partial spectra in fixed order,
//     runs the c2r (fallback_rfft_plan.hpp:38-55) as a packed inverse FFT in LDS,
//     scales by 1/2B and writes the last B samples (overlap_save.hpp:104-111).
//
// Device layout (HBM), all packed rows of B complex with bin 0 = {DC, Nyquist}
// (both purely real for real signals, so the fold is exact):
//   H    [C][R][B]   filter partitions (uniform_partition.hpp layout, packed; rows >= P unused)
//   FDL  [C][R][B]   frequency-domain delay line, a ring of R = P + kMaxBatch - 1 rows
//                    (write position w; the extra rows let a batch of T <= kMaxBatch
//                    new blocks be inserted before any of them is consumed)
//   prev [C][B]      previous input block (first half of the overlap-save window)
//   part [C][S][B]   per-split partial spectra; arrivals [C] split counters
#include "common.hpp"
#include "fft_device_real.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

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
template<int B, bool OLA, int E = (B / 8 <= 256 ? 8 : B / 256)>
__device__ __forceinline__ void window_fft(const float* prev_c, const float* in_c, cf* fft, const cf* tw1, int tid)
{
    constexpr int T = B / E;
    static_assert(T <= 256 && B % E == 0, "window FFT must fit one 256-lane workgroup");
    const bool active = tid < T;
    cf v[E];
    if (active) {
        const cf* pz = reinterpret_cast<const cf*>(prev_c);
        const cf* iz = reinterpret_cast<const cf*>(in_c);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int n = tid + m * T;
            if constexpr (OLA) v[m] = n < B / 2 ? iz[n] : cf{0.f, 0.f};
            else v[m] = n < B / 2 ? pz[n] : iz[n - B / 2];
        }
    }
    __syncthreads();  // twiddles staged by the caller
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
template<int B, bool OLA, int E = (B / 4 <= 256 ? 4 : B / 256)>
__device__ __forceinline__ void c2r_tail(const cf* X, cf* fft, const cf* tw, float* out_c, float* ovl_c, int tid)
{
    using K = upols_cfg<B>;
    constexpr int T = B / E;
    static_assert(T <= 256 && B % E == 0, "c2r must fit one 256-lane workgroup");
    const bool active = tid < T;
    cf v[E];
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = tid + m * T;
            const cf x0 = X[0];
            v[m] = k == 0 ? c2r_join<B>(cf{x0.x, 0.f}, cf{x0.y, 0.f}, tw + K::TW1, 0)
                          : c2r_join<B>(X[k], X[B - k], tw + K::TW1, k);
        }
    }
    stockham<B, E, +1>(v, fft, tw, tid, active);
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
                o[n] = {v[m].x * scale + old.x, v[m].y * scale + old.y};
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
                o[n - B / 2] = {v[m].x * scale, v[m].y * scale};
            }
        }
    }
}

// One whole block step for every channel (grid C x S, 256 lanes). Workgroup (c, s)
// accumulates partitions [p0, p1) into a partial spectrum; split 0 first runs the
// window r2c and inserts FDL row w. Each workgroup publishes its slab, and the last
// of a channel's S workgroups to arrive (agent-scope release -> counter -> acquire,
// cdna_hip_programming.md §6 G16 / split-K seam) sums the slabs in the fixed order
// s = 0..S-1 and runs the c2r: one launch per block, deterministic results.
// TAIL (upola_convolver_v2 sub-block pieces): no window / insert, partitions p >= 1 only
// (overlap_add_convolver.hpp:96-108), slabs summed by k_upola2_piece.
template<int B, bool FUSED, bool OLA, bool TAIL = false, int UNROLL = upols_cfg<B>::U>
__global__ __launch_bounds__(256, (B <= 1024 ? 8 : 2)) void k_upols_step(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, cf* __restrict__ part, int* __restrict__ arrivals,
    const cf* __restrict__ twg, int P, int ring, int S, int rows, int w, int64_t cstride, int64_t pstride)
{
    using K = upols_cfg<B>;
    static_assert(!(TAIL && FUSED), "the v2 tail is summed by k_upola2_piece");
    __shared__ __attribute__((aligned(16))) cf xnew[B];  // new spectrum; later the summed spectrum
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    __shared__ __attribute__((aligned(16))) float4 red[K::RPI > 1 ? 256 * 2 * K::VPT : 1];
    __shared__ int last;

    const int tid = threadIdx.x;
    const int c = blockIdx.x / S, s = blockIdx.x - c * S;
    const int p0 = s * rows, p1 = min(P, p0 + rows);
    const int64_t crow = int64_t(c) * cstride;  // channel base in H / FDL (complex units); row p at + p * pstride
    const int64_t ps4 = pstride / 2;            // row stride in float4 units

    if (!TAIL && s == 0) {
        for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
        const float* in_c = in + int64_t(c) * ld_in;
        float* prev_c = prev + int64_t(c) * B;
        window_fft<B, OLA>(prev_c, in_c, fft, tw, tid);
        cf* row = fdl + crow + int64_t(w) * pstride;
        for (int k = tid; k < B; k += 256) {
            const cf x = r2c_split<B>(fft, tw + K::TW1, k);
            xnew[k] = x;
            row[k] = x;
        }
        if constexpr (!OLA) {  // the window's second half becomes the next call's first half
            for (int i = tid; i < B / 4; i += 256)
                reinterpret_cast<float4*>(prev_c)[i] = reinterpret_cast<const float4*>(in_c)[i];
        }
        __syncthreads();
    }

    const int rs = tid / K::QT, q0 = tid - rs * K::QT;
    acc4 a[2 * K::VPT];
#pragma unroll
    for (int v = 0; v < 2 * K::VPT; ++v) a[v] = {0.f, 0.f, 0.f, 0.f};

    const float4* H4 = reinterpret_cast<const float4*>(H + crow);
    const float4* F4 = reinterpret_cast<const float4*>(fdl + crow);
    int pstart = p0;
    if (TAIL && p0 == 0) pstart = 1;
    if (!TAIL && p0 == 0) {
        if (rs == 0) {
            const float4* Xn = reinterpret_cast<const float4*>(xnew);
#pragma unroll
            for (int v = 0; v < K::VPT; ++v) {
                const int q = q0 + v * K::QT;
                mac2(a[2 * v], a[2 * v + 1], H4[q], Xn[q]);
            }
        }
        pstart = 1;
    }
    // main loop: UNROLL row-groups in flight, no bounds checks inside
    int p = pstart + rs;
    for (; p + (UNROLL - 1) * K::RPI < p1; p += UNROLL * K::RPI) {
        float4 hv[UNROLL][K::VPT], xv[UNROLL][K::VPT];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int pp = p + u * K::RPI;
            const int fr = w >= pp ? w - pp : w - pp + ring;  // fdl_index.hpp:28-31 ring
#pragma unroll
            for (int v = 0; v < K::VPT; ++v) {
                const int q = q0 + v * K::QT;
                hv[u][v] = ld4_nt(H4 + int64_t(pp) * ps4 + q);
                xv[u][v] = ld4_nt(F4 + int64_t(fr) * ps4 + q);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int v = 0; v < K::VPT; ++v) mac2(a[2 * v], a[2 * v + 1], hv[u][v], xv[u][v]);
    }
    for (; p < p1; p += K::RPI) {
        const int fr = w >= p ? w - p : w - p + ring;
#pragma unroll
        for (int v = 0; v < K::VPT; ++v) {
            const int q = q0 + v * K::QT;
            mac2(a[2 * v], a[2 * v + 1], ld4_nt(H4 + int64_t(p) * ps4 + q), ld4_nt(F4 + int64_t(fr) * ps4 + q));
        }
    }

    if constexpr (K::RPI > 1) {
        // fold the row groups into group 0 (fixed order -> deterministic)
#pragma unroll
        for (int v = 0; v < K::VPT; ++v) {
            red[(tid * K::VPT + v) * 2 + 0] = make_float4(a[2 * v].rr, a[2 * v].ii, a[2 * v].ri, a[2 * v].ir);
            red[(tid * K::VPT + v) * 2 + 1] =
                make_float4(a[2 * v + 1].rr, a[2 * v + 1].ii, a[2 * v + 1].ri, a[2 * v + 1].ir);
        }
        __syncthreads();
        if (rs == 0) {
            for (int g = 1; g < K::RPI; ++g) {
#pragma unroll
                for (int v = 0; v < K::VPT; ++v) {
                    const int idx = ((g * K::QT + q0) * K::VPT + v) * 2;
                    const float4 r0 = red[idx], r1 = red[idx + 1];
                    a[2 * v].rr += r0.x; a[2 * v].ii += r0.y; a[2 * v].ri += r0.z; a[2 * v].ir += r0.w;
                    a[2 * v + 1].rr += r1.x; a[2 * v + 1].ii += r1.y; a[2 * v + 1].ri += r1.z; a[2 * v + 1].ir += r1.w;
                }
            }
        }
    }
    float* out_c = out + int64_t(c) * ld_out;

    if (FUSED && S == 1) {  // whole channel in this workgroup: finish straight from registers
        __syncthreads();  // xnew reads (p = 0) done before it is overwritten
        if (rs == 0) {
#pragma unroll
            for (int v = 0; v < K::VPT; ++v) {
                const int q = q0 + v * K::QT;
                const cf b0 = finish(a[2 * v], q == 0), b1 = finish(a[2 * v + 1], false);
                reinterpret_cast<float4*>(xnew)[q] = make_float4(b0.x, b0.y, b1.x, b1.y);
            }
        }
        __syncthreads();
        c2r_tail<B, OLA>(xnew, fft, tw, out_c, prev + int64_t(c) * B, tid);
        return;
    }

    // publish this split's slab
    float4* slab = reinterpret_cast<float4*>(part + (int64_t(c) * S + s) * B);
    if (rs == 0) {
#pragma unroll
        for (int v = 0; v < K::VPT; ++v) {
            const int q = q0 + v * K::QT;
            const cf b0 = finish(a[2 * v], q == 0), b1 = finish(a[2 * v + 1], false);
            slab[q] = make_float4(b0.x, b0.y, b1.x, b1.y);
        }
    }
    if constexpr (!FUSED) return;  // k_upols_finish sums the slabs in the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the release's wait (G16 pitfall)
        const int before = __hip_atomic_fetch_add(arrivals + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = before == S - 1;
    }
    __syncthreads();
    if (!last) return;  // uniform per workgroup
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(arrivals + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next step
    }
    if (s != 0)
        for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    __syncthreads();

    // sum the S slabs in order s = 0..S-1, 8 loads in flight
    const float4* p4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * B);
    for (int q = tid; q < K::Q; q += 256) {
        float4 sum = p4[q];
        int t = 1;
        for (; t + 7 < S; t += 8) {
            float4 r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) r[u] = p4[int64_t(t + u) * K::Q + q];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                sum.x += r[u].x; sum.y += r[u].y; sum.z += r[u].z; sum.w += r[u].w;
            }
        }
        for (; t < S; ++t) {
            const float4 r = p4[int64_t(t) * K::Q + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        reinterpret_cast<float4*>(xnew)[q] = sum;
    }
    __syncthreads();
    c2r_tail<B, OLA>(xnew, fft, tw, out_c, prev + int64_t(c) * B, tid);
}

// Unfused tail (one workgroup per channel): sum the S slabs in order, c2r, write.
template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_upols_finish(const cf* __restrict__ part, float* __restrict__ out,
                                                      int64_t ld_out, float* __restrict__ ovl,
                                                      const cf* __restrict__ twg, int S)
{
    using K = upols_cfg<B>;
    __shared__ __attribute__((aligned(16))) cf X[B];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    const float4* p4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * B);
    for (int q = tid; q < K::Q; q += 256) {
        float4 sum = p4[q];
        int t = 1;
        for (; t + 7 < S; t += 8) {
            float4 r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) r[u] = p4[int64_t(t + u) * K::Q + q];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                sum.x += r[u].x; sum.y += r[u].y; sum.z += r[u].z; sum.w += r[u].w;
            }
        }
        for (; t < S; ++t) {
            const float4 r = p4[int64_t(t) * K::Q + q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        reinterpret_cast<float4*>(X)[q] = sum;
    }
    __syncthreads();
    c2r_tail<B, OLA, NEO_FINISH_E(B)>(X, fft, tw, out + int64_t(c) * ld_out,
                                                                     ovl + int64_t(c) * B, tid);
}

// upola_convolver_v2 piece (overlap_add_convolver.hpp:71-136), one workgroup per channel,
// for n samples at block position pos. The real window [C][2B] is state, exactly as in
// the reference: the irfft result is written back into it (:114), so a later piece of
// the same block transforms [earlier output | new samples | earlier output]. Steps:
//   sum_first (pos == 0): tmp = sum of the TAIL slabs (partitions p >= 1, :96-108)
//   window[pos, pos+n) = input; X = rfft(window); FDL row w = X          (:90-94)
//   acc = tmp + X * H[0]                                                 (:110-112)
//   window = irfft(acc) / 2B; out = window[pos, pos+n) + overlap[...]    (:114-118)
//   complete (pos + n == B): overlap = window[B, 2B); window = 0         (:122-131)
// Whole blocks at pos 0 take the UPOLA launch pair instead: with a zero window and
// full input the two are the same computation.
template<int B>
__global__ __launch_bounds__(256) void k_upola2_piece(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, int n, int pos,
    float* __restrict__ window, float* __restrict__ ovl, cf* __restrict__ tmp, const cf* __restrict__ part, int S,
    int sum_first, const cf* __restrict__ H, cf* __restrict__ fdl, int w, const cf* __restrict__ twg, int64_t cstride,
    int64_t pstride)
{
    using K = upols_cfg<B>;
    constexpr int E = K::E, T = K::T;
    __shared__ __attribute__((aligned(16))) float wl[2 * B];  // real window, then the irfft output
    __shared__ __attribute__((aligned(16))) cf acc[B];
    __shared__ cf fft[K::LL];
    __shared__ cf tw[K::TW1 + K::TW2];
    const int tid = threadIdx.x, c = blockIdx.x;
    for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];

    cf* tmp_c = tmp + int64_t(c) * B;
    if (sum_first) {  // fixed order s = 0..S-1, like k_upols_finish
        const cf* pc = part + int64_t(c) * S * B;
        for (int k = tid; k < B; k += 256) {
            cf sum = pc[k];
            for (int t = 1; t < S; ++t) {
                const cf r = pc[int64_t(t) * B + k];
                sum.x += r.x;
                sum.y += r.y;
            }
            acc[k] = sum;
            tmp_c[k] = sum;
        }
    } else {
        for (int k = tid; k < B; k += 256) acc[k] = tmp_c[k];
    }
    float* win_c = window + int64_t(c) * 2 * B;
    const float* in_c = in + int64_t(c) * ld_in;
    for (int i = tid; i < 2 * B; i += 256) wl[i] = (i >= pos && i < pos + n) ? in_c[i - pos] : win_c[i];
    __syncthreads();

    const bool active = tid < T;
    cf v[E];
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = reinterpret_cast<const cf*>(wl)[tid + m * T];
    }
    stockham<B, E, -1>(v, fft, tw, tid, active);
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) fft[lpad(tid + m * T)] = v[m];
    }
    __syncthreads();
    cf* row = fdl + int64_t(c) * cstride + int64_t(w) * pstride;
    const cf* h0 = H + int64_t(c) * cstride;  // partition 0
    for (int k = tid; k < B; k += 256) {
        const cf x = r2c_split<B>(fft, tw + K::TW1, k), h = h0[k], a = acc[k];
        row[k] = x;
        acc[k] = k == 0 ? cf{x.x * h.x + a.x, x.y * h.y + a.y}  // packed {DC, Nyquist}: real products
                        : cf{(x.x * h.x - x.y * h.y) + a.x, (x.x * h.y + x.y * h.x) + a.y};
    }
    __syncthreads();
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = tid + m * T;
            const cf a0 = acc[0];
            v[m] = k == 0 ? c2r_join<B>(cf{a0.x, 0.f}, cf{a0.y, 0.f}, tw + K::TW1, 0)
                          : c2r_join<B>(acc[k], acc[B - k], tw + K::TW1, k);
        }
    }
    stockham<B, E, +1>(v, fft, tw, tid, active);
    if (active) {
        const float scale = 1.0f / float(2 * B);  // :115
#pragma unroll
        for (int m = 0; m < E; ++m) reinterpret_cast<cf*>(wl)[tid + m * T] = {v[m].x * scale, v[m].y * scale};
    }
    __syncthreads();
    float* out_c = out + int64_t(c) * ld_out;
    float* ovl_c = ovl + int64_t(c) * B;
    for (int j = tid; j < n; j += 256) out_c[j] = wl[pos + j] + ovl_c[pos + j];
    if (pos + n == B) {
        __syncthreads();  // overlap reads above are done before it is replaced
        for (int i = tid; i < B; i += 256) ovl_c[i] = wl[B + i];
        for (int i = tid; i < 2 * B; i += 256) win_c[i] = 0.0f;
    } else {
        for (int i = tid; i < 2 * B; i += 256) win_c[i] = wl[i];
    }
}

// ---------------------------------------------------------------------------
// Batched blocks (process_blocks): T consecutive blocks per pass over H and the FDL.
// ---------------------------------------------------------------------------
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
    const bool valid = p < p1;  // the last chunk of a split may run past p1: zero filter row
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        f[(T - U) % T][v] = pf[slot][v];
        hv[v] = valid ? ph[slot][v] : bvec<NB>(0.0f);
    }
    const int pn = p + D < p1 ? p + D : p1 - 1;  // past the end: a harmless re-read, no branch
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
                                                                   int64_t cstride, int64_t pstride)
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
    V f[T][VPT];
#pragma unroll
    for (int sl = 1; sl < T; ++sl) {  // rows block sl needs at p0
        int r = w + sl - p0;
        r = r < 0 ? r + ring : (r >= ring ? r - ring : r);
#pragma unroll
        for (int v = 0; v < VPT; ++v) f[sl][v] = __builtin_nontemporal_load(Fv + int64_t(r) * psv + tid + v * L);
    }
    V ph[D][VPT], pf[D][VPT];
#pragma unroll
    for (int d = 0; d < D; ++d) {  // prefetch partitions p0 .. p0 + D - 1
        const int p = p0 + d < p1 ? p0 + d : p0;
        int r = w - p;
        r = r < 0 ? r + ring : r;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            pf[d][v] = __builtin_nontemporal_load(Fv + int64_t(r) * psv + tid + v * L);
            ph[d][v] = __builtin_nontemporal_load(Hv + int64_t(p) * psv + tid + v * L);
        }
    }
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

// ---------------------------------------------------------------------------
// setup path
// ---------------------------------------------------------------------------
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

}  // namespace neo_hip

using namespace neo_hip;

namespace neo_hip {
constexpr int kMaxBatch = 32;
constexpr double kFusedMaxBytes = 64.0 * 1024 * 1024;  // filter + FDL bytes below which a step is one launch  // most blocks one batched MAC pass consumes (process_blocks)
}

struct neo_hip_upols {
    int device = 0, C = 0, B = 0, P = 0, S = 1, rows = 1;
    int ring = 0;  // FDL ring rows R = P + kMaxBatch - 1
    hipStream_t stream = nullptr;
    cf* H = nullptr;
    cf* fdl = nullptr;
    cf* part = nullptr;
    float* prev = nullptr;
    int* arrivals = nullptr;  // per-channel split arrival counters (zero between steps)
    int wpos = 0;             // FDL write position (fdl_index.hpp:35-37), host-side
    cf* tw = nullptr;
    float* io = nullptr;       // device staging for host-pointer process()
    float* io_host = nullptr;  // pinned staging
    bool batch = true;      // process_blocks runs T blocks per MAC pass (neo_hip_upols_set_batch)
    int Sb = 1, rows_b = 1; // batched-pass splits per channel and partitions per split
    int bT = 32, bNB = 1;   // batched pass: blocks per pass (capped by batch_t), bins per lane-vector
    cf* part_b = nullptr;   // batched partial spectra [C][Sb][T][B]
    float* tail = nullptr;  // batched OLA tails [C][T][B]
    float* samples_dev = nullptr;   // process_samples host staging (device side)
    float* samples_host = nullptr;  // process_samples host staging (pinned)
    size_t samples_cap = 0;
    bool timing = false;
    bool ola = false;  // upola_convolver (overlap-add stage) instead of upols (overlap-save)
    bool v2 = false;   // upola_convolver_v2: sub-block input (implies ola)
    int in_pos = 0;    // v2: samples of the current block already consumed (_input_pos)
    float* window = nullptr;  // v2: real window [C][2B]
    cf* tmp = nullptr;        // v2: tail accumulator [C][B] packed (_tmp_accumulator)
    // one launch per block (last-arriver tail) instead of MAC + finish: on for small filter
    // + FDL working sets, where the step is launch-bound (C3: 10.6 vs 12.4 us per block),
    // off for HBM-bound ones (C5: 0.342 vs 0.303 ms); NEO_HIP_FUSED=0/1 overrides
    bool fused = false;
    // H / FDL layout: row p of channel c at c * cstride + p * pstride (complex units).
    // Default [C][P][B]; NEO_HIP_LAYOUT=pcb selects partition-major [P][C][B] (A/B).
    int64_t cstride = 0, pstride = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // pool, reused across timing windows
    size_t events_used = 0;
    double mac_ms = 0.0;
    int64_t launches = 0;
};

namespace {

using upols_t = neo_hip_upols;

bool valid_block(int b) { return b >= 16 && b <= 4096 && (b & (b - 1)) == 0; }

#define NEO_UPOLS_DISPATCH(B_, BODY) \
    switch (B_) {                    \
        case 16: { constexpr int BB = 16; BODY; break; }     \
        case 32: { constexpr int BB = 32; BODY; break; }     \
        case 64: { constexpr int BB = 64; BODY; break; }     \
        case 128: { constexpr int BB = 128; BODY; break; }   \
        case 256: { constexpr int BB = 256; BODY; break; }   \
        case 512: { constexpr int BB = 512; BODY; break; }   \
        case 1024: { constexpr int BB = 1024; BODY; break; } \
        case 2048: { constexpr int BB = 2048; BODY; break; } \
        case 4096: { constexpr int BB = 4096; BODY; break; } \
        default: return fail(NEO_HIP_EINVAL, "unsupported block size %d", B_); \
    }

int64_t partitions_for(int64_t L, int B)
{
    // stft.hpp:21-25 with overlap 0: idiv(L - B, B) + 1 (= ceil(L/B) for L >= B);
    // the reference underflows for L < B, we clamp to one partition.
    if (L <= B) return 1;
    return (L - B + B - 1) / B + 1;
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

int reset_state(upols_t* h, hipStream_t s)
{
    NEO_HIP_CHECK(hipMemsetAsync(h->fdl, 0, size_t(h->C) * h->ring * h->B * sizeof(cf), s));
    NEO_HIP_CHECK(hipMemsetAsync(h->prev, 0, size_t(h->C) * h->B * sizeof(float), s));
    NEO_HIP_CHECK(hipMemsetAsync(h->arrivals, 0, size_t(h->C) * sizeof(int), s));
    if (h->v2) {
        NEO_HIP_CHECK(hipMemsetAsync(h->window, 0, size_t(h->C) * 2 * h->B * sizeof(float), s));
        NEO_HIP_CHECK(hipMemsetAsync(h->tmp, 0, size_t(h->C) * h->B * sizeof(cf), s));
    }
    h->wpos = 0;
    h->in_pos = 0;
    return NEO_HIP_OK;
}

void destroy(upols_t* h)
{
    if (!h) return;
    for (auto& e : h->events) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    (void)hipFree(h->H);
    (void)hipFree(h->fdl);
    (void)hipFree(h->part);
    (void)hipFree(h->prev);
    (void)hipFree(h->arrivals);
    (void)hipFree(h->window);
    (void)hipFree(h->tmp);
    (void)hipFree(h->tw);
    (void)hipFree(h->io);
    if (h->io_host) (void)hipHostFree(h->io_host);
    (void)hipFree(h->samples_dev);
    (void)hipFree(h->part_b);
    (void)hipFree(h->tail);
    if (h->samples_host) (void)hipHostFree(h->samples_host);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

// normalize (optional) + partition ir [C][L] (device) into packed or unpacked rows.
int partition_device(const float* d_ir, int C, int64_t L, int B, bool packed, cf* out, const cf* tw, hipStream_t s,
                     int64_t cstride = 0, int64_t pstride = 0)
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

int launch_step(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s)
{
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (h->timing) {
        if (h->events_used == h->events.size()) {
            NEO_HIP_CHECK(hipEventCreate(&ev.first));
            NEO_HIP_CHECK(hipEventCreate(&ev.second));
            h->events.push_back(ev);
        }
        ev = h->events[h->events_used];
        NEO_HIP_CHECK(hipEventRecord(ev.first, s));
    }
    const unsigned grid = unsigned(h->C) * unsigned(h->S);
#define NEO_STEP(FU, OL)                                                                                      \
    NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_step<BB, FU, OL>), dim3(grid), dim3(256), 0, s, in, ld_in, \
                                                out, ld_out, h->prev, h->H, h->fdl, h->part, h->arrivals, h->tw,   \
                                                h->P, h->ring, h->S, h->rows, h->wpos, h->cstride, h->pstride))
    if (h->fused) {
        if (h->ola) NEO_STEP(true, true) else NEO_STEP(true, false)
    } else {
        if (h->ola) NEO_STEP(false, true) else NEO_STEP(false, false)
    }
#undef NEO_STEP
    NEO_HIP_LAUNCH_CHECK();
    if (h->timing) {
        NEO_HIP_CHECK(hipEventRecord(ev.second, s));
        ++h->events_used;
    }
    if (!h->fused) {
        if (h->ola) {
            NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_finish<BB, true>), dim3(unsigned(h->C)), dim3(256), 0,
                                                        s, h->part, out, ld_out, h->prev, h->tw, h->S))
        } else {
            NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_finish<BB, false>), dim3(unsigned(h->C)), dim3(256),
                                                        0, s, h->part, out, ld_out, h->prev, h->tw, h->S))
        }
        NEO_HIP_LAUNCH_CHECK();
    }
    h->wpos = h->wpos + 1 >= h->ring ? 0 : h->wpos + 1;  // fdl_index.hpp:35-37
    return NEO_HIP_OK;
}

// blocks per batched pass for block B and NB bins per lane-vector: the requested T,
// capped so one lane's accumulators (T * NB * VPT * 4 floats) stay <= 128 registers
constexpr int batch_t(int B, int NB, int want)
{
    (void)B;
    const int VPT = 1;
    int t = want;
    while (t > 2 && t * NB * VPT > 32) t /= 2;
    return t;
}

int batch_blocks(const upols_t* h) { return batch_t(h->B, h->bNB, h->bT); }

// dispatch k_batch_mac over (B, NB, T) for the valid combinations
template<int BB, int NB>
int launch_batch_mac(const upols_t* h, int T, hipStream_t s)
{
    constexpr int L = batch_cfg<BB, NB>::L;
    const unsigned grid = unsigned(h->C) * unsigned(h->Sb) * unsigned(batch_cfg<BB, NB>::G);
#define NEO_BATCH_T(TT)                                                                                          \
    case TT:                                                                                                     \
        if constexpr (batch_t(BB, NB, TT) == TT) {                                                               \
            hipLaunchKernelGGL((k_batch_mac<BB, TT, NB>), dim3(grid), dim3(L), 0, s, h->H, h->fdl, h->part_b, h->P, \
                               h->ring, h->Sb, h->rows_b, h->wpos, h->cstride, h->pstride);                      \
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
int launch_batch(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int T, hipStream_t s)
{
    const int B = h->B;
    if (!h->part_b) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->part_b),
                                size_t(h->C) * h->Sb * kMaxBatch * B * sizeof(cf)));
        if (h->ola)
            NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->tail), size_t(h->C) * kMaxBatch * B * sizeof(float)));
    }
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
    if (h->timing) {
        if (h->events_used == h->events.size()) {
            NEO_HIP_CHECK(hipEventCreate(&ev.first));
            NEO_HIP_CHECK(hipEventCreate(&ev.second));
            h->events.push_back(ev);
        }
        ev = h->events[h->events_used];
        NEO_HIP_CHECK(hipEventRecord(ev.first, s));
    }
    int rc = NEO_HIP_OK;
    if (h->bNB == 2) {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 2>(h, T, s)))
    } else {
        NEO_UPOLS_DISPATCH(B, rc = (launch_batch_mac<BB, 1>(h, T, s)))
    }
    if (rc) return rc;
    if (h->timing) {
        NEO_HIP_CHECK(hipEventRecord(ev.second, s));
        ++h->events_used;
    }
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

// One v2 piece of n samples at block position h->in_pos (n <= B - in_pos).
int launch_piece(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int n, hipStream_t s)
{
    const int sum_first = h->in_pos == 0;
    if (sum_first) {  // tail MAC over partitions p >= 1 into the split slabs
        const unsigned grid = unsigned(h->C) * unsigned(h->S);
        NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_step<BB, false, true, true>), dim3(grid), dim3(256), 0, s,
                                                    in, ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part,
                                                    h->arrivals, h->tw, h->P, h->ring, h->S, h->rows, h->wpos,
                                                    h->cstride,
                                                    h->pstride))
        NEO_HIP_LAUNCH_CHECK();
    }
    NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upola2_piece<BB>), dim3(unsigned(h->C)), dim3(256), 0, s, in, ld_in,
                                                out, ld_out, n, h->in_pos, h->window, h->prev, h->tmp, h->part, h->S,
                                                sum_first, h->H, h->fdl, h->wpos, h->tw, h->cstride, h->pstride))
    NEO_HIP_LAUNCH_CHECK();
    h->in_pos += n;
    if (h->in_pos == h->B) {  // block complete: next FDL row (overlap_add_convolver.hpp:131)
        h->in_pos = 0;
        h->wpos = h->wpos + 1 >= h->ring ? 0 : h->wpos + 1;
    }
    return NEO_HIP_OK;
}

// Any number of samples for every channel (channel c at in + c * ld_in). upols / upola
// handles take whole blocks only; v2 handles split the samples at block boundaries
// (overlap_add_convolver.hpp:80-134) and run whole aligned blocks through launch_step.
int process_samples(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int64_t n, hipStream_t s)
{
    const int B = h->B;
    const int T = h->batch ? batch_blocks(h) : 1;
    const bool a16 = !((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) &&
                     !((ld_in | ld_out) & 3);
    if (!h->v2) {
        if (n % B) return fail(NEO_HIP_EINVAL, "upols/upola convolvers take whole blocks (%lld samples, block %d)",
                               (long long)n, B);
        if (!a16) return fail(NEO_HIP_EINVAL, "device I/O must be 16-byte aligned (ld multiple of 4)");
    }
    int64_t done = 0;
    while (done < n) {
        const float* ip = in + done;
        float* op = out + done;
        int rc;
        // the largest power-of-two batch (<= T) of whole blocks left, one pass over H + FDL
        int tb = 1;
        while (tb * 2 <= T && n - done >= int64_t(tb) * 2 * B) tb *= 2;
        if (h->in_pos == 0 && tb > 1 && a16 && done % 4 == 0) {
            rc = launch_batch(h, ip, ld_in, op, ld_out, tb, s);
            done += int64_t(tb) * B;
        } else if (!h->v2) {
            rc = launch_step(h, ip, ld_in, op, ld_out, s);
            done += B;
        } else {
            const int k = int(std::min<int64_t>(n - done, B - h->in_pos));
            // whole block on an 8-byte grid: the UPOLA pair computes the same thing
            const bool pair = h->in_pos == 0 && k == B &&
                              !((reinterpret_cast<uintptr_t>(ip) | reinterpret_cast<uintptr_t>(op)) & 7) &&
                              !((ld_in | ld_out) & 1);
            rc = pair ? launch_step(h, ip, ld_in, op, ld_out, s) : launch_piece(h, ip, ld_in, op, ld_out, k, s);
            done += k;
        }
        if (rc) return rc;
    }
    return NEO_HIP_OK;
}

}  // namespace

extern "C" {

NEO_HIP_API int neo_hip_num_partitions(int64_t length, int block, int64_t* partitions)
{
    if (!partitions || block < 1 || length < 0) return fail(NEO_HIP_EINVAL, "bad arguments");
    *partitions = partitions_for(length, block);
    return NEO_HIP_OK;
}

}  // extern "C"

namespace {
int create_convolver(int channels, int block, int partitions, int device, bool ola, bool v2, neo_hip_upols** out)
{
    if (!out) return fail(NEO_HIP_EINVAL, "handle pointer is null");
    *out = nullptr;
    if (channels < 1) return fail(NEO_HIP_EINVAL, "channels must be >= 1");
    if (!valid_block(block)) return fail(NEO_HIP_EINVAL, "block must be a power of two in [16, 4096], got %d", block);
    if (partitions < 1) return fail(NEO_HIP_EINVAL, "partitions must be >= 1");
    device_guard g(device);
    if (g.rc) return g.rc;
    auto* h = new upols_t{};
    (void)hipGetDevice(&h->device);
    h->C = channels;
    h->B = block;
    h->P = partitions;
    h->ring = partitions + kMaxBatch - 1;
    if (const char* e = std::getenv("NEO_HIP_RING_EXTRA"))  // A/B: ring rows beyond P
        h->ring = partitions + std::max(0, std::min(kMaxBatch - 1, std::atoi(e)));
    h->ola = ola || v2;
    h->v2 = v2;
    h->fused = 2.0 * 8.0 * double(channels) * double(partitions) * double(block) < double(kFusedMaxBytes);
    if (const char* e = std::getenv("NEO_HIP_FUSED")) h->fused = std::atoi(e) != 0;
    h->cstride = int64_t(h->ring) * block;
    h->pstride = block;
    if (const char* e = std::getenv("NEO_HIP_LAYOUT"); e && std::string(e) == "pcb") {
        h->cstride = block;
        h->pstride = int64_t(channels) * block;
    }
    // splits per channel: aim for ~1024 workgroups (4 per CU, all resident at 8 waves/SIMD;
    // A/B on MI355X: 1024 beat 512/768/2048/4096 at C4 and C5), <= 64 partial slabs
    int target = 1024;
    if (const char* e = std::getenv("NEO_HIP_SPLIT_WGS")) target = std::max(1, std::atoi(e));
    // >= 8 rows per split keeps the out kernel's slab sum short at small C (C3: 24 splits)
    int S = std::max(1, std::min({(target + channels - 1) / channels, (partitions + 7) / 8, 64}));
    h->rows = (partitions + S - 1) / S;
    h->S = (partitions + h->rows - 1) / h->rows;
    // batched passes: same workgroup target, >= 2T partitions per split so the sliding FDL
    // window's warm-up (T - 1 extra rows per split) stays under half the split's rows
    if (const char* e = std::getenv("NEO_HIP_BATCH_T")) h->bT = std::max(2, std::min(kMaxBatch, std::atoi(e)));
    if (const char* e = std::getenv("NEO_HIP_BATCH_NB")) h->bNB = std::atoi(e) == 1 ? 1 : 2;
    int btarget = target;
    if (const char* e = std::getenv("NEO_HIP_BATCH_WGS")) btarget = std::max(1, std::atoi(e));
    const int bt = batch_t(block, h->bNB, h->bT);
    int Sb = std::max(1, std::min({(btarget + channels - 1) / channels, partitions / (2 * bt), 64}));
    if (h->ring - partitions < bt - 1) h->batch = false;  // ring too short for a batch
    h->rows_b = (partitions + Sb - 1) / Sb;
    h->Sb = (partitions + h->rows_b - 1) / h->rows_b;
    const size_t rowbytes = size_t(block) * sizeof(cf);
    const size_t nrows = size_t(channels) * size_t(h->ring);  // H uses the first P rows of each channel
    auto bail = [&](int code) {
        destroy(h);
        return code;
    };
    if (hipStreamCreateWithFlags(&h->stream, hipStreamDefault) != hipSuccess)
        return bail(fail(NEO_HIP_ERUNTIME, "hipStreamCreate failed"));
    if (hipMalloc(reinterpret_cast<void**>(&h->H), nrows * rowbytes) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&h->fdl), nrows * rowbytes) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&h->part), size_t(channels) * h->S * rowbytes) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&h->prev), size_t(channels) * block * sizeof(float)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&h->arrivals), size_t(channels) * sizeof(int)) != hipSuccess ||
        (v2 && (hipMalloc(reinterpret_cast<void**>(&h->window), size_t(channels) * 2 * block * sizeof(float)) !=
                    hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&h->tmp), size_t(channels) * rowbytes) != hipSuccess)))
        return bail(fail(NEO_HIP_ENOMEM, "device allocation of %zu bytes failed", 2 * nrows * rowbytes));
    int rc = upload_tw(&h->tw, block);
    if (rc) return bail(rc);
    if (hipMemset(h->H, 0, nrows * rowbytes) != hipSuccess) return bail(fail(NEO_HIP_ERUNTIME, "memset failed"));
    if ((rc = reset_state(h, h->stream))) return bail(rc);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(NEO_HIP_ERUNTIME, "sync failed"));
    *out = h;
    return NEO_HIP_OK;
}
}  // namespace

extern "C" {

NEO_HIP_API int neo_hip_upols_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, false, false, out);
}

NEO_HIP_API int neo_hip_upola_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, true, false, out);
}

NEO_HIP_API int neo_hip_upola2_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, true, true, out);
}

NEO_HIP_API int neo_hip_upols_destroy(neo_hip_upols* h)
{
    if (!h) return NEO_HIP_OK;
    device_guard g(h->device);
    (void)hipStreamSynchronize(h->stream);
    destroy(h);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_info(neo_hip_upols* h, int* channels, int* block, int* partitions, int* splits)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (channels) *channels = h->C;
    if (block) *block = h->B;
    if (partitions) *partitions = h->P;
    if (splits) *splits = h->S;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_reset(neo_hip_upols* h)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    device_guard g(h->device);
    NEO_HIP_CHECK(hipDeviceSynchronize());  // setup calls order after all prior work, any stream
    int rc = reset_state(h, h->stream);
    if (rc) return rc;
    NEO_HIP_CHECK(hipStreamSynchronize(h->stream));
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_filter(neo_hip_upols* h, const void* filter, int is_device)
{
    if (!h || !filter) return fail(NEO_HIP_EINVAL, "null handle or filter");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    NEO_HIP_CHECK(hipDeviceSynchronize());  // setup calls order after all prior work, any stream
    const int64_t rows = int64_t(h->C) * h->P;
    const size_t bytes = size_t(rows) * size_t(h->B + 1) * sizeof(cf);
    const cf* src = static_cast<const cf*>(filter);
    cf* tmp = nullptr;
    if (!is_device) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&tmp), bytes));
        NEO_HIP_CHECK(hipMemcpyAsync(tmp, filter, bytes, hipMemcpyHostToDevice, h->stream));
        src = tmp;
    }
    const int64_t total = rows * h->B;
    hipLaunchKernelGGL(k_pack_filter, dim3(unsigned((total + 255) / 256)), dim3(256), 0, h->stream, src, h->H, h->B,
                       rows, h->P, h->cstride, h->pstride);
    int rc = hipGetLastError() == hipSuccess ? NEO_HIP_OK : fail(NEO_HIP_ERUNTIME, "pack kernel launch failed");
    if (!rc) rc = reset_state(h, h->stream);
    if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    if (tmp) (void)hipFree(tmp);
    return rc;
}

NEO_HIP_API int neo_hip_upols_set_impulse(neo_hip_upols* h, const float* ir, int64_t length, int normalize,
                                          int is_device)
{
    if (!h || !ir || length < 1) return fail(NEO_HIP_EINVAL, "null handle/ir or empty impulse");
    if (partitions_for(length, h->B) != h->P)
        return fail(NEO_HIP_EINVAL, "impulse of %lld taps gives %lld partitions, convolver has %d", (long long)length,
                    (long long)partitions_for(length, h->B), h->P);
    device_guard g(h->device);
    if (g.rc) return g.rc;
    NEO_HIP_CHECK(hipDeviceSynchronize());  // setup calls order after all prior work, any stream
    const size_t bytes = size_t(h->C) * size_t(length) * sizeof(float);
    float* d = nullptr;
    NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d), bytes));
    int rc = NEO_HIP_OK;
    if (hipMemcpyAsync(d, ir, bytes, is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream) !=
        hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "impulse copy failed");
    if (!rc && normalize) rc = normalize_device(d, h->C, length, h->stream);
    if (!rc) rc = partition_device(d, h->C, length, h->B, true, h->H, h->tw, h->stream, h->cstride, h->pstride);
    if (!rc) rc = reset_state(h, h->stream);
    if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    (void)hipFree(d);
    return rc;
}

NEO_HIP_API int neo_hip_upols_process_device(neo_hip_upols* h, const float* in, int64_t ld_in, float* out,
                                             int64_t ld_out, void* stream)
{
    if (!h || !in || !out) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (ld_in < h->B || ld_out < h->B) return fail(NEO_HIP_EINVAL, "leading dimension smaller than the block");
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15 || (ld_in | ld_out) & 3)
        return fail(NEO_HIP_EINVAL, "device I/O must be 16-byte aligned (ld multiple of 4)");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    if (h->v2) return process_samples(h, in, ld_in, out, ld_out, h->B, as_stream(stream));  // may be mid-block
    return launch_step(h, in, ld_in, out, ld_out, as_stream(stream));  // NULL = HIP null stream
}

NEO_HIP_API int neo_hip_upols_process_blocks(neo_hip_upols* h, const float* in, float* out, int64_t ld, int64_t nblocks,
                                             void* stream)
{
    if (!h || !in || !out) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (nblocks < 0 || ld < nblocks * h->B) return fail(NEO_HIP_EINVAL, "ld < nblocks * block");
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15 || ld & 3)
        return fail(NEO_HIP_EINVAL, "device I/O must be 16-byte aligned (ld multiple of 4)");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    // whole groups of T blocks per pass (batching on), the rest one block per pass
    return process_samples(h, in, ld, out, ld, nblocks * h->B, as_stream(stream));
}

NEO_HIP_API int neo_hip_upols_process(neo_hip_upols* h, float* io, int io_is_device, void* stream)
{
    if (!h || !io) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (io_is_device) return neo_hip_upols_process_device(h, io, h->B, io, h->B, stream);
    device_guard g(h->device);
    if (g.rc) return g.rc;
    hipStream_t s = stream ? as_stream(stream) : h->stream;  // host I/O: own stream unless given
    const size_t bytes = size_t(h->C) * h->B * sizeof(float);
    if (!h->io) {
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->io), bytes));
        NEO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h->io_host), bytes, hipHostMallocDefault));
    }
    std::copy(io, io + size_t(h->C) * h->B, h->io_host);
    NEO_HIP_CHECK(hipMemcpyAsync(h->io, h->io_host, bytes, hipMemcpyHostToDevice, s));
    int rc = h->v2 ? process_samples(h, h->io, h->B, h->io, h->B, h->B, s) : launch_step(h, h->io, h->B, h->io, h->B, s);
    if (rc) return rc;
    NEO_HIP_CHECK(hipMemcpyAsync(h->io_host, h->io, bytes, hipMemcpyDeviceToHost, s));
    NEO_HIP_CHECK(hipStreamSynchronize(s));
    std::copy(h->io_host, h->io_host + size_t(h->C) * h->B, io);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_process_samples(neo_hip_upols* h, const float* in, int64_t ld_in, float* out,
                                              int64_t ld_out, int64_t num_samples, int is_device, void* stream)
{
    if (!h || !in || !out) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    if (num_samples < 0 || ld_in < num_samples || ld_out < num_samples)
        return fail(NEO_HIP_EINVAL, "num_samples must be in [0, ld]");
    if (num_samples == 0) return NEO_HIP_OK;
    device_guard g(h->device);
    if (g.rc) return g.rc;
    if (is_device) return process_samples(h, in, ld_in, out, ld_out, num_samples, as_stream(stream));
    hipStream_t s = stream ? as_stream(stream) : h->stream;
    // host I/O: pinned staging (grown on demand), 1-D copies, synchronous like process()
    const size_t count = size_t(h->C) * size_t(num_samples);
    if (count > h->samples_cap) {
        (void)hipFree(h->samples_dev);
    (void)hipFree(h->part_b);
    (void)hipFree(h->tail);
        if (h->samples_host) (void)hipHostFree(h->samples_host);
        h->samples_dev = nullptr;
        h->samples_host = nullptr;
        h->samples_cap = 0;
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&h->samples_dev), count * sizeof(float)));
        NEO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h->samples_host), count * sizeof(float),
                                    hipHostMallocDefault));
        h->samples_cap = count;
    }
    for (int c = 0; c < h->C; ++c)
        std::copy(in + c * ld_in, in + c * ld_in + num_samples, h->samples_host + size_t(c) * num_samples);
    NEO_HIP_CHECK(hipMemcpyAsync(h->samples_dev, h->samples_host, count * sizeof(float), hipMemcpyHostToDevice, s));
    int rc = process_samples(h, h->samples_dev, num_samples, h->samples_dev, num_samples, num_samples, s);
    if (rc) return rc;
    NEO_HIP_CHECK(hipMemcpyAsync(h->samples_host, h->samples_dev, count * sizeof(float), hipMemcpyDeviceToHost, s));
    NEO_HIP_CHECK(hipStreamSynchronize(s));
    for (int c = 0; c < h->C; ++c)
        std::copy(h->samples_host + size_t(c) * num_samples, h->samples_host + size_t(c + 1) * num_samples,
                  out + c * ld_out);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_batch_info(neo_hip_upols* h, int* blocks_per_pass, int* splits)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (blocks_per_pass) *blocks_per_pass = h->batch ? batch_blocks(h) : 1;
    if (splits) *splits = h->batch ? h->Sb : h->S;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_batch(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    h->batch = enable != 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_timing(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    h->timing = enable != 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_timing(neo_hip_upols* h, double* mac_ms, int64_t* launches)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    device_guard g(h->device);
    for (size_t i = 0; i < h->events_used; ++i) {
        auto& e = h->events[i];
        NEO_HIP_CHECK(hipEventSynchronize(e.second));
        float ms = 0.f;
        NEO_HIP_CHECK(hipEventElapsedTime(&ms, e.first, e.second));
        h->mac_ms += ms;
        ++h->launches;
    }
    h->events_used = 0;
    if (mac_ms) *mac_ms = h->mac_ms;
    if (launches) *launches = h->launches;
    h->mac_ms = 0.0;
    h->launches = 0;
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
    if (is_device) NEO_HIP_CHECK(hipDeviceSynchronize());  // order after producers on any stream
    NEO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamDefault));
    cf* tw = nullptr;
    const float* d_ir = ir;
    float* tmp_in = nullptr;
    cf* d_out = static_cast<cf*>(out);
    int rc = upload_tw(&tw, block);
    if (!rc && !is_device) {
        if (hipMalloc(reinterpret_cast<void**>(&tmp_in), in_bytes) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&d_out), out_bytes) != hipSuccess)
            rc = fail(NEO_HIP_ENOMEM, "allocation failed");
        else if (hipMemcpyAsync(tmp_in, ir, in_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy failed");
        d_ir = tmp_in;
    }
    if (!rc) rc = partition_device(d_ir, channels, length, block, false, d_out, tw, s);
    if (!rc && !is_device && hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    if (!is_device) {
        (void)hipFree(tmp_in);
        (void)hipFree(d_out);
    }
    (void)hipFree(tw);
    (void)hipStreamDestroy(s);
    return rc;
}

NEO_HIP_API int neo_hip_normalize_impulse(float* ir, int channels, int64_t length, int is_device, int device)
{
    if (!ir || channels < 0 || length < 0) return fail(NEO_HIP_EINVAL, "bad arguments");
    if (channels == 0 || length == 0) return NEO_HIP_OK;
    device_guard g(device);
    if (g.rc) return g.rc;
    hipStream_t s = nullptr;
    if (is_device) NEO_HIP_CHECK(hipDeviceSynchronize());  // order after producers on any stream
    NEO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamDefault));
    const size_t bytes = size_t(channels) * size_t(length) * sizeof(float);
    float* d = ir;
    int rc = NEO_HIP_OK;
    if (!is_device) {
        if (hipMalloc(reinterpret_cast<void**>(&d), bytes) != hipSuccess) rc = fail(NEO_HIP_ENOMEM, "alloc failed");
        else if (hipMemcpyAsync(d, ir, bytes, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(NEO_HIP_ERUNTIME, "copy failed");
    }
    if (!rc) rc = normalize_device(d, channels, length, s);
    if (!rc && !is_device && hipMemcpyAsync(ir, d, bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "copy back failed");
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    if (!is_device && d) (void)hipFree(d);
    (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"
