// upols_levels.hip — the streaming UPOLS step (one block per call) with the same work in
// every step: time-distributed partition levels.
//
// Per bin k the convolver output is a convolution along the block axis
//   Y[t][k] = sum_{p < P} H[p][k] X[t - p][k]       (uniform_partitioned_convolver.hpp:47-65;
//                                                   fdl_index.hpp:23-36: partition p meets FDL row t - p)
// The partitions are cut into bands by level:
//   level 0   p in [0, 16)        the block step itself (its own FDL row for p = 0, rows t-15..t-1)
//   level 1   p in [16, 32)       T = 8-block windows
//   level 2   p in [32, 64)       T = 16
//   level 3   p in [64, 256)      T = 32
//   far       p in [256, P)       T = 128, by a 256-point transform along the partition axis
// A level with window T covers band [2T, b): for the blocks t_W + j (j < T) of a window its
// rows t_W + j - p are at most t_W - T - 1, so the whole window's contribution can be computed
// during the PREVIOUS window, 1/T of it per block step (1/T of the bins of every channel),
// into a slab per block of the window (double-buffered). A block step then only adds its
// slabs and the 15 newest partitions: every step does the same work, there is no window
// pass, and no step waits for one (the lookahead of round 1 ran a pass over the filter at the
// start of every 32-block window and a 0.63 ms far pass every 128 blocks).
//
// Levels 1-3 are direct Toeplitz MACs (k_lvl_toep); the far level is, per bin, a sum over
// segments q >= 2 of 128 partitions of DFT256(S_q) . DFT256(h_q) with S_q the 256 FDL rows
// t_W - (q+1) 128 ... t_W - (q-1) 128 - 1 (outputs 128..255 of the circular convolution are
// the window's 128 blocks, no wrap reaches them). S_{q+1} of window W+1 is S_q of window W, so
// each window transforms ONE new row pair per bin (segment 2) and keeps the spectra in a ring
// of NSEG slots (XF); the rest is a stream of XF . HF products (k_lvf_slice).
#include "upols_device.hpp"
#include "upols_handle.hpp"

#include <algorithm>
#include <vector>

namespace neo_hip {

// ---------------------------------------------------------------------------------------
// level plan (host; also exported for the CPU schedule test, neo_hip_upols_level_plan)
void plan_levels(int P, level_plan& lp)
{
    lp = level_plan{};
    lp.a0 = std::min(P, kLvA0);
    static constexpr int T[3] = {8, 16, 32}, A[3] = {16, 32, 64}, Bd[3] = {32, 64, kFarA};
    for (int l = 0; l < 3; ++l) {
        if (P <= A[l]) break;
        lp.T[lp.n] = T[l];
        lp.a[lp.n] = A[l];
        lp.b[lp.n] = std::min(P, Bd[l]);
        ++lp.n;
    }
    lp.nseg = P > kFarA ? (P - kFarA + kFarT - 1) / kFarT : 0;
}

// ---------------------------------------------------------------------------------------
// Toeplitz level slice: for the 16-column units [u0, u1) (unit u = channel u / gpc, columns
// 16 (u % gpc) ...), the T slabs of the window starting at ring row tw:
//   slab[c][j][k] = sum_{p = a}^{b-1} H[c][p][k] X[c][(tw + j - p) mod R][k],  j < T.
// Lanes: 16 columns x NPG partition groups of NPL partitions; a lane loads its NPL filter
// rows and the NPL + T - 1 FDL rows they meet, MACs in registers, and the groups are summed
// (shuffles in the wave, LDS across waves). 256 lanes = 256 / (16 NPG) units per workgroup.
template<int T, int NPL, int NPG>
__global__ __launch_bounds__(256) void k_lvl_toep(const cf* __restrict__ H, const cf* __restrict__ fdl,
                                                  cf* __restrict__ slab, int a, int b, int tw, int ring, int u0,
                                                  int u1, int gpc, int C, int B, int64_t cstride, int64_t pstride)
{
    static_assert(NPG >= 4 && NPG <= 16 && T % 4 == 0, "toeplitz slice geometry");
    constexpr int UPW = 256 / (16 * NPG), WPU = NPG / 4, NX = NPL + T - 1;
    __shared__ cf red[WPU > 1 ? UPW * (WPU - 1) * T * 16 : 1];
    const int t = threadIdx.x, col = t & 15, pg = (t >> 4) % NPG, us = t / (16 * NPG);
    const int wu = pg >> 2, q4 = pg & 3;  // wave of the unit, group within the wave
    const int u = u0 + int(blockIdx.x) * UPW + us;
    const bool live = u < u1;
    const int uc = live ? u : u1 - 1;
    const int c = uc / gpc, k = (uc - c * gpc) * 16 + col;
    const int pa = a + pg * NPL;
    const cf* Hc = H + int64_t(c) * cstride + k;
    const cf* Xc = fdl + int64_t(c) * cstride + k;
    cf acc[T];
#pragma unroll
    for (int j = 0; j < T; ++j) acc[j] = cf{0.f, 0.f};
    if (live && pa < b) {
        cf xr[NX], hm[NPL];
        // xr[i] = X[tw + T - 1 - pa - i]: partition pa + m meets block j at i = T - 1 - j + m
#pragma unroll
        for (int i = 0; i < NX; ++i) {
            int r = tw + T - 1 - pa - i;
            r = r < 0 ? r + ring : r;
            xr[i] = ld_nt(Xc + int64_t(r) * pstride);
        }
#pragma unroll
        for (int m = 0; m < NPL; ++m) hm[m] = pa + m < b ? ld_nt(Hc + int64_t(pa + m) * pstride) : cf{0.f, 0.f};
        // packed bin 0 = {DC, Nyquist}: two real products (hr xr, hi xi) instead of the complex one
        const bool z = k == 0;
#pragma unroll
        for (int m = 0; m < NPL; ++m) {
            const cf h = hm[m];
            const float hn = z ? 0.f : -h.y, ha = z ? h.y : h.x, hb = z ? 0.f : h.y;
#pragma unroll
            for (int j = 0; j < T; ++j) {
                const cf x = xr[T - 1 - j + m];
                acc[j].x = fmaf(h.x, x.x, fmaf(hn, x.y, acc[j].x));
                acc[j].y = fmaf(ha, x.y, fmaf(hb, x.x, acc[j].y));
            }
        }
    }
    // the 4 groups of a wave (lanes 16 apart)
#pragma unroll
    for (int j = 0; j < T; ++j) {
        acc[j].x += __shfl_xor(acc[j].x, 16);
        acc[j].y += __shfl_xor(acc[j].y, 16);
        acc[j].x += __shfl_xor(acc[j].x, 32);
        acc[j].y += __shfl_xor(acc[j].y, 32);
    }
    // every lane of a wave now holds its wave's sum; lane group q4 owns blocks j = 4 i + q4
    if constexpr (WPU > 1) {
        if (wu > 0) {
#pragma unroll
            for (int i = 0; i < T / 4; ++i) {
                cf v = acc[4 * i];
                v = q4 == 1 ? acc[4 * i + 1] : v;
                v = q4 == 2 ? acc[4 * i + 2] : v;
                v = q4 == 3 ? acc[4 * i + 3] : v;
                red[((us * (WPU - 1) + wu - 1) * T + 4 * i + q4) * 16 + col] = v;
            }
        }
        __syncthreads();
    }
    if (wu == 0 && live) {
        cf* o = slab + (int64_t(c) * T) * B + k;
#pragma unroll
        for (int i = 0; i < T / 4; ++i) {
            cf v = acc[4 * i];
            v = q4 == 1 ? acc[4 * i + 1] : v;
            v = q4 == 2 ? acc[4 * i + 2] : v;
            v = q4 == 3 ? acc[4 * i + 3] : v;
            if constexpr (WPU > 1) {
#pragma unroll
                for (int w = 1; w < WPU; ++w) {
                    const cf r = red[((us * (WPU - 1) + w - 1) * T + 4 * i + q4) * 16 + col];
                    v.x += r.x;
                    v.y += r.y;
                }
            }
            o[int64_t(4 * i + q4) * B] = v;
        }
    }
    (void)C;
}

// ---------------------------------------------------------------------------------------
// far level
constexpr int kFN = 2 * kFarT;  // partition-axis transform length

// 256-point transform of the column held by lanes (a, cp): on entry v[n2] = x[a + 16 n2], on
// exit v[k1] = X[16 k1 + a] (16-point DFTs in registers, twiddle, LDS transpose, 16-point DFTs)
template<int DIR>
__device__ __forceinline__ void col_fft(cf (&v)[16], cf* lds, const cf* tw, int a, int cp)
{
    dft<16, DIR>(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], twiddle<kFN, DIR>(tw, a * k));
#pragma unroll
    for (int k = 0; k < 16; ++k) lds[(k * 16 + a) * 16 + cp] = v[k];
    __syncthreads();
#pragma unroll
    for (int n = 0; n < 16; ++n) v[n] = lds[(a * 16 + n) * 16 + cp];
    __syncthreads();
    dft<16, DIR>(v);
}

// Segment spectra (grid C x NSEG x B/16): hf[c][s][f][k] = DFT256 over r < 128 of
// H[c][128 (s + 2) + r][k] (zero past P). Packed bin 0 holds two real sequences (DC and
// Nyquist), so its partition-axis convolution is two real convolutions: with
// Z = DFT(x_dc + i x_ny) and G = DFT(h_dc + i h_ny) the packed result's spectrum is
// Z[f] A[f] + conj(Z[-f]) Bv[f], A = (Hdc + Hny) / 2, Bv = (Hdc - Hny) / 2,
// Hdc = (G[f] + conj(G[-f])) / 2, Hny = (G[f] - conj(G[-f])) / 2i: A takes bin 0's slot,
// hf0[c][s][f] = Bv.
__global__ __launch_bounds__(256) void k_lvf_filter(const cf* __restrict__ H, cf* __restrict__ hf,
                                                    cf* __restrict__ hf0, const cf* __restrict__ twg, int B, int P,
                                                    int nseg, int64_t cstride, int64_t pstride)
{
    __shared__ cf lds[16 * 16 * 16];
    __shared__ cf z[kFN];
    __shared__ cf tw[kFN];
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int ng = B / 16, g = blockIdx.x % ng, cs = blockIdx.x / ng, s = cs % nseg, c = cs / nseg;
    const int k = g * 16 + cp;
    tw[t] = twg[t];
    __syncthreads();
    cf v[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
        const int r = a + 16 * n2, p = (s + 2) * kFarT + r;
        v[n2] = (r < kFarT && p < P) ? H[int64_t(c) * cstride + int64_t(p) * pstride + k] : cf{0.f, 0.f};
    }
    col_fft<-1>(v, lds, tw, a, cp);
    const bool b0 = g == 0;
    cf* dst = hf + (int64_t(c) * nseg + s) * kFN * B + k;
    if (b0) {  // uniform per workgroup
        if (cp == 0) {
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) z[16 * k1 + a] = v[k1];
        }
        __syncthreads();
        if (cp == 0) {
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) {
                const int f = 16 * k1 + a;
                const cf gf = v[k1], gm = cconj(z[(kFN - f) & (kFN - 1)]);
                const cf hdc = cscale(cadd(gf, gm), 0.5f);
                const cf d = cscale(csub(gf, gm), 0.5f);
                const cf hny = {d.y, -d.x};  // d / i
                v[k1] = cscale(cadd(hdc, hny), 0.5f);
                hf0[(int64_t(c) * nseg + s) * kFN + f] = cscale(csub(hdc, hny), 0.5f);
            }
        }
    }
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) dst[int64_t(16 * k1 + a) * B] = v[k1];
}

// Far slice: for the 16-column units [u0, u0 + grid / nsub) the far field of window wn
// (first block at ring row tw): ff[c][j][k], j < 128. Sub-unit sg of a unit takes segments
// s = sg * SPG ... (segment s = q - 2); segments s < nfresh are transformed from the FDL rows
// (s = 0 in steady state, all of them when the pipeline is primed) and their spectra stored
// in XF slot (wn - s - 1) mod M, the others read from it. With nsub > 1 every sub-unit
// publishes its partial spectrum and the last to arrive (agent-scope release / acquire on
// the unit's counter) sums them in sub-unit order, so the result does not depend on arrival
// order; it then runs the inverse transform and stores the window's 128 blocks.
template<int SPG>
__global__ __launch_bounds__(256) void k_lvf_slice(const cf* __restrict__ fdl, const cf* __restrict__ hf,
                                                   const cf* __restrict__ hf0, cf* __restrict__ xf,
                                                   cf* __restrict__ xf0m, cf* __restrict__ part,
                                                   int* __restrict__ cnt, cf* __restrict__ ff,
                                                   const cf* __restrict__ twg, int tw, int ring, int wn, int M,
                                                   int nseg, int nfresh, int u0, int nsub, int gpc, int C, int B,
                                                   int64_t cstride, int64_t pstride)
{
    __shared__ cf lds[16 * 16 * 16];
    __shared__ cf z[SPG][kFN];
    __shared__ cf tws[kFN];
    __shared__ int last;
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int ul = int(blockIdx.x) / nsub, sg = int(blockIdx.x) - ul * nsub;
    const int u = u0 + ul, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool b0 = g == 0;  // packed bin 0 lives in lane cp == 0 of these units
    tws[t] = twg[t];
    const int s0 = sg * SPG;
    auto slot = [&](int s) { return ((wn - s - 1) % M + M) % M; };
    const cf* X = fdl + int64_t(c) * cstride + k;
    cf acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = cf{0.f, 0.f};
    cf v[SPG][16], h[SPG][16];
    // stored spectra and filter spectra of this sub-unit's segments, all loads issued up front
#pragma unroll
    for (int i = 0; i < SPG; ++i) {
        const int s = s0 + i;
        if (s < nseg) {
            const cf* hs = hf + (int64_t(c) * nseg + s) * kFN * B + k;
            const cf* xs = xf + (int64_t(c) * M + slot(s)) * kFN * B + k;
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) {
                h[i][k1] = ld_nt(hs + int64_t(16 * k1 + a) * B);
                if (s >= nfresh) v[i][k1] = ld_nt(xs + int64_t(16 * k1 + a) * B);
            }
        }
    }
    __syncthreads();  // tws
#pragma unroll
    for (int i = 0; i < SPG; ++i) {
        const int s = s0 + i;
        if (s < nseg && s < nfresh) {  // uniform per workgroup
            // S_q[n] = X[tw - (q + 1) 128 + n], q = s + 2
            const int base = tw - (s + 3) * kFarT;
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) {
                int r = (base + a + 16 * n2) % ring;
                r = r < 0 ? r + ring : r;
                v[i][n2] = ld_nt(X + int64_t(r) * pstride);
            }
            col_fft<-1>(v[i], lds, tws, a, cp);
            cf* xs = xf + (int64_t(c) * M + slot(s)) * kFN * B + k;
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) xs[int64_t(16 * k1 + a) * B] = v[i][k1];
            if (b0) {  // bin 0's conj(Z[-f]): kept in LDS for this launch, stored for later windows
                if (cp == 0) {
#pragma unroll
                    for (int k1 = 0; k1 < 16; ++k1) z[i][16 * k1 + a] = v[i][k1];
                }
                __syncthreads();
                if (cp == 0) {
                    cf* zm = xf0m + (int64_t(c) * M + slot(s)) * kFN;
#pragma unroll
                    for (int k1 = 0; k1 < 16; ++k1) {
                        const int f = 16 * k1 + a;
                        zm[f] = cconj(z[i][(kFN - f) & (kFN - 1)]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < SPG; ++i) {
        if (s0 + i < nseg) {
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) acc[k1] = cadd(acc[k1], cmul(v[i][k1], h[i][k1]));
        }
    }
    if (b0 && cp == 0) {  // bin 0's second term conj(Z[-f]) Bv[f]
#pragma unroll
        for (int i = 0; i < SPG; ++i) {
            const int s = s0 + i;
            if (s < nseg) {
                const cf* bv = hf0 + (int64_t(c) * nseg + s) * kFN;
                const cf* zm = xf0m + (int64_t(c) * M + slot(s)) * kFN;
#pragma unroll
                for (int k1 = 0; k1 < 16; ++k1) {
                    const int f = 16 * k1 + a;
                    const cf mm = s < nfresh ? cconj(z[i][(kFN - f) & (kFN - 1)]) : zm[f];
                    acc[k1] = cadd(acc[k1], cmul(mm, bv[f]));
                }
            }
        }
    }
    if (nsub > 1) {
        cf* pp = part + int64_t(ul * nsub + sg) * (kFN * 16);
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) pp[(16 * k1 + a) * 16 + cp] = acc[k1];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int before = __hip_atomic_fetch_add(cnt + ul, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = before == nsub - 1;
        }
        __syncthreads();
        if (!last) return;  // uniform per workgroup
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(cnt + ul, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        const cf* p0 = part + int64_t(ul * nsub) * (kFN * 16);
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) acc[k1] = p0[(16 * k1 + a) * 16 + cp];
        for (int s2 = 1; s2 < nsub; ++s2) {
            const cf* ps = p0 + int64_t(s2) * (kFN * 16);
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) acc[k1] = cadd(acc[k1], ps[(16 * k1 + a) * 16 + cp]);
        }
    }
    // inverse along f: acc[k1] sits at f = a + 16 k1, the layout col_fft takes
    col_fft<1>(acc, lds, tws, a, cp);
    constexpr float sc = 1.0f / kFN;
    cf* o = ff + int64_t(c) * kFarT * B + k;
#pragma unroll
    for (int m = 8; m < 16; ++m) {  // n = 16 m + a >= 128: block j = n - 128
        const int j = 16 * (m - 8) + a;
        o[int64_t(j) * B] = cscale(acc[m], sc);
    }
    (void)C;
}

// ---------------------------------------------------------------------------------------
// Block step (grid C, 64 + NG B/2 lanes): wave 0 loads the overlap window, stores this block
// as the next call's previous block and runs the window transform (wave-synchronous Stockham);
// NG groups of B/2 lanes meanwhile sum the level slabs of this block and MAC partitions
// 1 .. a0 - 1 (rows w - p). After one barrier lane i of group 0 owns the mirror pair of bins
// (i, B - i): r2c split, FDL row w, Y = partials + H0 X, c2r join; after a second, wave 0
// runs the inverse transform and stores the block (OLS: window samples [B, 2B); OLA: first
// half + overlap).
struct lvl_in {
    const cf* p[kLvMax];  // slab of this block for channel 0
    int64_t cs[kLvMax];   // channel stride (complex)
    int n;
};

template<int B>
struct lstep_cfg {
    static constexpr int Q = B / 2;                                  // float4 (2 bins) per row
    static constexpr int NG = Q >= 768 ? 1 : (768 / Q > 6 ? 6 : 768 / Q);  // MAC groups
    static constexpr int EW = B >= 512 ? B / 64 : 8;                 // transform elements per lane
    static constexpr int TW = B / EW;                                // transform lanes (<= 64)
    static constexpr int NT = 64 + NG * Q;                           // workgroup size
    static constexpr int KC = 8;                                     // row pairs in flight per lane
};

template<int B, bool OLA>
__global__ __launch_bounds__(lstep_cfg<B>::NT) void k_upols_lvl(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, const cf* __restrict__ twg, int ring, int w, int a0,
    int64_t cstride, int64_t pstride, lvl_in lv)
{
    using K = upols_cfg<B>;
    using A = lstep_cfg<B>;
    constexpr int Q = A::Q, NG = A::NG, EW = A::EW, TW = A::TW, KC = A::KC;
    static_assert(TW <= 64 && A::NT <= 1024 && EW % 2 == 0, "block step geometry");
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
    const int i0 = tid - 64, k0 = i0, k1 = i0 == 0 ? B / 2 : B - i0;
    cf h0a = {0.f, 0.f}, h0b = h0a;
    if (tid >= 64 && tid < 64 + Q) {
        h0a = H[crow + k0];
        h0b = H[crow + k1];
    }
    if (tid < 64) {  // wave 0: window r2c, previous block
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
                // the window's second half becomes the next call's first half, stored from
                // registers; the lane read prev_c[n] in an earlier load of the same wave
                cf* pw = reinterpret_cast<cf*>(prev_c);
#pragma unroll
                for (int m = EW / 2; m < EW; ++m) pw[tid + m * TW - B / 2] = v[m];
            }
        }
        twr.store(tw, tid);
        wave_sync();
        stockham<B, EW, -1, 1, true>(v, fft, tw, tid, tid < TW);
        if (tid < TW) {
#pragma unroll
            for (int m = 0; m < EW; ++m) fft[lpad(tid + m * TW)] = v[m];
        }
    } else {  // MAC groups: level slabs + partitions 1 .. a0 - 1
        const int u = tid - 64, g = u / Q, q = u - g * Q;
        const float4* F4 = reinterpret_cast<const float4*>(fdl + crow);
        float4 sum = {0.f, 0.f, 0.f, 0.f};
        for (int l = g; l < lv.n; l += NG) {
            const float4 r = reinterpret_cast<const float4*>(lv.p[l] + int64_t(c) * lv.cs[l])[q];
            sum.x += r.x; sum.y += r.y; sum.z += r.z; sum.w += r.w;
        }
        acc4 a0v = {0.f, 0.f, 0.f, 0.f}, a1v = a0v;
        for (int pb = 1 + g; pb < a0; pb += NG * KC) {
            float4 hv[KC], xv[KC];
#pragma unroll
            for (int kk = 0; kk < KC; ++kk) {
                const int p = pb + kk * NG;
                if (p < a0) {
                    const int r = w - p < 0 ? w - p + ring : w - p;
                    hv[kk] = H4[int64_t(p) * ps4 + q];
                    xv[kk] = F4[int64_t(r) * ps4 + q];
                }
            }
#pragma unroll
            for (int kk = 0; kk < KC; ++kk)
                if (pb + kk * NG < a0) mac2(a0v, a1v, hv[kk], xv[kk]);
        }
        const cf b0 = finish(a0v, q == 0), b1 = finish(a1v, false);
        acc[g][q] = make_float4(sum.x + b0.x, sum.y + b0.y, sum.z + b1.x, sum.w + b1.y);
    }
    __syncthreads();
    if (tid >= 64 && tid < 64 + Q) {
        // group 0, bin pair (k0, k1): r2c split of the window transform, FDL row w, Y = the
        // groups' partial sums + H0 X, then the c2r join; w(B - k) = -conj(w(k))
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
    if (tid < 64) c2r_tail<B, OLA, EW, true, true>(X, fft, tw, out + int64_t(c) * ld_out, prev_c, tid);
}

// ---------------------------------------------------------------------------------------
// host side

int lvl_setup(upols_t* h)
{
    plan_levels(h->P, h->lv);
    return NEO_HIP_OK;
}

// device buffers of the level pipeline (allocated on the first streaming step), all or none
static int lvl_buffers(upols_t* h)
{
    if (h->lv_ready) return NEO_HIP_OK;
    const level_plan& lp = h->lv;
    const size_t C = size_t(h->C), B = size_t(h->B);
    std::vector<void**> got;
    auto alloc = [&](void** p, size_t bytes) {
        if (hipMalloc(p, bytes) != hipSuccess) return false;
        got.push_back(p);
        return true;
    };
    auto undo = [&](const char* what, size_t bytes) {
        for (void** p : got) {
            (void)hipFree(*p);
            *p = nullptr;
        }
        return fail(NEO_HIP_ENOMEM, "level pipeline: allocation of %s (%zu bytes) failed", what, bytes);
    };
    for (int l = 0; l < lp.n; ++l) {
        const size_t bytes = 2 * C * size_t(lp.T[l]) * B * sizeof(cf);
        if (!alloc(reinterpret_cast<void**>(&h->lv_slab[l]), bytes)) return undo("level slabs", bytes);
    }
    if (lp.nseg) {
        const int M = lp.nseg, U = h->C * (h->B / 16);
        const int upw = (U + kFarT - 1) / kFarT;  // units per steady-state slice
        const int nsub = (lp.nseg + kFarSPG - 1) / kFarSPG;
        const size_t spec = C * size_t(lp.nseg) * kFN * B * sizeof(cf);
        const size_t xfb = C * size_t(M) * kFN * B * sizeof(cf);
        const size_t partb = size_t(upw) * nsub * kFN * 16 * sizeof(cf);
        if (!alloc(reinterpret_cast<void**>(&h->fv_hf), spec)) return undo("far segment spectra", spec);
        if (!alloc(reinterpret_cast<void**>(&h->fv_hf0), C * lp.nseg * kFN * sizeof(cf)))
            return undo("far bin-0 spectra", C * lp.nseg * kFN * sizeof(cf));
        if (!alloc(reinterpret_cast<void**>(&h->fv_xf), xfb)) return undo("far FDL spectra", xfb);
        if (!alloc(reinterpret_cast<void**>(&h->fv_xf0m), C * M * kFN * sizeof(cf)))
            return undo("far bin-0 FDL spectra", C * M * kFN * sizeof(cf));
        if (!alloc(reinterpret_cast<void**>(&h->fv_ff), 2 * C * kFarT * B * sizeof(cf)))
            return undo("far field", 2 * C * kFarT * B * sizeof(cf));
        if (!alloc(reinterpret_cast<void**>(&h->fv_part), partb)) return undo("far partials", partb);
        if (!alloc(reinterpret_cast<void**>(&h->fv_cnt), size_t(upw) * sizeof(int)))
            return undo("far counters", size_t(upw) * sizeof(int));
        if (!alloc(reinterpret_cast<void**>(&h->fv_tw), kFN * sizeof(cf))) return undo("far twiddles", kFN * sizeof(cf));
        const auto t = make_twiddle_table(kFN);
        NEO_HIP_CHECK(hipMemcpy(h->fv_tw, t.data(), kFN * sizeof(cf), hipMemcpyHostToDevice));
        NEO_HIP_CHECK(hipMemset(h->fv_cnt, 0, size_t(upw) * sizeof(int)));
        h->fv_nsub = nsub;
        h->fv_dirty = true;
    }
    h->lv_ready = true;
    return NEO_HIP_OK;
}

void lvl_free(upols_t* h)
{
    for (auto& p : h->lv_slab) {
        (void)hipFree(p);
        p = nullptr;
    }
    for (cf** p : {&h->fv_hf, &h->fv_hf0, &h->fv_xf, &h->fv_xf0m, &h->fv_ff, &h->fv_part, &h->fv_tw}) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    (void)hipFree(h->fv_cnt);
    h->fv_cnt = nullptr;
    h->lv_ready = false;
}

// the filter changed: the far segment spectra are recomputed before the next streaming step
void lvl_filter_changed(upols_t* h)
{
    h->fv_dirty = true;
    h->lv_n = -1;
}

static int launch_toep(const upols_t* h, int l, int tw, int u0, int u1, int buf, hipStream_t s)
{
    const level_plan& lp = h->lv;
    const int T = lp.T[l], gpc = h->B / 16;
    cf* slab = h->lv_slab[l] + size_t(buf) * h->C * T * h->B;
#define NEO_TOEP(TT, NPL, NPG)                                                                                   \
    {                                                                                                            \
        constexpr int UPW = 256 / (16 * NPG);                                                                    \
        const unsigned grid = unsigned((u1 - u0 + UPW - 1) / UPW);                                               \
        hipLaunchKernelGGL((k_lvl_toep<TT, NPL, NPG>), dim3(grid), dim3(256), 0, s, h->H, h->fdl, slab, lp.a[l], \
                           lp.b[l], tw, h->ring, u0, u1, gpc, h->C, h->B, h->cstride, h->pstride);               \
    }
    switch (T) {
        case 8: NEO_TOEP(8, 4, 4) break;
        case 16: NEO_TOEP(16, 4, 8) break;
        case 32: NEO_TOEP(32, 12, 16) break;
        default: return fail(NEO_HIP_EINVAL, "no Toeplitz level of %d blocks", T);
    }
#undef NEO_TOEP
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

static int launch_far(const upols_t* h, int tw, int wn, int u0, int u1, int nfresh, hipStream_t s)
{
    const level_plan& lp = h->lv;
    const int nsub = h->fv_nsub;
    cf* ff = h->fv_ff + size_t(wn & 1) * h->C * kFarT * h->B;
    const unsigned grid = unsigned(u1 - u0) * unsigned(nsub);
    hipLaunchKernelGGL((k_lvf_slice<kFarSPG>), dim3(grid), dim3(256), 0, s, h->fdl, h->fv_hf, h->fv_hf0, h->fv_xf,
                       h->fv_xf0m, h->fv_part, h->fv_cnt, ff, h->fv_tw, tw, h->ring, wn, lp.nseg, lp.nseg, nfresh, u0,
                       nsub, h->B / 16, h->C, h->B, h->cstride, h->pstride);
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

// First streaming step after a reset / filter change / batched pass: window 0 of every level
// starts at this block; compute it whole (all units; the far level transforms every segment).
static int lvl_prime(upols_t* h, hipStream_t s)
{
    const level_plan& lp = h->lv;
    int rc;
    if (lp.nseg && h->fv_dirty) {
        const unsigned grid = unsigned(h->C) * unsigned(lp.nseg) * unsigned(h->B / 16);
        hipLaunchKernelGGL(k_lvf_filter, dim3(grid), dim3(256), 0, s, h->H, h->fv_hf, h->fv_hf0, h->fv_tw, h->B, h->P,
                           lp.nseg, h->cstride, h->pstride);
        NEO_HIP_LAUNCH_CHECK();
        h->fv_dirty = false;
    }
    const int U = h->C * (h->B / 16);
    for (int l = 0; l < lp.n; ++l)
        if ((rc = launch_toep(h, l, h->wpos, 0, U, 0, s))) return rc;
    if (lp.nseg) {
        // in slices of the steady-state size (the partial buffer holds one slice)
        for (int st = 0; st < kFarT; ++st) {
            const int u0 = int(int64_t(st) * U / kFarT), u1 = int(int64_t(st + 1) * U / kFarT);
            if (u1 > u0 && (rc = launch_far(h, h->wpos, 0, u0, u1, lp.nseg, s))) return rc;
        }
    }
    return NEO_HIP_OK;
}

int launch_levels(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s)
{
    int rc = lvl_buffers(h);
    if (rc) return rc;
    const level_plan& lp = h->lv;
    if (h->lv_n < 0) {
        if ((rc = lvl_prime(h, s))) return rc;
        h->lv_n = 0;
    }
    const int64_t n = h->lv_n;
    const int B = h->B, C = h->C, R = h->ring, U = C * (B / 16);
    lvl_in li{};
    for (int l = 0; l < lp.n; ++l) {
        const int T = lp.T[l];
        const int64_t buf = (n / T) & 1, j = n % T;
        li.p[li.n] = h->lv_slab[l] + (buf * C * T + j) * B;
        li.cs[li.n] = int64_t(T) * B;
        ++li.n;
    }
    if (lp.nseg) {
        const int64_t buf = (n / kFarT) & 1, j = n % kFarT;
        li.p[li.n] = h->fv_ff + (buf * C * kFarT + j) * B;
        li.cs[li.n] = int64_t(kFarT) * B;
        ++li.n;
    }
    upols_t::ev_group* ev = nullptr;
    if ((rc = timing_begin(h, 4, &ev)) || (rc = timing_mark(ev, 0, s))) return rc;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(B, if constexpr (BB <= 1024) hipLaunchKernelGGL(
                                  (k_upols_lvl<BB, true>), dim3(unsigned(C)), dim3(lstep_cfg<BB>::NT), 0, s, in, ld_in,
                                  out, ld_out, h->prev, h->H, h->fdl, h->tw, R, h->wpos, lp.a0, h->cstride, h->pstride, li))
    } else {
        NEO_UPOLS_DISPATCH(B, if constexpr (BB <= 1024) hipLaunchKernelGGL(
                                  (k_upols_lvl<BB, false>), dim3(unsigned(C)), dim3(lstep_cfg<BB>::NT), 0, s, in, ld_in,
                                  out, ld_out, h->prev, h->H, h->fdl, h->tw, R, h->wpos, lp.a0, h->cstride, h->pstride, li))
    }
    NEO_HIP_LAUNCH_CHECK();
    if ((rc = timing_mark(ev, 1, s))) return rc;
    // 1/T of the next window of every level (rows <= this block - 1 only)
    for (int l = 0; l < lp.n; ++l) {
        const int T = lp.T[l], st = int(n % T);
        const int u0 = int(int64_t(st) * U / T), u1 = int(int64_t(st + 1) * U / T);
        if (u1 <= u0) continue;
        const int tw = ((h->wpos - st + T) % R + R) % R;
        if ((rc = launch_toep(h, l, tw, u0, u1, int(((n / T) + 1) & 1), s))) return rc;
    }
    if ((rc = timing_mark(ev, 2, s))) return rc;
    if (lp.nseg) {
        const int st = int(n % kFarT);
        const int u0 = int(int64_t(st) * U / kFarT), u1 = int(int64_t(st + 1) * U / kFarT);
        if (u1 > u0) {
            const int tw = ((h->wpos - st + kFarT) % R + R) % R;
            if ((rc = launch_far(h, tw, int(n / kFarT + 1), u0, u1, 1, s))) return rc;
        }
    }
    if ((rc = timing_mark(ev, 3, s))) return rc;
    h->wpos = h->wpos + 1 >= R ? 0 : h->wpos + 1;
    h->lv_n = n + 1;
    return NEO_HIP_OK;
}

}  // namespace neo_hip

// The level plan of a (block, partitions) convolver, for tests of the schedule: a0 = the
// block step's partitions, then per level its window and band [a, b); nseg far segments.
extern "C" NEO_HIP_API int neo_hip_upols_level_plan(int partitions, int* a0, int* nlevels, int* T, int* a, int* b,
                                                    int* nseg)
{
    if (partitions < 1) return neo_hip::fail(NEO_HIP_EINVAL, "partitions must be >= 1");
    neo_hip::level_plan lp;
    neo_hip::plan_levels(partitions, lp);
    if (a0) *a0 = lp.a0;
    if (nlevels) *nlevels = lp.n;
    for (int l = 0; l < lp.n; ++l) {
        if (T) T[l] = lp.T[l];
        if (a) a[l] = lp.a[l];
        if (b) b[l] = lp.b[l];
    }
    if (nseg) *nseg = lp.nseg;
    return NEO_HIP_OK;
}
