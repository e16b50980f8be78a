// upols_levels.hip — the streaming UPOLS step (one block per call) with the same work in
// every step: time-distributed partition levels, all in ONE launch per block.
//
// Per bin k the convolver output is a convolution along the block axis
//   Y[t][k] = sum_{p < P} H[p][k] X[t - p][k]       (uniform_partitioned_convolver.hpp:47-65;
//                                                   fdl_index.hpp:23-36: partition p meets FDL row t - p)
// The partitions are cut into bands (plan_levels):
//   p in [0, 8)                   the block itself (its own FDL row and 7 older ones)
//   Toeplitz  [8, 16) [16, 32) [32, 64) [64, 256): windows of T = 4, 8, 16, 32 blocks
//   far       p in [256, P)       T = 128, by a 256-point transform along the partition axis
// A level with window T covers a band starting at 2T: for the blocks t_W + j (j < T) of a
// window its rows t_W + j - p are at most t_W - T - 1, so the whole window's contribution can
// be computed during the PREVIOUS window, 1/T of it per step (a slice of the columns of every
// channel), into a slab per block of the window (double-buffered). The step kernel
// (k_lvl_step) runs the block and those slices side by side; no role reads what another role
// of the same launch writes (see k_lvl_step). Round 1 instead ran a pass over the filter at
// the start of every 32-block window and a 0.63 ms far pass every 128 blocks.
//
// The far level is, per bin, a sum over segments q >= 2 of 128 partitions of
// DFT256(S_q) . DFT256(h_q) with S_q the 256 FDL rows t_W - (q+1) 128 ... t_W - (q-1) 128 - 1
// (outputs 128..255 of the circular convolution are the window's 128 blocks, no wrap reaches
// them). S_{q+1} of window W+1 is S_q of window W, so each window transforms ONE new row
// pair per bin (segment 2) and keeps the spectra in a ring of NSEG slots (XF); the rest is a
// stream of XF . HF products (far1_role / far2_role).
#include "upols_device.hpp"
#include "upols_handle.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

namespace neo_hip {

// timeline builds: thread 0 stamps the workgroup's mid-point (a role's loads landed)
#ifdef NEO_TIMELINE
#define NEO_TL_MARK(a)                                                                                 \
    do {                                                                                               \
        if (threadIdx.x == 0 && (a).tl)                                                                \
            static_cast<unsigned long long*>((a).tl)[4 * int64_t(blockIdx.x) + 3] = wall_clock64();    \
    } while (0)
#else
#define NEO_TL_MARK(a) \
    do {               \
    } while (0)
#endif
// latency-mode probe builds (NEO_PS_PROBE): thread 0 stamps point i of the block role into a.tl
#ifdef NEO_PS_PROBE
#define NEO_PS_MARK(a, i)                                                                              \
    do {                                                                                               \
        if (threadIdx.x == 0 && (a).tl)                                                                \
            static_cast<unsigned long long*>((a).tl)[i] = wall_clock64(); /* plain: no wait added */  \
    } while (0)
#else
#define NEO_PS_MARK(a, i) \
    do {                  \
    } while (0)
#endif


// ---------------------------------------------------------------------------------------
// level plan (host; also exported for the CPU schedule test, neo_hip_upols_level_plan)
void plan_levels(int P, level_plan& lp, int far)
{
    lp = level_plan{};
    lp.a0 = std::min(P, kLvA0);
    static constexpr int T[4] = {4, 8, 16, 32}, A[4] = {8, 16, 32, 64}, Bd[4] = {16, 32, 64, kFarA};
    for (int l = 0; l < 4; ++l) {
        if (P <= A[l]) break;
        lp.T[lp.n] = T[l];
        lp.a[lp.n] = A[l];
        lp.b[lp.n] = std::min(P, Bd[l]);
        ++lp.n;
    }
    if (P <= kFarA) return;
    if (far != 0) {
        lp.nseg = (P - kFarA + kFarT - 1) / kFarT;
    } else {  // [256, P) by the big Toeplitz level (slot 4)
        lp.T[lp.n] = kBigT;
        lp.a[lp.n] = 2 * kBigT;
        lp.b[lp.n] = P;
        ++lp.n;
    }
}

// ---------------------------------------------------------------------------------------
// device helpers

constexpr int kFN = 2 * kFarT;  // far level: partition-axis transform length

// Channel strides (complex units) of the level buffers: kPad rows more than the data, so that no
// channel stride is a multiple of a large power of two -- every channel's row n of a slab, of the
// far field or of a segment spectrum would otherwise sit at the same offset modulo 512 KB .. 8 MB
// (an FDL ring of 1280 rows, 5 x 2^20 bytes per channel at B = 512, cost the c5full step 4 %)
#ifndef NEO_PAD
#define NEO_PAD 1  // diagnostic builds (A/B): 0 = unpadded strides
#endif
constexpr int kPad = NEO_PAD;
__host__ __device__ constexpr int64_t slab_cs(int T, int B) { return int64_t(T + kPad) * B; }
__host__ __device__ constexpr int64_t ff_cs(int B) { return int64_t(kFarT + kPad) * B; }
__host__ __device__ constexpr int64_t spec_cs(int nseg, int B) { return (int64_t(nseg) * kFN + kPad) * B; }

// 256-point transforms of NC columns held by lanes (a, cp), a < 16, cp < NC: on entry
// v[n2] = x[a + 16 n2], on exit v[k1] = X[16 k1 + a] (16-point DFTs in registers, twiddle,
// LDS transpose, 16-point DFTs). Every lane of the workgroup calls it (barriers inside);
// lanes with active = false only take part in the barriers.
template<int DIR, int NC>
__device__ __forceinline__ void col_fft(cf (&v)[16], cf* lds, const cf* tw, int a, int cp, bool active)
{
    if (active) {
        dft<16, DIR>(v);
#pragma unroll
        for (int k = 1; k < 16; ++k) v[k] = cmul(v[k], twiddle<kFN, DIR>(tw, a * k));
#pragma unroll
        for (int k = 0; k < 16; ++k) lds[(k * 16 + a) * NC + cp] = v[k];
    }
    __syncthreads();
    if (active) {
#pragma unroll
        for (int n = 0; n < 16; ++n) v[n] = lds[(a * 16 + n) * NC + cp];
    }
    __syncthreads();
    if (active) dft<16, DIR>(v);
}

// packed complex MAC: acc = (re, im) += h x as (hr, hr)(xr, xi) + (-hi, hi)(xi, xr), two
// v_pk_fma_f32; the packed bin 0 (DC, Nyquist: two real products) takes (hr, hi)(xr, xi)
struct pk_coef {
    f2v h1, h2;
    __device__ __forceinline__ pk_coef(cf h, bool bin0)
    {
        const float s = bin0 ? 0.f : h.y;
        h1 = f2v{h.x, bin0 ? h.y : h.x};
        h2 = f2v{-s, s};
    }
    __device__ __forceinline__ void mac(f2v& acc, cf x) const
    {
        const f2v xv = {x.x, x.y};
        acc = __builtin_elementwise_fma(h1, xv, acc);
        acc = __builtin_elementwise_fma(h2, xv.yx, acc);
    }
};

// ---------------------------------------------------------------------------------------
// The per-step slices kernel: one launch after every block step, workgroups by role.
//   rest      the next block's spectrum without partition 0: its partitions 1 .. a0 - 1
//             (rows up to this block's) plus the level slabs of the next block
//   Toeplitz  1/T of the next window of each Toeplitz level (a slice of its columns)
//   far       1/128 of the next far window (a slice of its 8-column units)
// Every role reads FDL rows up to this step's block only; the block step of the next call
// then needs nothing but its window, this spectrum and H0.
struct toep_arg {
    cf* slab;           // the target window's slabs [C][T][B]
    int T, a, b;        // window, band [a, b)
    int tw;             // ring row of the window's first block
    int u0, u1, nwg;    // units (16 columns x one of JH window parts) of this slice, workgroups
    int jh;             // window parts per column group (toep_geom)
    int64_t cs;         // the slab's channel stride (slab_cs)
};

struct slice_args {
    const cf* H;
    cf* fdl;
    int ring, C, B;
    int64_t cstride, pstride;
    // block role: this step's block, one workgroup per channel (nblk = 0 in priming launches)
    // from channel blk_c0 on
    int nblk, blk_c0;
    const float* in;
    int64_t ld_in;
    float* out;
    int64_t ld_out;
    float* prev;
    float* snap;            // not null: a copy of each channel's input block, [C][B] (upols_group.hip: the
                            // frame the leader's launch read in place, for the later members' comparisons)
    const cf* twg;
    int w, a0;              // ring row of the block; partitions the block role MACs directly
    int nsl;
    const cf* sl[kLvToep];  // slab row of this block per level, channel 0
    int64_t scs[kLvToep];   // channel strides
    const cf* ff;           // far field row of this block, channel 0 (null: no far level)
    int64_t fcs;
    // Toeplitz roles
    int ntp;
    toep_arg tp[kLvToep];
    // far level (16-column units), common
    int M, nseg, fnfresh, P;
    int64_t fsc;  // segment / row-pair spectra channel stride (spec_cs; M = nseg slots)
    const cf* hf;
    cf* xf;
    const cf* twf;
    int fU;     // units (16 columns) of all channels
    // far phase 1: stored-segment MAC, groups of kF1UG units; in pair mode a group takes two
    // windows at once (far1_role)
    int f1nwg, f1u0, f1u1, f1wn, f1fpl;  // slice units [f1u0, f1u1); target window; f rows per lane
    int fK;                              // windows per phase-1 pass (1: one window per pass)
    int f1g0, f1gs, f1mode, f1cls;       // first group, group step; 0 single, 1 the class's groups, 2 every group; class
    cf* f1acc;  // partial sums [fK (window mod fK)][fU][256 f][16]
    // far phase 2a (the slice phase 1 takes in the same launch): the fresh row pairs'
    // transforms, stored to their ring slots
    int f2nwg, f2u0, f2tw, f2wn;
    // far phase 2b (the slice of the previous launch): the stored fresh spectra's products,
    // phase 1's partial sums, the window group's extra segments, the inverse transform
    int f3nwg, f3u0, f3wn;
    int f2grp;    // phase-1 window groups on: a unit in window j of its group takes segments 1..j in 2b
    int f2comb;   // 1: 2b also runs 2a's fresh transform for its units (f2tw: its rows), no slot read-back (far2c_role);
                  // 2: the recomputed far level (far2r_role, every segment from the filter and FDL rows)
    cf* f2acc;    // as f1acc
    cf* f3ff;     // 2b's target far window [C][128][B]
    void* tl;     // timeline builds (NEO_TIMELINE): per-workgroup records of the launch
    int bid0;     // paced background pieces: the first workgroup of the launch this piece runs
};

// the T = 32 Toeplitz level stages its band in LDS: filter rows [64, 256) and the FDL rows
// they meet, 16 columns each, column-major with padded strides
constexpr int kT32Band = 192;                                       // [64, 256)
constexpr int kFarLds = (16 * 16 * 16 + 2 * 256 + 8 * 256) * int(sizeof(cf));  // far roles: transposes, bin-0 exchange,
                                                                               // twiddles, far2r_role's half pair
// toep_tile<32, 192>: 53760 B, 3 workgroups per CU (VGPRs allow 3 too; the band in two chunks
// of 96, 29184 B, with a 128-VGPR budget for 4 per CU measured slower: spills, serialized chunks)
constexpr int kT32Lds = 16 * ((kT32Band + 2) + (kT32Band + 34)) * int(sizeof(cf));
constexpr int kSliceLds = kFarLds > kT32Lds ? kFarLds : kT32Lds;

// Block role (lanes 0 .. B/2 - 1 of the workgroup, the others idle): lane i gathers, for the
// mirror pair of bins (i, B - i), everything but partition 0 -- partitions 1 .. a0 - 1 (FDL
// rows of the previous blocks), the level slabs and the far field of this block (their
// windows finished in earlier launches) -- and loads H0; with those loads in flight wave 0
// loads the overlap window, stores this block as the next call's previous block and runs the
// window transform (wave-synchronous Stockham). After one barrier the pair lanes run the r2c
// split, insert FDL row w, form Y = rest + H0 X and the c2r join; after a second, wave 0 runs
// the inverse transform and stores the block (OLS: window samples [B, 2B); OLA: first half +
// overlap).
template<int B>
struct lstep_cfg {
    static constexpr int Q = B / 2;                   // bin pairs
    // transform elements per lane: 64 transform lanes from B = 256 on (B = 256 with 8 elements on 32
    // lanes: C4's block launch 12.5 -> 11.1 us per step in a same-box A/B at 4 on 64)
    static constexpr int EW = B >= 256 ? B / 64 : 8;
    static constexpr int TW = B / EW;                 // transform lanes (<= 64)
    static constexpr int NT = Q > 64 ? Q : 64;        // lanes of the role
    static constexpr int WG = NT > 256 ? NT : 256;    // workgroup size of the step kernel
};

// y += h x; the packed bin 0 ({DC, Nyquist}) takes two real products
__device__ __forceinline__ void cmac(cf& y, cf h, cf x, bool bin0)
{
    if (bin0) {
        y.x = fmaf(h.x, x.x, y.x);
        y.y = fmaf(h.y, x.y, y.y);
    } else {
        y.x = fmaf(h.x, x.x, fmaf(-h.y, x.y, y.x));
        y.y = fmaf(h.x, x.y, fmaf(h.y, x.x, y.y));
    }
}

template<int B, bool OLA, bool WT = false>
__device__ __forceinline__ void block_role(const slice_args& a, int c, char* smem)
{
    using K = upols_cfg<B>;
    using A = lstep_cfg<B>;
    constexpr int EW = A::EW, TW = A::TW;
    static_assert(TW <= 64 && A::NT <= 1024 && EW % 2 == 0, "block step geometry");
    cf* X = reinterpret_cast<cf*>(smem);
    cf* fft = X + B;
    cf* tw = fft + K::LL;
    const int tid = threadIdx.x;
    const int64_t crow = int64_t(c) * a.cstride;
    const float* in_c = a.in + int64_t(c) * a.ld_in;
    float* prev_c = a.prev + int64_t(c) * B;
    const int k0 = tid, k1 = tid == 0 ? B / 2 : B - tid;
    const bool pair = tid < A::Q;
    cf h0a = {0.f, 0.f}, h0b = h0a, ra = h0a, rb = h0a;
    // wave 0 issues its window loads first: its transform waits for them only, not for the
    // bin-pair loads it issues next (loads return in order)
    tw_regs<K::TW1 + K::TW2, 64> twr;
    cf v[EW];
    if (tid < 64) {
        twr.load(a.twg, tid);
        if (tid < TW) {
            const cf* pz = reinterpret_cast<const cf*>(prev_c);
            const cf* iz = reinterpret_cast<const cf*>(in_c);
            // WT (latency mode): the caller's block read at system scope, past every cache (another
            // kernel or the host may have rewritten it since this persistent kernel last read there)
            auto in_ld = [&](int i) {
                if constexpr (WT)
                    return __builtin_bit_cast(cf, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(iz + i),
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
                else return iz[i];
            };
#pragma unroll
            for (int m = 0; m < EW; ++m) {
                const int n = tid + m * TW;
                if constexpr (OLA) v[m] = n < B / 2 ? in_ld(n) : cf{0.f, 0.f};
                else v[m] = n < B / 2 ? pz[n] : in_ld(n - B / 2);
            }
            if (a.snap) {  // the input block as read (uniform per launch)
                cf* sz = reinterpret_cast<cf*>(a.snap + int64_t(c) * B);
#pragma unroll
                for (int m = 0; m < EW; ++m) {
                    const int n = tid + m * TW;
                    if constexpr (OLA) {
                        if (n < B / 2) sz[n] = v[m];
                    } else {
                        if (n >= B / 2) sz[n - B / 2] = v[m];
                    }
                }
            }
        }
    }
    cf ha[kLvA0 - 1], hb[kLvA0 - 1], xa[kLvA0 - 1], xb[kLvA0 - 1], sla[kLvToep + 1], slb[kLvToep + 1];
    if (pair) {  // loads only; the sums follow the transform
        h0a = a.H[crow + k0];
        h0b = a.H[crow + k1];
#pragma unroll
        for (int p = 1; p < kLvA0; ++p) {
            if (p < a.a0) {
                const int r = a.w - p < 0 ? a.w - p + a.ring : a.w - p;
                ha[p - 1] = a.H[crow + int64_t(p) * a.pstride + k0];
                hb[p - 1] = a.H[crow + int64_t(p) * a.pstride + k1];
                xa[p - 1] = a.fdl[crow + int64_t(r) * a.pstride + k0];
                xb[p - 1] = a.fdl[crow + int64_t(r) * a.pstride + k1];
            }
        }
#pragma unroll
        for (int l = 0; l < kLvToep; ++l) {
            if (l < a.nsl) {
                const cf* sr = a.sl[l] + int64_t(c) * a.scs[l];
                sla[l] = sr[k0];
                slb[l] = sr[k1];
            }
        }
        if (a.ff) {
            sla[kLvToep] = a.ff[int64_t(c) * a.fcs + k0];
            slb[kLvToep] = a.ff[int64_t(c) * a.fcs + k1];
        }
    }
    if (tid < 64) {  // wave 0: previous block, window r2c
        if constexpr (!OLA) {
            if (tid < TW) {
                // the window's second half becomes the next call's first half, stored from
                // registers; the lane read prev_c[n] in an earlier load of the same wave
                cf* pw = reinterpret_cast<cf*>(prev_c);
#pragma unroll
                for (int m = EW / 2; m < EW; ++m) pw[tid + m * TW - B / 2] = v[m];
            }
        }
        twr.store(tw, tid);
        wave_sync();
        NEO_PS_MARK(a, 1);  // wave 0 issued its loads and stored the previous block
        stockham<B, EW, -1, 1, true>(v, fft, tw, tid, tid < TW);
        NEO_PS_MARK(a, 2);  // r2c done (the window's loads had landed)
        if (tid < TW) {
#pragma unroll
            for (int m = 0; m < EW; ++m) fft[lpad(tid + m * TW)] = v[m];
        }
    }
    if (pair) {
#pragma unroll
        for (int l = 0; l < kLvToep; ++l) {
            if (l < a.nsl) {
                ra = cadd(ra, sla[l]);
                rb = cadd(rb, slb[l]);
            }
        }
        if (a.ff) {
            ra = cadd(ra, sla[kLvToep]);
            rb = cadd(rb, slb[kLvToep]);
        }
#pragma unroll
        for (int p = 1; p < kLvA0; ++p) {
            if (p < a.a0) {
                cmac(ra, ha[p - 1], xa[p - 1], k0 == 0);
                cmac(rb, hb[p - 1], xb[p - 1], false);
            }
        }
    }
    __syncthreads();
    NEO_TL_MARK(a);
    NEO_PS_MARK(a, 3);  // every pair lane's loads landed
    if (pair) {
        // bin pair (k0, k1): r2c split, FDL row w, Y = rest + H0 X, c2r join; w(B - k) = -conj(w(k))
        const cf wa = k0 == 0 ? cf{1.f, 0.f} : twiddle<2 * B, -1>(tw + K::TW1, k0);
        const cf wb = k0 == 0 ? cf{0.f, -1.f} : cf{-wa.x, wa.y};
        const cf xa = r2c_split_w<B>(fft, wa, k0), xb = r2c_split_w<B>(fft, wb, k1);
        cf* row = a.fdl + crow + int64_t(a.w) * a.pstride;
        row[k0] = xa;
        row[k1] = xb;
        cf ya = ra, yb = rb;
        cmac(ya, h0a, xa, k0 == 0);
        cmac(yb, h0b, xb, false);
        X[k0] = k0 == 0 ? c2r_join_w<B>(cf{ya.x, 0.f}, cf{ya.y, 0.f}, cf{1.f, 0.f}, 0)
                        : c2r_join_w<B>(ya, yb, cf{wa.x, -wa.y}, k0);
        X[k1] = c2r_join_w<B>(yb, k0 == 0 ? yb : ya, cf{wb.x, -wb.y}, k1);
    }
    __syncthreads();
    NEO_PS_MARK(a, 4);  // joined spectrum in LDS
    if (tid < 64) c2r_tail<B, OLA, EW, true, true, WT>(X, fft, tw, a.out + int64_t(c) * a.ld_out, prev_c, tid);
    NEO_PS_MARK(a, 5);  // output stores issued
}

// buffer loads / stores: 32-bit lane offsets, uniform offsets in SGPRs (fewer VGPRs than
// 64-bit addresses); offsets past the size read 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, int(bytes), 0x00020000);
}

__device__ __forceinline__ cf buf_ld(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    return __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 2 /* streaming */));
}

__device__ __forceinline__ void buf_st(cf v, __amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, voff, soff, 0);
}

// Toeplitz levels' filter rows: nontemporal (the default) or, NEO_H_POLICY 1, the default cache
// policy for the levels whose band ends by partition 64 (diagnostic A/B: the small bands' filter
// rows, re-read every T steps, may stay in the Infinity Cache at the 256-channel shapes)
#ifndef NEO_H_POLICY
#define NEO_H_POLICY 0
#endif
__device__ __forceinline__ cf ld_h(const cf* p, int band_end)
{
    if (NEO_H_POLICY && band_end <= 64) return *p;
    return ld_nt(p);
}

// v + v of the lane D = 16 / 32 apart (v_permlane16_swap / v_permlane32_swap, gfx950): the
// swap of v with itself leaves v and its partner in the two halves of the pair, whose sum is
// the same float sum in every lane as v + __shfl_xor(v, D)
template<int D>
__device__ __forceinline__ float xor_sum(float v)
{
    const unsigned u = __float_as_uint(v);
    if constexpr (D == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else {
        static_assert(D == 32, "lane distance 16 or 32");
        const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
}

// Toeplitz level: for the units [u0, u1) (unit u = (channel, 16 columns, block half jh)),
//   slab[c][j][k] = sum_{p = a}^{b-1} H[c][p][k] X[c][(tw + j - p) mod R][k],  j in half jh.
// Lanes: 16 columns x NPG partition groups of NPL partitions; a lane loads its NPL filter
// rows and the NPL + T/JH - 1 FDL rows they meet and MACs in registers (packed FMA); the
// groups are summed (shuffles in the wave, LDS across waves). NPG = 1: a lane takes the
// whole band of its column.
template<int T, int NPL, int NPG, int JH>
__device__ __forceinline__ void toep_role(const slice_args& sa, const toep_arg& ta, int bid, char* smem)
{
    static_assert((NPG == 1 || NPG == 4 || NPG == 8 || NPG == 16) && T % JH == 0, "toeplitz slice geometry");
    constexpr int TJ = T / JH, LPU = 16 * NPG, UPW = 256 / LPU, WPU = NPG < 4 ? 1 : NPG / 4, NX = NPL + TJ - 1;
    f2v* red = reinterpret_cast<f2v*>(smem);  // [UPW][WPU - 1][TJ][16]
    const int t = threadIdx.x, col = t & 15, pg = (t >> 4) % NPG, us = t / LPU;
    const int wu = pg >> 2, q4 = pg & 3;  // wave of the unit, group within the wave
    const int gpc = sa.B / 16;
    // two block halves of the same columns read the same filter and most of the same FDL rows:
    // their workgroups run on one XCD (workgroups go round-robin over the 8 XCDs) so the second
    // read hits its L2 -- within every 16 workgroups, XCD x takes the unit pair 2 x, 2 x + 1
    int wb = bid;
    if constexpr (JH == 2 && UPW == 1) {
        if (bid < ta.nwg / 16 * 16) {
            const int r = bid & 15;
            wb = (bid & ~15) + (r & 7) * 2 + (r >> 3);
        }
    }
    const int u = ta.u0 + wb * UPW + us;
    const bool live = u < ta.u1;
    const int uc = live ? u : ta.u1 - 1;
    const int jh = uc % JH, cg = uc / JH, c = cg / gpc, k = (cg - c * gpc) * 16 + col;
    const int j0 = jh * TJ, pa = ta.a + pg * NPL;
    f2v acc[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[j] = f2v(0.f);
    if constexpr (UPW == 1) {
        // one unit per workgroup: channel and block half are uniform, buffer loads with the
        // row offsets in SGPRs; filter rows past the band read 0 (the buffer ends at b)
        const int cu = __builtin_amdgcn_readfirstlane(c);
        const int ps8 = int(sa.pstride * int(sizeof(cf)));
        const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.H + int64_t(cu) * sa.cstride, int64_t(ta.b) * ps8);
        const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.fdl + int64_t(cu) * sa.cstride, int64_t(sa.ring) * ps8);
        if (live && pa < ta.b) {
            cf xr[NX], hm[NPL];
            // xr[i] = X[tw + j0 + TJ - 1 - pa - i] = row r0 + NX - 1 - i, r0 the lane's oldest
            // row; rows from r0 + dw on wrap to the ring's start
            int r0 = ta.tw + j0 + TJ - 1 - pa - (NX - 1);
            r0 = r0 < 0 ? r0 + sa.ring : r0;
            const int dw = sa.ring - r0;
            const int v0 = r0 * ps8 + k * int(sizeof(cf)), vw = v0 - sa.ring * ps8;
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const int d = NX - 1 - i;
                xr[i] = buf_ld(xres, (d >= dw ? vw : v0) + d * ps8, 0);  // >= 0 either way
            }
            const int hv0 = pa * ps8 + k * int(sizeof(cf));
#pragma unroll
            for (int m = 0; m < NPL; ++m) hm[m] = buf_ld(hres, hv0, m * ps8);
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                const pk_coef h(hm[m], k == 0);
#pragma unroll
                for (int jj = 0; jj < TJ; ++jj) h.mac(acc[jj], xr[TJ - 1 - jj + m]);
            }
        }
    } else {
        const cf* Hc = sa.H + int64_t(c) * sa.cstride + k;
        const cf* Xc = sa.fdl + int64_t(c) * sa.cstride + k;
        if (live && pa < ta.b) {
            cf xr[NX], hm[NPL];
            // xr[i] = X[tw + j0 + TJ - 1 - pa - i]: partition pa + m meets block j0 + jj at i = TJ - 1 - jj + m
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                int r = ta.tw + j0 + TJ - 1 - pa - i;
                r = r < 0 ? r + sa.ring : r;
                xr[i] = ld_nt(Xc + int64_t(r) * sa.pstride);
            }
#pragma unroll
            for (int m = 0; m < NPL; ++m) hm[m] = pa + m < ta.b ? ld_h(Hc + int64_t(pa + m) * sa.pstride, ta.b) : cf{0.f, 0.f};
#pragma unroll
            for (int m = 0; m < NPL; ++m) {
                const pk_coef h(hm[m], k == 0);
#pragma unroll
                for (int jj = 0; jj < TJ; ++jj) h.mac(acc[jj], xr[TJ - 1 - jj + m]);
            }
        }
    }
    if constexpr (NPG >= 4) {  // the 4 groups of a wave (lanes 16 apart): VALU lane swaps, no LDS
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            acc[j].x = xor_sum<16>(acc[j].x);
            acc[j].y = xor_sum<16>(acc[j].y);
            acc[j].x = xor_sum<32>(acc[j].x);
            acc[j].y = xor_sum<32>(acc[j].y);
        }
    }
    // every lane of a wave now holds its wave's sum; the lanes of group 0 carry it on (a
    // per-lane choice of blocks would index the accumulators at run time: scratch)
    if constexpr (WPU > 1) {
        if (wu > 0 && q4 == 0) {
#pragma unroll
            for (int j = 0; j < TJ; ++j) red[((us * (WPU - 1) + wu - 1) * TJ + j) * 16 + col] = acc[j];
        }
        __syncthreads();
    }
    if (wu == 0 && q4 == 0 && live) {
        cf* o = ta.slab + int64_t(c) * ta.cs + int64_t(j0) * sa.B + k;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            f2v v = acc[j];
            if constexpr (WPU > 1) {
#pragma unroll
                for (int w = 1; w < WPU; ++w) v += red[((us * (WPU - 1) + w - 1) * TJ + j) * 16 + col];
            }
            o[int64_t(j) * sa.B] = cf{v.x, v.y};
        }
    }
}

// Toeplitz levels: slab[c][j][k] = sum_{p = a}^{b-1} H[c][p][k] X[c][(tw + j - p) mod R][k],
// j < T, for the next window (toep_lds_role below). Complex MAC in two packed FMAs, the
// splat / swap / sign folded into operand modifiers: acc += (hr, hr)(xr, xi) + (-hi, hi)(xi, xr).
__device__ __forceinline__ void cmac_pk(f2v& acc, cf h, cf x)
{
    const f2v xv = {x.x, x.y};
    acc = __builtin_elementwise_fma(f2v{h.x, h.x}, xv, acc);
    acc = __builtin_elementwise_fma(f2v{-h.y, h.y}, xv.yx, acc);
}

template<bool BIN0>
__device__ __forceinline__ void t32_step(f2v (&acc)[4], cf (&xw)[4], cf h, cf xn, bool z0)
{
    xw[3] = xw[2];
    xw[2] = xw[1];
    xw[1] = xw[0];
    xw[0] = xn;
    if constexpr (BIN0) {
        const pk_coef hk(h, z0);
#pragma unroll
        for (int o = 0; o < 4; ++o) hk.mac(acc[o], xw[o]);
    } else {
#pragma unroll
        for (int o = 0; o < 4; ++o) cmac_pk(acc[o], h, xw[o]);
    }
}

// partitions m = m0 .. m1 - 1 (p = a + m, m0 even): output j0 + o (o < 4) meets FDL value
// i = ib - m + o (ib = j0 + nb - 1), so each partition brings one new value, xc[ib - m], and
// the other three slide over. Partition pairs (m, m + 1) come as one 16-B LDS read of the
// filter column and one of the FDL column (xc is offset so that xc + ib - m - 1 is 16-B
// aligned), four pairs per chunk with all their reads issued first.
template<bool BIN0>
__device__ __forceinline__ void t32_walk(const cf* hc, const cf* xc, int ib, int m0, int m1, bool z0, f2v (&acc)[4])
{
    constexpr int KP = 4;
    cf xw[4];
#pragma unroll
    for (int o = 0; o < 3; ++o) xw[o] = xc[ib - m0 + 1 + o];
    int m = m0;
    for (; m + 2 * KP <= m1; m += 2 * KP) {
        float4 h2[KP], x2[KP];
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            h2[i] = *reinterpret_cast<const float4*>(hc + m + 2 * i);
            x2[i] = *reinterpret_cast<const float4*>(xc + ib - (m + 2 * i) - 1);
        }
#pragma unroll
        for (int i = 0; i < KP; ++i) {
            t32_step<BIN0>(acc, xw, cf{h2[i].x, h2[i].y}, cf{x2[i].z, x2[i].w}, z0);
            t32_step<BIN0>(acc, xw, cf{h2[i].z, h2[i].w}, cf{x2[i].x, x2[i].y}, z0);
        }
    }
    for (; m < m1; ++m) t32_step<BIN0>(acc, xw, hc[m], xc[ib - m], z0);
}

// Toeplitz level with window T through LDS, for every level (band [a, b), b - a <= NB):
// 32 / T units of 16 columns per workgroup, each with the whole window. A unit's filter rows
// and the FDL rows they meet (b - a and b - a + T - 1 rows of 16 columns: its distinct data,
// loaded once, coalesced) go to an LDS tile, column-major; lane (col, q4, half) then owns
// outputs 4 q4 .. 4 q4 + 3 of its column over half of the band (t32_walk), and the halves
// meet through LDS.
template<int T, int NB, int JH>
struct toep_tile {
    static constexpr int UPW = 32 / T, LPU = 256 / UPW, NQ = LPU / 16;  // units per workgroup, lanes per unit
    static constexpr int TP = T / JH, QUADS = TP / 4, NG = NQ / QUADS;  // outputs per unit, lanes per column, band groups
    static constexpr int HS = NB + 2, XS = NB + TP + 2;                 // even column strides (16-B aligned pair reads)
    static constexpr int NH = (NB + NQ - 1) / NQ, NXL = (NB + TP - 1 + NQ - 1) / NQ;
    static constexpr int LDS = UPW * 16 * (HS + XS) * int(sizeof(cf));
    static_assert(NG >= 2 && NQ % QUADS == 0 && TP % 4 == 0, "toeplitz tile geometry");
};

// unit u = (column group u / JH, window part u mod JH of T / JH outputs); JH = 2 where a step
// has few units (one channel: the part halves the longest chain of the step)
template<int T, int NB, int JH>
__device__ __forceinline__ void toep_lds_role(const slice_args& sa, const toep_arg& ta, int bid, char* smem)
{
    using G = toep_tile<T, NB, JH>;
    static_assert(G::LDS <= kSliceLds, "toeplitz tile");
    const int t = threadIdx.x, us = t / G::LPU, lt = t % G::LPU, col = lt & 15, q = lt >> 4;
    cf* hs = reinterpret_cast<cf*>(smem) + us * 16 * (G::HS + G::XS);  // hs[col][m] = H[p = a + m]
    cf* xs = hs + 16 * G::HS;                                          // xs[col][i] = X[the oldest row + i]
    const int u = ta.u0 + bid * G::UPW + us, gpc = sa.B / 16;
    const bool live = u < ta.u1;
    const int uc = live ? u : ta.u1 - 1, jp = uc % JH, cg = uc / JH, c = cg / gpc, g = cg - c * gpc;
    const int k = g * 16 + col, nb = ta.b - ta.a, nx = nb + G::TP - 1, R = sa.ring, jpart = jp * G::TP;
    int rb = ta.tw + jpart - (ta.b - 1);  // the oldest row (b - 1 < 256 < R: one wrap at most)
    rb = rb < 0 ? rb + R : rb;
    cf hv[G::NH], xv[G::NXL];  // every load of the lane in flight, then the LDS writes
    if constexpr (G::UPW == 1) {  // channel uniform: buffer loads, row offsets in SGPRs
        const int cu = __builtin_amdgcn_readfirstlane(c), ps8 = int(sa.pstride * int(sizeof(cf)));
        const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.H + int64_t(cu) * sa.cstride, int64_t(ta.b) * ps8);
        const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.fdl + int64_t(cu) * sa.cstride, int64_t(R) * ps8);
#pragma unroll
        for (int i = 0; i < G::NH; ++i) {
            const int m = q + G::NQ * i;
            if (m < nb) hv[i] = buf_ld(hres, (ta.a + m) * ps8 + k * int(sizeof(cf)), 0);
        }
#pragma unroll
        for (int i = 0; i < G::NXL; ++i) {
            const int r = q + G::NQ * i;
            if (r < nx) xv[i] = buf_ld(xres, (rb + r >= R ? rb + r - R : rb + r) * ps8 + k * int(sizeof(cf)), 0);
        }
    } else {
        const cf* Hc = sa.H + int64_t(c) * sa.cstride + k;
        const cf* Xc = sa.fdl + int64_t(c) * sa.cstride + k;
#pragma unroll
        for (int i = 0; i < G::NH; ++i) {
            const int m = q + G::NQ * i;
            if (live && m < nb) hv[i] = ld_h(Hc + int64_t(ta.a + m) * sa.pstride, ta.b);
        }
#pragma unroll
        for (int i = 0; i < G::NXL; ++i) {
            const int r = q + G::NQ * i;
            if (live && r < nx) xv[i] = ld_nt(Xc + int64_t(rb + r >= R ? rb + r - R : rb + r) * sa.pstride);
        }
    }
    const int odd = nb & 1;  // FDL column shift: keeps the pair reads 16-B aligned (t32_walk)
    if (live) {
#pragma unroll
        for (int i = 0; i < G::NH; ++i)
            if (q + G::NQ * i < nb) hs[col * G::HS + q + G::NQ * i] = hv[i];
#pragma unroll
        for (int i = 0; i < G::NXL; ++i)
            if (q + G::NQ * i < nx) xs[col * G::XS + odd + q + G::NQ * i] = xv[i];
    }
    __syncthreads();
    NEO_TL_MARK(sa);
    // lane (col, quad, group): outputs 4 quad .. 4 quad + 3 of the part, partitions of band group
    const int grp = q / G::QUADS, j0 = 4 * (q - grp * G::QUADS), nq = ((nb + G::NG - 1) / G::NG + 1) & ~1;
    const int m0 = grp * nq < nb ? grp * nq : nb, m1 = m0 + nq < nb ? m0 + nq : nb;
    f2v acc[4] = {f2v(0.f), f2v(0.f), f2v(0.f), f2v(0.f)};
    const cf* hc = hs + col * G::HS;
    const cf* xc = xs + col * G::XS + odd;
    if (live && m0 < m1) {
        if (g == 0) t32_walk<true>(hc, xc, j0 + nb - 1, m0, m1, col == 0, acc);  // uniform per unit
        else t32_walk<false>(hc, xc, j0 + nb - 1, m0, m1, false, acc);
    }
    __syncthreads();  // the tiles are free: the band groups meet there
    constexpr int LG = 16 * G::QUADS;          // lanes per band group
    f2v* red = reinterpret_cast<f2v*>(smem);  // [units][NG - 1][LG][4]
    const int lg = lt - grp * LG;
    if (grp) {
#pragma unroll
        for (int o = 0; o < 4; ++o) red[((us * (G::NG - 1) + grp - 1) * LG + lg) * 4 + o] = acc[o];
    }
    __syncthreads();
    if (!grp && live) {
        cf* o = ta.slab + int64_t(c) * ta.cs + int64_t(jpart + j0) * sa.B + k;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f2v v = acc[i];
#pragma unroll
            for (int r = 1; r < G::NG; ++r) v += red[((us * (G::NG - 1) + r - 1) * LG + lg) * 4 + i];
            o[int64_t(i) * sa.B] = cf{v.x, v.y};
        }
    }
}

// The big Toeplitz level (window kBigT = 128, band [256, P), instead of the far level when
// neo_hip_upols_opts.far_level = 0): per 16-column unit, kBigJH parts of kBigJP = 16 outputs, one
// workgroup each (the parts of a column group on one XCD: they share filter rows and most
// FDL rows through its L2). The band goes through an LDS tile in chunks of kBigNC
// partitions; lane (col, quad, quarter) owns 4 outputs of the part over a quarter of each
// chunk (t32_walk), and the quarters meet through LDS at the end.
constexpr int kBigJH = 8, kBigJP = kBigT / kBigJH, kBigNC = 192;
constexpr int kBigHS = kBigNC + 2, kBigXS = kBigNC + kBigJP + 2;  // even column strides
static_assert(16 * (kBigHS + kBigXS) * int(sizeof(cf)) <= kSliceLds, "big level tile");

__device__ __forceinline__ void toep_big_role(const slice_args& sa, const toep_arg& ta, int bid, char* smem)
{
    constexpr int NH = kBigNC / 16, NXL = (kBigNC + kBigJP - 1 + 15) / 16;
    cf* hs = reinterpret_cast<cf*>(smem);  // hs[col][m] = H[p = a + mc + m]
    cf* xs = hs + 16 * kBigHS;             // xs[col][i] = X[the chunk's oldest row + i]
    const int t = threadIdx.x, col = t & 15, qq = t >> 4, quad = qq & 3, quarter = qq >> 2;
    int wb = bid;  // within every 64 workgroups, XCD x (= blockIdx mod 8) takes the 8 parts of column groups x, x + 8, ...
    if (bid < ta.nwg / 64 * 64) {
        const int r = bid & 63;
        wb = (bid & ~63) + (r & 7) * 8 + (r >> 3);
    }
    const int u = ta.u0 + wb, jp = u % kBigJH, cg = u / kBigJH, gpc = sa.B / 16;
    const int c = __builtin_amdgcn_readfirstlane(cg / gpc), g = __builtin_amdgcn_readfirstlane(cg - (cg / gpc) * gpc);
    const int k = g * 16 + col, nb = ta.b - ta.a, R = sa.ring, jpart = jp * kBigJP;
    const int ps8 = int(sa.pstride * int(sizeof(cf)));
    const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.H + int64_t(c) * sa.cstride, int64_t(ta.b) * ps8);
    const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.fdl + int64_t(c) * sa.cstride, int64_t(R) * ps8);
    f2v acc[4] = {f2v(0.f), f2v(0.f), f2v(0.f), f2v(0.f)};
    for (int mc = 0; mc < nb; mc += kBigNC) {  // uniform per workgroup
        const int nc = nb - mc < kBigNC ? nb - mc : kBigNC, nx = nc + kBigJP - 1;
        // the chunk's oldest FDL row: tw + jpart - (a + mc + nc - 1), at most P + 127 < R + 128 rows back
        int rb = (ta.tw + jpart - (ta.a + mc + nc - 1)) % R;
        rb = rb < 0 ? rb + R : rb;
        cf hv[NH], xv[NXL];
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            const int m = qq + 16 * i;
            if (m < nc) hv[i] = buf_ld(hres, (ta.a + mc + m) * ps8 + k * int(sizeof(cf)), 0);
        }
#pragma unroll
        for (int i = 0; i < NXL; ++i) {
            const int r = qq + 16 * i;
            if (r < nx) xv[i] = buf_ld(xres, (rb + r >= R ? rb + r - R : rb + r) * ps8 + k * int(sizeof(cf)), 0);
        }
        if (mc) __syncthreads();  // the previous chunk's walk is done with the tile
        const int odd = nc & 1;   // FDL column shift: keeps the pair reads 16-B aligned (t32_walk)
#pragma unroll
        for (int i = 0; i < NH; ++i)
            if (qq + 16 * i < nc) hs[col * kBigHS + qq + 16 * i] = hv[i];
#pragma unroll
        for (int i = 0; i < NXL; ++i)
            if (qq + 16 * i < nx) xs[col * kBigXS + odd + qq + 16 * i] = xv[i];
        __syncthreads();
        const int nq = ((nc + 3) / 4 + 1) & ~1, m0 = quarter * nq, m1 = m0 + nq < nc ? m0 + nq : nc;
        if (m0 < m1) {
            const cf* hc = hs + col * kBigHS;
            const cf* xc = xs + col * kBigXS + odd;
            if (g == 0) t32_walk<true>(hc, xc, nc - 1 + 4 * quad, m0, m1, col == 0, acc);  // uniform branch
            else t32_walk<false>(hc, xc, nc - 1 + 4 * quad, m0, m1, false, acc);
        }
    }
    __syncthreads();  // the tile is free: the quarters meet there
    f2v* red = reinterpret_cast<f2v*>(smem);  // [3][64][4]
    const int ql = t & 63;                    // (col, quad)
    if (quarter) {
#pragma unroll
        for (int o = 0; o < 4; ++o) red[((quarter - 1) * 64 + ql) * 4 + o] = acc[o];
    }
    __syncthreads();
    if (!quarter) {
        cf* o = ta.slab + int64_t(c) * ta.cs + int64_t(jpart + 4 * quad) * sa.B + k;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const f2v v = acc[i] + red[ql * 4 + i] + red[(64 + ql) * 4 + i] + red[(128 + ql) * 4 + i];
            o[int64_t(i) * sa.B] = cf{v.x, v.y};
        }
    }
}

// Far level, for 16-column units (unit = channel c, columns 16 g ...): the far field of window
// wn (first block at ring row tw), ff[c][j][k], j < 128:
//   FF[j] = IDFT256( sum_s XF_s . HF_s )[128 + j] / 256,   s = 0 .. nseg - 1 (segment q = s + 2)
// XF_s = DFT256 of the FDL rows tw - (s + 3) 128 ... + 255 (the row pair of segment s), stored
// in slot (wn - s - 1) mod M. Segments s < fnfresh are transformed from the FDL (s = 0 in
// steady state, all when the pipeline is primed), the others were stored by earlier windows.
// Two phases, one step apart (the kernel boundary between them is the only synchronization:
// an agent-scope release per workgroup costs an L2 write-back across the XCDs):
//   phase 1  16 workgroups per unit MAC the stored segments for 16 f each, one (f, column) per
//            lane with every load of the lane in flight at once, into acc[unit][f][col]
//   phase 2  one workgroup per unit: the fresh row pairs' transforms (stored to their slots
//            for later windows) and products, + acc, the inverse transform
// Phase 2 reads FDL rows up to tw - 129, the last block before the window in progress, which
// an earlier launch wrote. Packed bin 0 holds two real sequences (DC and Nyquist): its spectra are
// stored packed the real-FFT way, W[f] = X_dc[f] (f <= 128) and W[256 - f] = X_ny[f]
// (0 < f < 128), with W[0] = (X_dc[0], X_ny[0]) and W[128] = (X_dc[128], X_ny[128]) real pairs
// (k_lvf_filter packs the segment spectra the same way): the MAC is the same complex product
// except two real products at f = 0 and 128, and one unpack before the inverse transform
// restores Y = Y_dc + i Y_ny.

// Z = DFT(x_dc + i x_ny) -> packed W (real-FFT packing of X_dc, X_ny) at f, from Z[f], Z[-f]
__device__ __forceinline__ cf pack_bin0(cf zf, cf zm, int f)
{
    if (f == 0 || f == kFN / 2) return zf;  // (Re, Im) = (X_dc, X_ny), both real here
    if (f < kFN / 2) return cscale(cadd(zf, cconj(zm)), 0.5f);  // X_dc[f]
    const cf d = csub(zm, cconj(zf));                            // f > 128: X_ny[256 - f] = (Z[-f] - conj Z[f]) / 2i
    return cf{0.5f * d.y, -0.5f * d.x};
}

// packed W of bin 0 -> Y = Y_dc + i Y_ny at f, from W[f], W[-f]
__device__ __forceinline__ cf unpack_bin0(cf wf, cf wm, int f)
{
    if (f == 0 || f == kFN / 2) return wf;
    // f < 128: Y_dc[f] + i Y_ny[f] = W[f] + i W[256 - f]; f > 128: conj(W[256 - f]) + i conj(W[f])
    const cf dc = f < kFN / 2 ? wf : cconj(wm);
    const cf ny = f < kFN / 2 ? wm : cconj(wf);
    return cf{dc.x - ny.y, dc.y + ny.x};
}

// bin 0 (column 0, lanes cp == 0) of a spectrum held with v[i] at f = a + 16 i: pack or unpack
// through LDS z; every lane calls (barrier inside)
template<bool PACK>
__device__ __forceinline__ void bin0_exchange(cf (&v)[16], cf* z, int a, int cp)
{
    if (cp == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) z[a + 16 * i] = v[i];
    }
    __syncthreads();
    if (cp == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int f = a + 16 * i;
            const cf m = z[(kFN - f) & (kFN - 1)];
            v[i] = PACK ? pack_bin0(v[i], m, f) : unpack_bin0(v[i], m, f);
        }
    }
}

// phase 1, FPL f rows per lane: a workgroup takes kF1UG units side by side (64 columns:
// every wave-load reads 512 contiguous bytes of one f row) and 4 FPL f rows of them, so
// kFN / (4 FPL) workgroups per unit group; the host picks FPL so that one round of NS =
// 16 / FPL segments covers the stored ones (every load of a lane in flight at once).
// Window groups: the stored segments of window wn are s = 1 .. nseg - 1 (XF slot wn - s - 1),
// those of window wn + j are s = j + 1 .. nseg - 1 (slot wn + j - s - 1: the same slots, j
// segments on) -- so a unit group of class c = (group index) mod K takes K windows in one pass
// over its spectra (each XF and HF value read once for up to K products) when wn = c mod K, and
// the other classes take theirs in the other windows: 1/K of the phase-1 reads. Segments 1 .. j
// of window wn + j (slots not yet stored when the pass runs: phase 2 of windows wn .. wn + j - 1
// writes them) are phase 2's, in that window (f2grp). K ~ sqrt(2 (nseg - 1)) (far_group) balances
// the two: 2 (nseg - 1) / K + K - 1 spectra per window and column instead of 2 (nseg - 1).
constexpr int kF1UG = 4;
constexpr int kFarKMax = 4;

// first window >= 1 whose phase-1 pass a unit group of class c starts (earlier windows after
// priming: one window per pass)
__host__ __device__ __forceinline__ int far_first(int c, int K) { return 1 + ((c - 1) % K + K) % K; }

template<int FPL, int K>
__device__ __forceinline__ void far1_mac(const slice_args& sa, int u, int f0, int col)
{
    constexpr int NS = 16 / FPL;  // segments per round
    static_assert(NS >= K - 1 || K == 1, "history of the previous round");
    const int gpc = sa.B / 16, c = u / gpc, g = u - c * gpc, k = g * 16 + col;
    const int M = sa.M, nseg = sa.nseg, wn = sa.f1wn;
    auto slot = [&](int s) { return ((wn - s - 1) % M + M) % M; };
    const int64_t fs = sa.B, sp = int64_t(kFN) * fs;  // one spectrum
    const int s0 = sa.fnfresh < nseg ? sa.fnfresh : nseg;  // first stored segment (1 when K > 1)
    const cf* hc = sa.hf + int64_t(c) * sa.fsc + int64_t(f0) * fs + k;
    const cf* xc = sa.xf + int64_t(c) * sa.fsc + int64_t(f0) * fs + k;
    f2v acc[K][FPL];             // window wn + j
    cf xp[K > 1 ? K - 1 : 1][FPL];  // xp[d]: segment sb - 1 - d's spectra (the previous rounds)
    bool z0[FPL];                // packed bin 0, f = 0 and 128
#pragma unroll
    for (int j = 0; j < FPL; ++j) {
#pragma unroll
        for (int w = 0; w < K; ++w) acc[w][j] = f2v(0.f);
        z0[j] = g == 0 && col == 0 && ((f0 + 4 * j) & (kFN / 2 - 1)) == 0;
    }
    for (int sb = s0; sb < nseg; sb += NS) {
        cf xv[NS][FPL], hv[NS][FPL];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (sb + i < nseg) {
                const cf* hs = hc + (sb + i) * sp;
                const cf* xs = xc + slot(sb + i) * sp;
#pragma unroll
                for (int j = 0; j < FPL; ++j) {
                    hv[i][j] = ld_nt(hs + 4 * j * fs);
                    xv[i][j] = ld_nt(xs + 4 * j * fs);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (sb + i < nseg) {
#pragma unroll
                for (int j = 0; j < FPL; ++j) {
                    const pk_coef h(hv[i][j], z0[j]);
#pragma unroll
                    for (int w = 0; w < K; ++w)  // window wn + w: segment sb + i meets slot of sb + i - w
                        if (sb + i - w >= s0) h.mac(acc[w][j], i >= w ? xv[i - w][j] : xp[w - i - 1][j]);
                }
            }
        }
        if constexpr (K > 1) {
#pragma unroll
            for (int d = 0; d < K - 1; ++d)
#pragma unroll
                for (int j = 0; j < FPL; ++j) xp[d][j] = xv[NS - 1 - d][j];  // read only if the next round runs
        }
    }
#pragma unroll
    for (int w = 0; w < K; ++w) {
        cf* o = sa.f1acc + (int64_t(((wn + w) % sa.fK) * sa.fU + u) * kFN + f0) * 16 + col;
#pragma unroll
        for (int j = 0; j < FPL; ++j) o[4 * j * 16] = cf{acc[w][j].x, acc[w][j].y};
    }
}

// KMAX: the largest window group the kernel is built for (2: pairs only, the smaller register
// budget of the shapes below kFarGroupUnits; kFarKMax: any group, far_group's choice)
template<int FPL, int KMAX>
__device__ __forceinline__ void far1_role(const slice_args& sa, int bid)
{
    constexpr int FR = 4 * FPL, PPG = kFN / FR;  // f rows per workgroup, workgroups per group
    const int t = threadIdx.x, cl = t & 63, fq = t >> 6;
    const int grp = bid / PPG, part = bid - grp * PPG;
    const int g4 = sa.f1g0 + grp * sa.f1gs;  // the group (global index; uniform per workgroup)
    const int u = g4 * kF1UG + (cl >> 4);    // the lane's unit
    if (u < sa.f1u0 || u >= sa.f1u1) return;  // groups straddle slices (no barriers in this role)
    const int f0 = part * FR + fq;            // f = f0 + 4 j
    const int K = sa.fK, cls = sa.f1mode ? g4 % K : 0;
    if (sa.f1mode == 0 || (cls != sa.f1cls && far_first(cls, K) > sa.f1wn)) {
        far1_mac<FPL, 1>(sa, u, f0, cl & 15);  // one window (priming, or the class has not started)
    } else if (cls == sa.f1cls) {
        if constexpr (KMAX <= 2) {
            far1_mac<FPL, 2>(sa, u, f0, cl & 15);
        } else {
            if (K == 2) far1_mac<FPL, 2>(sa, u, f0, cl & 15);
            else if (K == 3) far1_mac<FPL, 3>(sa, u, f0, cl & 15);
            else far1_mac<FPL, kFarKMax>(sa, u, f0, cl & 15);
        }
    }
}

// far phase 2a: the fresh row pairs (segments s < fnfresh: s = 0 in steady state, all of them
// when the level primes) -> 256-point transforms along the partition axis, packed bin 0 ->
// their XF ring slots, which 2b reads one launch later
__device__ __forceinline__ void far2a_role(const slice_args& sa, int bid, char* smem)
{
    cf* lds = reinterpret_cast<cf*>(smem);  // [16][16][16] transposes
    cf* z = lds + 16 * 16 * 16;              // bin-0 exchange
    cf* tws = z + kFN;                       // twiddles
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int gpc = sa.B / 16, u = sa.f2u0 + bid, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool unit0 = g == 0;  // uniform per workgroup: the unit holding packed bin 0
    const int M = sa.M, nseg = sa.nseg;
    auto slot = [&](int s) { return ((sa.f2wn - s - 1) % M + M) % M; };
    const int64_t fs = sa.B;
    const int spec = int(int64_t(kFN) * fs * int(sizeof(cf)));
    const int s0 = sa.fnfresh < nseg ? sa.fnfresh : nseg;
    tws[t] = sa.twf[t];
    const __amdgpu_buffer_rsrc_t fres =
        buf_rsrc(sa.fdl + int64_t(c) * sa.cstride, int64_t(sa.ring) * sa.pstride * int(sizeof(cf)));
    const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.xf + int64_t(c) * sa.fsc, int64_t(M) * spec);
    const int vo = int((int64_t(a) * fs + k) * int(sizeof(cf)));
    for (int s = 0; s < s0; ++s) {  // uniform per workgroup (one segment in steady state)
        // rows tw - (s + 3) 128 + a + 16 n (the ring holds >= kFarRing > 256 rows: one wrap at most)
        cf x[16];
        int r0 = (sa.f2tw - (s + 3) * kFarT + a) % sa.ring;
        r0 = r0 < 0 ? r0 + sa.ring : r0;
#pragma unroll
        for (int n = 0; n < 16; ++n) {
            const int r = r0 + 16 * n >= sa.ring ? r0 + 16 * n - sa.ring : r0 + 16 * n;
            x[n] = buf_ld(fres, int((int64_t(r) * sa.pstride + k) * int(sizeof(cf))), 0);
        }
        __syncthreads();  // twiddles; the previous segment's LDS use is done
        col_fft<-1, 16>(x, lds, tws, a, cp, true);
        if (s == 0) NEO_TL_MARK(sa);
        if (unit0) bin0_exchange<true>(x, z, a, cp);  // uniform per workgroup
#pragma unroll
        for (int i = 0; i < 16; ++i) buf_st(x[i], xres, vo, slot(s) * spec + int(16 * i * fs * int(sizeof(cf))));
    }
}

// far phase 2b, one launch after 2a for the same units: v[i] at f = a + 16 i (col_fft's layout)
// = phase 1's partial sums (stored segments) + the fresh segments' products XF_s . HF_s from
// the slots 2a wrote + (window groups) segments 1 .. j of window j of the unit's phase-1 group;
// unpack bin 0, inverse transform, the window's 128 far-field rows
template<int KMAX>
__device__ __forceinline__ void far2b_role(const slice_args& sa, int bid, char* smem)
{
    cf* lds = reinterpret_cast<cf*>(smem);  // [16][16][16] transposes
    cf* z = lds + 16 * 16 * 16;              // bin-0 exchange
    cf* tws = z + kFN;                       // twiddles
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int gpc = sa.B / 16, u = sa.f3u0 + bid, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool unit0 = g == 0;  // uniform per workgroup: the unit holding packed bin 0
    const int M = sa.M, nseg = sa.nseg;
    auto slot = [&](int s) { return ((sa.f3wn - s - 1) % M + M) % M; };
    const int64_t fs = sa.B;
    const int spec = int(int64_t(kFN) * fs * int(sizeof(cf)));
    const int s0 = sa.fnfresh < nseg ? sa.fnfresh : nseg;
    tws[t] = sa.twf[t];
    const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.hf + int64_t(c) * sa.fsc, int64_t(nseg) * spec);
    const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.xf + int64_t(c) * sa.fsc, int64_t(M) * spec);
    const __amdgpu_buffer_rsrc_t ares =
        buf_rsrc(sa.f2acc + int64_t((sa.f3wn % sa.fK) * sa.fU + u) * kFN * 16, kFN * 16 * int(sizeof(cf)));
    const int vo = int((int64_t(a) * fs + k) * int(sizeof(cf)));
    const int ao = (a * 16 + cp) * int(sizeof(cf)), as = 16 * 16 * int(sizeof(cf));  // f = a + 16 i
    auto z0 = [&](int i) { return unit0 && cp == 0 && ((a + 16 * i) & (kFN / 2 - 1)) == 0; };
    cf v[16];
    {  // the partial sums and segment 0's spectra in one round of loads
        cf hv[16], xv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = buf_ld(ares, ao, i * as);
            hv[i] = buf_ld(hres, vo, int(16 * i * fs * int(sizeof(cf))));
            xv[i] = buf_ld(xres, vo, slot(0) * spec + int(16 * i * fs * int(sizeof(cf))));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f2v w = {v[i].x, v[i].y};
            pk_coef(hv[i], z0(i)).mac(w, xv[i]);
            v[i] = cf{w.x, w.y};
        }
    }
    // the other fresh segments (priming: every segment), then the window group's segments
    // 1 .. j (slots f3wn - 2 .. f3wn - j - 1, stored by the group's earlier windows; not
    // there when the group's phase-1 pass ran)
    int jw = 0;
    if (sa.f2grp) {  // uniform per workgroup
        const int K = sa.fK, cls = (u / kF1UG) % K, first = far_first(cls, K);
        jw = sa.f3wn >= first ? (sa.f3wn - cls) % K : 0;
    }
    const int s1 = s0 > 1 ? s0 : (jw + 1 < nseg ? jw + 1 : nseg);  // segments [1, s1) from slots
    for (int s = 1; s < s1 && (s0 > 1 || s < KMAX); ++s) {  // uniform per workgroup
        cf hv[16], xv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            hv[i] = buf_ld(hres, vo, s * spec + int(16 * i * fs * int(sizeof(cf))));
            xv[i] = buf_ld(xres, vo, slot(s) * spec + int(16 * i * fs * int(sizeof(cf))));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f2v w = {v[i].x, v[i].y};
            pk_coef(hv[i], z0(i)).mac(w, xv[i]);
            v[i] = cf{w.x, w.y};
        }
    }
    __syncthreads();  // twiddles
    NEO_TL_MARK(sa);
    if (unit0) bin0_exchange<false>(v, z, a, cp);  // uniform per workgroup
    col_fft<1, 16>(v, lds, tws, a, cp, true);
    constexpr float sc = 1.0f / kFN;
    const __amdgpu_buffer_rsrc_t ores = buf_rsrc(sa.f3ff + int64_t(c) * sa.fcs, spec / 2);
#pragma unroll
    for (int m = 8; m < 16; ++m)  // n = 16 m + a >= 128
        buf_st(cscale(v[m], sc), ores, vo, int(16 * (m - 8) * fs * int(sizeof(cf))));
}

// far phase 2 in one workgroup (step groups' background launches, where phase 2's chain is not
// the step's longest): the fresh row pair's transform (stored to its slot for later windows, as
// 2a) kept in registers for the products of 2b -- no write-then-read of the slot within a window.
// Steady state only (one fresh segment); priming runs 2a and 2b.
template<int KMAX>
__device__ __forceinline__ void far2c_role(const slice_args& sa, int bid, char* smem)
{
    cf* lds = reinterpret_cast<cf*>(smem);  // [16][16][16] transposes
    cf* z = lds + 16 * 16 * 16;              // bin-0 exchange
    cf* tws = z + kFN;                       // twiddles
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int gpc = sa.B / 16, u = sa.f3u0 + bid, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool unit0 = g == 0;  // uniform per workgroup: the unit holding packed bin 0
    const int M = sa.M, nseg = sa.nseg;
    auto slot = [&](int s) { return ((sa.f3wn - s - 1) % M + M) % M; };
    const int64_t fs = sa.B;
    const int spec = int(int64_t(kFN) * fs * int(sizeof(cf)));
    tws[t] = sa.twf[t];
    const __amdgpu_buffer_rsrc_t fres =
        buf_rsrc(sa.fdl + int64_t(c) * sa.cstride, int64_t(sa.ring) * sa.pstride * int(sizeof(cf)));
    const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.hf + int64_t(c) * sa.fsc, int64_t(nseg) * spec);
    const __amdgpu_buffer_rsrc_t xres = buf_rsrc(sa.xf + int64_t(c) * sa.fsc, int64_t(M) * spec);
    const __amdgpu_buffer_rsrc_t ares =
        buf_rsrc(sa.f2acc + int64_t((sa.f3wn % sa.fK) * sa.fU + u) * kFN * 16, kFN * 16 * int(sizeof(cf)));
    const int vo = int((int64_t(a) * fs + k) * int(sizeof(cf)));
    const int ao = (a * 16 + cp) * int(sizeof(cf)), as = 16 * 16 * int(sizeof(cf));  // f = a + 16 i
    auto z0 = [&](int i) { return unit0 && cp == 0 && ((a + 16 * i) & (kFN / 2 - 1)) == 0; };
    // the fresh row pair: rows tw - 3 128 + a + 16 n (one wrap of the ring at most)
    cf x[16];
    {
        int r0 = (sa.f2tw - 3 * kFarT + a) % sa.ring;
        r0 = r0 < 0 ? r0 + sa.ring : r0;
#pragma unroll
        for (int n = 0; n < 16; ++n) {
            const int r = r0 + 16 * n >= sa.ring ? r0 + 16 * n - sa.ring : r0 + 16 * n;
            x[n] = buf_ld(fres, int((int64_t(r) * sa.pstride + k) * int(sizeof(cf))), 0);
        }
    }
    __syncthreads();  // twiddles
    col_fft<-1, 16>(x, lds, tws, a, cp, true);
    if (unit0) bin0_exchange<true>(x, z, a, cp);  // uniform per workgroup
    cf v[16];
    {
        cf hv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = buf_ld(ares, ao, i * as);
            hv[i] = buf_ld(hres, vo, int(16 * i * fs * int(sizeof(cf))));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) buf_st(x[i], xres, vo, slot(0) * spec + int(16 * i * fs * int(sizeof(cf))));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f2v w = {v[i].x, v[i].y};
            pk_coef(hv[i], z0(i)).mac(w, x[i]);
            v[i] = cf{w.x, w.y};
        }
    }
    // the window group's segments 1 .. j (slots f3wn - 2 .. f3wn - j - 1), as far2b_role
    int jw = 0;
    if (sa.f2grp) {  // uniform per workgroup
        const int K = sa.fK, cls = (u / kF1UG) % K, first = far_first(cls, K);
        jw = sa.f3wn >= first ? (sa.f3wn - cls) % K : 0;
    }
    const int s1 = jw + 1 < nseg ? jw + 1 : nseg;
    for (int s = 1; s < s1 && s < KMAX; ++s) {  // uniform per workgroup
        cf hv[16], xv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            hv[i] = buf_ld(hres, vo, s * spec + int(16 * i * fs * int(sizeof(cf))));
            xv[i] = buf_ld(xres, vo, slot(s) * spec + int(16 * i * fs * int(sizeof(cf))));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f2v w = {v[i].x, v[i].y};
            pk_coef(hv[i], z0(i)).mac(w, xv[i]);
            v[i] = cf{w.x, w.y};
        }
    }
    __syncthreads();  // the pack exchange's reads of z are done
    NEO_TL_MARK(sa);
    if (unit0) bin0_exchange<false>(v, z, a, cp);  // uniform per workgroup
    col_fft<1, 16>(v, lds, tws, a, cp, true);
    constexpr float sc = 1.0f / kFN;
    const __amdgpu_buffer_rsrc_t ores = buf_rsrc(sa.f3ff + int64_t(c) * sa.fcs, spec / 2);
#pragma unroll
    for (int m = 8; m < 16; ++m)  // n = 16 m + a >= 128
        buf_st(cscale(v[m], sc), ores, vo, int(16 * (m - 8) * fs * int(sizeof(cf))));
}

// Far level, recomputed form (neo_hip_upols_opts.far_level = 2; the default with step groups):
// one workgroup per 16-column unit and window computes the window's whole far field from the
// filter's and the FDL's own rows, nothing stored between windows but the field. Segment s
// (partitions [128 (s + 2), 128 (s + 3))) meets the row pair tw - (s + 3) 128 + r, r < 256; the
// pair of s + 1 is the pair of s moved back 128 rows, so its second half (n >= 8 in col_fft's
// layout) is the first half of the pair before, kept in registers: each FDL row of the band is
// read once per window. The segment's 128 filter rows (zero-padded to 256, zero past P) are
// transformed beside it (the same packed bin 0 as k_lvf_filter), the products accumulate in
// registers, one inverse transform gives samples 128..255: the field. Per column and window
// (nseg + 1) 128 FDL rows, P - 256 filter rows and 128 field rows -- against 2 (nseg - 1) / K + K
// + 2 stored spectra, the fresh pair, its slot and phase 1's partial sums of the stored form --
// at 2 nseg + 1 transforms per unit and window.
__device__ __forceinline__ void far2r_role(const slice_args& sa, int bid, char* smem)
{
    cf* lds = reinterpret_cast<cf*>(smem);  // [16][16][16] transposes
    cf* z = lds + 16 * 16 * 16;              // bin-0 exchange
    cf* tws = z + kFN;                       // twiddles
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    cf* xh = tws + kFN + t;  // [8][256]: raw rows of the pair before, first half (this pair's second half)
    const int gpc = sa.B / 16, u = sa.f3u0 + bid, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool unit0 = g == 0;  // uniform per workgroup: the unit holding packed bin 0
    const int64_t fs = sa.B;
    tws[t] = sa.twf[t];
    const int rb = int(int64_t(sa.ring) * sa.pstride * int(sizeof(cf)));
    const __amdgpu_buffer_rsrc_t fres = buf_rsrc(sa.fdl + int64_t(c) * sa.cstride, rb);
    const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.H + int64_t(c) * sa.cstride, rb);
    const int ko = k * int(sizeof(cf));
    auto z0 = [&](int i) { return unit0 && cp == 0 && ((a + 16 * i) & (kFN / 2 - 1)) == 0; };
    f2v acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = f2v(0.f);
    int r0 = (sa.f2tw - 3 * kFarT + a) % sa.ring;  // pair 0's row a (the ring holds > P + 256 rows)
    r0 = r0 < 0 ? r0 + sa.ring : r0;
    for (int s = 0; s < sa.nseg; ++s) {  // uniform per workgroup
        cf x[16], hv[16];
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int r = r0 + 16 * n >= sa.ring ? r0 + 16 * n - sa.ring : r0 + 16 * n;
            x[n] = buf_ld(fres, int(int64_t(r) * sa.pstride * int(sizeof(cf))) + ko, 0);
            const int p = (s + 2) * kFarT + a + 16 * n;
            hv[n] = p < sa.P ? buf_ld(hres, int(int64_t(p) * sa.pstride * int(sizeof(cf))) + ko, 0) : cf{0.f, 0.f};
            hv[n + 8] = cf{0.f, 0.f};
        }
        if (s == 0) {
#pragma unroll
            for (int n = 8; n < 16; ++n) {
                const int r = r0 + 16 * n >= sa.ring ? r0 + 16 * n - sa.ring : r0 + 16 * n;
                x[n] = buf_ld(fres, int(int64_t(r) * sa.pstride * int(sizeof(cf))) + ko, 0);
            }
        } else {
#pragma unroll
            for (int n = 8; n < 16; ++n) x[n] = xh[(n - 8) * 256];  // this lane's own stores
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) xh[n * 256] = x[n];
        r0 = r0 - kFarT < 0 ? r0 - kFarT + sa.ring : r0 - kFarT;
        if (s == 0) __syncthreads();  // twiddles (later segments: col_fft's closing barrier)
        col_fft<-1, 16>(x, lds, tws, a, cp, true);
        if (unit0) bin0_exchange<true>(x, z, a, cp);  // uniform per workgroup
        col_fft<-1, 16>(hv, lds, tws, a, cp, true);   // its barriers also order bin0_exchange's z reads
        if (unit0) bin0_exchange<true>(hv, z, a, cp);
#pragma unroll
        for (int i = 0; i < 16; ++i) pk_coef(hv[i], z0(i)).mac(acc[i], x[i]);
    }
    cf v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = cf{acc[i].x, acc[i].y};
    __syncthreads();  // the last pack exchange's reads of z are done
    NEO_TL_MARK(sa);
    if (unit0) bin0_exchange<false>(v, z, a, cp);  // uniform per workgroup
    col_fft<1, 16>(v, lds, tws, a, cp, true);
    constexpr float sc = 1.0f / kFN;
    const __amdgpu_buffer_rsrc_t ores = buf_rsrc(sa.f3ff + int64_t(c) * sa.fcs, int(kFN * fs * int(sizeof(cf))) / 2);
    const int vo = int((int64_t(a) * fs + k) * int(sizeof(cf)));
#pragma unroll
    for (int m = 8; m < 16; ++m)  // n = 16 m + a >= 128
        buf_st(cscale(v[m], sc), ores, vo, int(16 * (m - 8) * fs * int(sizeof(cf))));
}

// ---------------------------------------------------------------------------------------
// Offline windows (process calls with batching on: every block of the call is known up front,
// dense_convolve / the plugin's offline harness, DenseConvolution.hpp:39-70). The far level's
// decomposition applied to EVERY partition: per bin, Y[t_W + j] (j < 128) = sum over segments
// q >= 0 of 128 partitions of samples 128 + j of IDFT256(DFT256(X pair) . DFT256(h_q)), the pair
// being FDL rows t_W - 128 (q + 1) ... + 255 -- for q = 0 it holds the window's own rows, which
// k_batch_window inserted before this launch. One workgroup per 16-column unit walks the
// segments from q = 0 back (each pair's second half is the previous pair's first half: every
// FDL row of the band read once per pass), multiplies with the filter's segment spectra
// (k_lvf_filter from partition 0, computed at the first pass after a filter change) and
// inverse-transforms once per window. WP = 2 windows per pass share every spectrum load: pair
// q of the first window is pair q + 1 of the second (rows t_W + 128 - 128 (q + 2) ...), so the
// second window's products reuse the previous segment's transform with this segment's spectrum.
// Per column and pass: (nseg + WP) 128 FDL rows, nseg 256 spectrum rows, WP 128 output rows,
// against 2 P rows for the batched MAC's 32 blocks; nseg + WP forward and WP inverse
// transforms instead of 128 WP P complex MACs.
struct off_args {
    const cf* fdl;
    const cf* hf;  // [C][nseg][256][B]
    const cf* twf;
    cf* y;         // [C][128 WP][B]: the windows' output spectra
    int64_t cstride, pstride;
    int64_t hcs;   // hf's channel stride (spec_cs)
    int ring, B, nseg, w;  // w: ring row of the pass's first block
};

#ifndef NEO_OFF_PF
#define NEO_OFF_PF 0  // diagnostic builds (A/B): k_off_mac's software prefetch depth
#endif
template<int WP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WP == 1 ? 3 : 2))) void k_off_mac(off_args sa)
{
    __shared__ cf lds[16 * 16 * 16];  // col_fft transposes
    __shared__ cf z[kFN];              // bin-0 exchange
    __shared__ cf tws[kFN];
    __shared__ cf xh[8 * 256];         // raw rows of the pair before, first half (this pair's second half)
    const int t = threadIdx.x, a = t >> 4, cp = t & 15;
    const int gpc = sa.B / 16, u = blockIdx.x, c = u / gpc, g = u - c * gpc, k = g * 16 + cp;
    const bool unit0 = g == 0;  // uniform per workgroup: the unit holding packed bin 0
    const int64_t fs = sa.B;
    const int spec = int(int64_t(kFN) * fs * int(sizeof(cf)));
    tws[t] = sa.twf[t];
    const __amdgpu_buffer_rsrc_t fres =
        buf_rsrc(sa.fdl + int64_t(c) * sa.cstride, int64_t(sa.ring) * sa.pstride * int(sizeof(cf)));
    const __amdgpu_buffer_rsrc_t hres = buf_rsrc(sa.hf + int64_t(c) * sa.hcs, int64_t(sa.nseg) * spec);
    const int ps8 = int(sa.pstride * int(sizeof(cf))), ko = k * int(sizeof(cf));
    const int vo = int((int64_t(a) * fs + k) * int(sizeof(cf)));
    auto z0 = [&](int i) { return unit0 && cp == 0 && ((a + 16 * i) & (kFN / 2 - 1)) == 0; };
    auto row = [&](int r) { return r >= sa.ring ? r - sa.ring : r; };
    f2v acc[WP][16];
#pragma unroll
    for (int w = 0; w < WP; ++w)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[w][i] = f2v(0.f);
    // the first pair: rows w + 128 (WP - 2) + r, r < 256 (WP = 1: w - 128; WP = 2: w, the second
    // window's pair of segment 0); its row a + 16 n
    int r0 = (sa.w + kFarT * (WP - 2) + a) % sa.ring;
    r0 = r0 < 0 ? r0 + sa.ring : r0;
    cf xp[WP > 1 ? 16 : 1];  // WP = 2: the previous pair's spectrum (the second window's segment q)
    // software prefetch (NEO_OFF_PF): 1 the next pair's new rows, 2 also the next segment's
    // spectrum, loaded before this segment's transform so their latency hides behind it
    cf nx[NEO_OFF_PF >= 1 ? 8 : 1], nh[NEO_OFF_PF >= 2 ? 16 : 1];
    auto load_rows = [&](cf* dst, int n0, int n1) {
#pragma unroll
        for (int n = n0; n < n1; ++n) dst[n - n0] = buf_ld(fres, row(r0 + 16 * n) * ps8 + ko, 0);
    };
    auto load_spec = [&](cf* dst, int q) {
#pragma unroll
        for (int i = 0; i < 16; ++i) dst[i] = buf_ld(hres, vo, q * spec + int(16 * i * fs * int(sizeof(cf))));
    };
    __syncthreads();  // twiddles
    for (int q = 1 - WP; q < sa.nseg; ++q) {  // uniform per workgroup; q < 0: the second window's pair only
        cf x[16], hv[16];
        if (q == 1 - WP) {
            load_rows(x, 0, 16);
        } else {
            if constexpr (NEO_OFF_PF >= 1) {
#pragma unroll
                for (int n = 0; n < 8; ++n) x[n] = nx[n];
            } else {
                load_rows(x, 0, 8);
            }
#pragma unroll
            for (int n = 8; n < 16; ++n) x[n] = xh[(n - 8) * 256 + t];  // this lane's own stores
        }
        if (q >= 0) {
            if constexpr (NEO_OFF_PF >= 2) {
                if (q == 0) load_spec(hv, 0);
                else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) hv[i] = nh[i];
                }
            } else {
                load_spec(hv, q);
            }
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) xh[n * 256 + t] = x[n];
        r0 = r0 - kFarT < 0 ? r0 - kFarT + sa.ring : r0 - kFarT;
        if constexpr (NEO_OFF_PF >= 1)
            if (q + 1 < sa.nseg) load_rows(nx, 0, 8);  // the next pair's first half
        if constexpr (NEO_OFF_PF >= 2)
            if (q + 1 < sa.nseg && q + 1 >= 1) load_spec(nh, q + 1);
        col_fft<-1, 16>(x, lds, tws, a, cp, true);
        if (unit0) bin0_exchange<true>(x, z, a, cp);  // uniform per workgroup; the next col_fft's barriers order z
        if (q >= 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const pk_coef h(hv[i], z0(i));
                h.mac(acc[0][i], x[i]);
                if constexpr (WP > 1) h.mac(acc[1][i], xp[i]);
            }
        }
        if constexpr (WP > 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) xp[i] = x[i];
        }
    }
    constexpr float sc = 1.0f / kFN;
#pragma unroll
    for (int w = 0; w < WP; ++w) {
        cf v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = cf{acc[w][i].x, acc[w][i].y};
        __syncthreads();  // the last pack exchange's (or the previous window's) reads of z / lds are done
        if (unit0) bin0_exchange<false>(v, z, a, cp);  // uniform per workgroup
        col_fft<1, 16>(v, lds, tws, a, cp, true);
        const __amdgpu_buffer_rsrc_t ores =
            buf_rsrc(sa.y + (int64_t(c) * WP + w) * kFarT * fs, int64_t(kFarT) * fs * int(sizeof(cf)));
#pragma unroll
        for (int m = 8; m < 16; ++m)  // n = 16 m + a >= 128: block n - 128 of window w
            buf_st(cscale(v[m], sc), ores, vo, int(16 * (m - 8) * fs * int(sizeof(cf))));
    }
}

#ifndef NEO_ROLES
#define NEO_ROLES 63  // diagnostic builds (tools/build_roles.sh): 1 block, 2 Toeplitz T <= 16, 4 T = 32, 8 far 1, 16 far 2a, 32 far 2b
#endif

// Toeplitz level L of the step kernel (window T = kLvT0 << L, geometry as toep_geom): runs the
// role and returns true if workgroup bid is one of its slice's, else moves bid past them.
template<int L>
__device__ __forceinline__ bool toep_level(const slice_args& a, int& bid, char* smem)
{
    if (L >= a.ntp) return false;
    const toep_arg ta = a.tp[L];  // static index, by value: registers, not a scratch copy
    if (bid >= ta.nwg) {
        bid -= ta.nwg;
        return false;
    }
    static_assert(kLvT0 == 4 && kLvToep == 5, "level slots: windows 4, 8, 16, 32 (bands 2T, 2T, 2T, 6T), 128");
    if constexpr (L == 0) {  // T = 4, 8: a lane takes its column's whole band in registers
        if (NEO_ROLES & 2) toep_role<4, 8, 1, 1>(a, ta, bid, smem);
    } else if constexpr (L == 1) {
        if (NEO_ROLES & 2) toep_role<8, 16, 1, 1>(a, ta, bid, smem);
    } else if constexpr (L == 2) {
        if (NEO_ROLES & 2) toep_lds_role<16, 32, 1>(a, ta, bid, smem);
    } else if constexpr (L == 3) {
        if (NEO_ROLES & 4) {
            if (ta.jh == 2) toep_lds_role<32, kT32Band, 2>(a, ta, bid, smem);  // uniform per launch
            else toep_lds_role<32, kT32Band, 1>(a, ta, bid, smem);
        }
    } else {
        if (NEO_ROLES & 4) toep_big_role(a, ta, bid, smem);
    }
    return true;
}

// the lanes past 256 of a larger workgroup: move bid past level L's workgroups (or stop there)
template<int L>
__device__ __forceinline__ bool toep_skip(const slice_args& a, int& bid)
{
    if (L >= a.ntp) return false;
    if (bid >= a.tp[L].nwg) {
        bid -= a.tp[L].nwg;
        return false;
    }
    return true;
}

// The step kernel (k_lvl_step): one launch per block, workgroups by role, the longest chains
// first -- far phase 2, the block itself, the Toeplitz slices (largest window first), far
// phase 1. No role reads what another role of the same launch writes: the block writes FDL
// row w and reads its slabs / far field (finished in earlier launches); the slices read FDL
// rows before the current window and write the next window's slabs / far field.
#ifndef NEO_STEP_WPE
#define NEO_STEP_WPE 3  // waves per SIMD the step kernel is compiled for (VGPR budget: 168)
#endif
// B = 1024 runs 512-lane workgroups (the block role's bin pairs): two waves per SIMD each
// KMAX = 1 (the recomputed far level, far2r_role: 184 VGPRs) runs two waves per SIMD, which also
// leaves a block-kernel wave (136 VGPRs) room beside two slice waves on a SIMD
#ifndef NEO_RAW_WPE
#define NEO_RAW_WPE 2  // diagnostic builds: 3 (the recomputed far level then spills)
#endif
template<int KMAX>
constexpr int slices_wpe() { return KMAX == 1 ? NEO_RAW_WPE : NEO_STEP_WPE; }
template<int B, int KMAX = 2>
constexpr int step_wpe() { return B > 512 ? 2 : (KMAX == 1 ? NEO_RAW_WPE : NEO_STEP_WPE); }
// the roles of one workgroup, in dispatch order (the longest chains first); returns the role
// (timeline builds: 1 far 2b, 2 far 2a, 3 block, 4 + L Toeplitz level L, 9 far phase 1)
#ifndef NEO_ORDER
#define NEO_ORDER 0  // diagnostic builds: 1 far phase 1 before the Toeplitz levels T <= 16, 2 Toeplitz T >= 32 first
#endif
// PART: 0 every role (one launch per step), 1 the block role alone, 2 every role but the block
// (step groups: the block of each call and the level slices of G calls in launches of their own)
template<int B, bool OLA, int KMAX, int PART = 0>
__device__ __forceinline__ int lvl_roles(const slice_args& a, char* smem)
{
    int bid = int(blockIdx.x) + a.bid0;
    auto far2b = [&]() {
        if (bid >= a.f3nwg) {
            bid -= a.f3nwg;
            return false;
        }
        if ((NEO_ROLES & 32) && threadIdx.x < 256) {
            if constexpr (KMAX == 1) far2r_role(a, bid, smem);  // the recomputed far level's build
            else if (a.f2comb) far2c_role<KMAX>(a, bid, smem);  // uniform per launch
            else far2b_role<KMAX>(a, bid, smem);
        }
        return true;
    };
    auto far2a = [&]() {
        if (bid >= a.f2nwg) {
            bid -= a.f2nwg;
            return false;
        }
        if constexpr (KMAX > 1)
            if ((NEO_ROLES & 16) && threadIdx.x < 256) far2a_role(a, bid, smem);
        return true;
    };
    auto block = [&]() {
        if constexpr (PART == 2) return false;
        if (bid >= a.nblk) {
            bid -= a.nblk;
            return false;
        }
        if (NEO_ROLES & 1) block_role<B, OLA>(a, a.blk_c0 + bid, smem);
        return true;
    };
    if constexpr (PART == 1) {  // the block and the levels too short for the background (T < 2 G)
        if (block()) return 3;
        if (threadIdx.x >= 256) return 0;
        if (toep_level<0>(a, bid, smem)) return 4;
        return toep_level<1>(a, bid, smem) ? 5 : 0;
    }
    auto far1 = [&]() {
        if (bid >= a.f1nwg) {
            bid -= a.f1nwg;
            return false;
        }
        if constexpr (KMAX > 1) {  // no phase 1 in the recomputed form
            if ((NEO_ROLES & 8) && threadIdx.x < 256) {
                if (a.f1fpl == 4) far1_role<4, KMAX>(a, bid);
                else if (a.f1fpl == 2) far1_role<2, KMAX>(a, bid);
                else far1_role<1, KMAX>(a, bid);
            }
        }
        return true;
    };
    // Toeplitz level L (window T = kLvT0 << L, plan_levels), one code copy per level; workgroups
    // of more than 256 lanes (B = 1024) take part with their first 256
    auto toep = [&](auto L) { return threadIdx.x < 256 ? toep_level<decltype(L)::value>(a, bid, smem)
                                                       : toep_skip<decltype(L)::value>(a, bid); };
    using L0 = std::integral_constant<int, 0>;
    using L1 = std::integral_constant<int, 1>;
    using L2 = std::integral_constant<int, 2>;
    using L3 = std::integral_constant<int, 3>;
    using L4 = std::integral_constant<int, 4>;
#if NEO_ORDER == 2
    if (toep(L4{})) return 8;
    if (toep(L3{})) return 7;
#endif
    if (far2b()) return 1;
    if (far2a()) return 2;
    if (block()) return 3;
#if NEO_ORDER == 3
    // far phase 1's workgroups spread evenly among the Toeplitz levels' (dispatch in bid order:
    // its HBM-bound loads beside the LDS tiles instead of a tail of their own)
    {
        int A = 0;
#pragma unroll
        for (int l = 0; l < kLvToep; ++l)
            if (l < a.ntp) A += a.tp[l].nwg;
        const int F = a.f1nwg, N = A + F;
        if (F > 0 && bid < N) {
            const int f0 = int(int64_t(bid) * F / N), f1 = int(int64_t(bid + 1) * F / N);
            if (f1 > f0) {
                bid = f0 + A;  // the far1 lambda below subtracts the Toeplitz workgroups first
            } else {
                bid -= f0;
            }
        }
    }
#endif
#if NEO_ORDER != 2
    if (toep(L4{})) return 8;
    if (toep(L3{})) return 7;
#endif
#if NEO_ORDER == 1
    if (far1()) return 9;
#endif
    if (toep(L2{})) return 6;
    if (toep(L1{})) return 5;
    if (toep(L0{})) return 4;
#if NEO_ORDER != 1
    if (far1()) return 9;
#endif
    return 0;
}

// LDS of the block role alone: the block's spectrum, the transform buffer, the twiddles
template<int B>
constexpr int block_lds() { return (B + upols_cfg<B>::LL + upols_cfg<B>::TW1 + upols_cfg<B>::TW2) * int(sizeof(cf)); }

// step groups: the block role of one step (the caller's stream) and the slice of the 4-block
// Toeplitz level where G = 4 (toep_role<4>: no LDS); the block's LDS only -- more workgroups
// resident per CU than the step kernel's 53.8 KB tile allows
#ifndef NEO_BLOCK_PRIO
#define NEO_BLOCK_PRIO 0
#endif
#ifndef NEO_BLOCK_WPE
#define NEO_BLOCK_WPE 1
#endif
#ifdef NEO_TIMELINE  // diagnostic builds: per-workgroup start / end (100 MHz clock) and role
template<int WG, class F>
__device__ __forceinline__ void tl_record(const slice_args& a, F roles)
{
    const unsigned long long t0 = wall_clock64();
    const int role = roles();
    if constexpr (WG > 256) return;  // lanes past 256 leave the roles early: no final barrier
    __syncthreads();
    if (threadIdx.x == 0 && a.tl) {
        unsigned long long* r = static_cast<unsigned long long*>(a.tl) + 4 * int64_t(blockIdx.x);
        r[0] = t0;
        r[1] = wall_clock64();
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15;  // HW_REG_XCC_ID
        r[2] = (unsigned long long)(role) | ((unsigned long long)(__smid()) << 32) | ((unsigned long long)(xcc) << 56);
    }
}
#define NEO_TL_ROLES(WG, EXPR) tl_record<WG>(a, [&] { return EXPR; })
#else
#define NEO_TL_ROLES(WG, EXPR) (void)(EXPR)
#endif

template<int B, bool OLA>
__global__ __launch_bounds__(lstep_cfg<B>::WG) __attribute__((amdgpu_waves_per_eu(NEO_BLOCK_WPE))) void k_lvl_block(slice_args a)
{
    __shared__ __attribute__((aligned(16))) char smem[block_lds<B>()];
    if constexpr (NEO_BLOCK_PRIO > 0) __builtin_amdgcn_s_setprio(NEO_BLOCK_PRIO);
    NEO_TL_ROLES(lstep_cfg<B>::WG, (lvl_roles<B, OLA, 2, 1>(a, smem)));
}

// step groups: every role but the block for the slices of G steps (the background stream);
// 256 lanes (the roles' geometry), the step kernel's register budget
template<int KMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(slices_wpe<KMAX>()))) void k_lvl_slices(slice_args a)
{
    __shared__ __attribute__((aligned(16))) char smem[kSliceLds];
    NEO_TL_ROLES(256, (lvl_roles<512, false, KMAX, 2>(a, smem)));
}

template<int B, bool OLA, int KMAX>
__global__ __launch_bounds__(lstep_cfg<B>::WG) __attribute__((amdgpu_waves_per_eu(step_wpe<B, KMAX>()))) void k_lvl_step(slice_args a)
{
    __shared__ __attribute__((aligned(16))) char smem[kSliceLds];
    NEO_TL_ROLES(lstep_cfg<B>::WG, (lvl_roles<B, OLA, KMAX>(a, smem)));
}

// Segment spectra (grid C x NSEG x B/16): hf[c][s][f][k] = DFT256 over r < 128 of
// H[c][128 (s + seg0) + r][k] (zero past P); packed bin 0 (two real sequences, DC and Nyquist)
// in the real-FFT packing of far_role (pack_bin0). seg0 = 2: the far level's segments (p >=
// 256); 0: every segment (offline windows, k_off_mac).
__global__ __launch_bounds__(256) void k_lvf_filter(const cf* __restrict__ H, cf* __restrict__ hf,
                                                    const cf* __restrict__ twg, int B, int P, int nseg,
                                                    int64_t cstride, int64_t pstride, int seg0, int64_t hcs)
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
        const int r = a + 16 * n2, p = (s + seg0) * kFarT + r;
        v[n2] = (r < kFarT && p < P) ? H[int64_t(c) * cstride + int64_t(p) * pstride + k] : cf{0.f, 0.f};
    }
    col_fft<-1, 16>(v, lds, tw, a, cp, true);
    if (g == 0) {  // uniform per workgroup
        if (cp == 0) {
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) z[16 * k1 + a] = v[k1];
        }
        __syncthreads();
        if (cp == 0) {
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) {
                const int f = 16 * k1 + a;
                v[k1] = pack_bin0(v[k1], z[(kFN - f) & (kFN - 1)], f);
            }
        }
    }
    cf* dst = hf + int64_t(c) * hcs + int64_t(s) * kFN * B + k;
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) dst[int64_t(16 * k1 + a) * B] = v[k1];
}

// ---------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------
// host side

// phase 1 f rows per lane: one load round covers the stored segments (far1_role)
static int far1_fpl(const upols_t* h)
{
#ifdef NEO_FAR_FPL  // diagnostic builds
    return NEO_FAR_FPL;
#endif
    return h->lv.nseg - 1 <= 4 ? 4 : (h->lv.nseg - 1 <= 8 ? 2 : 1);
}

static int64_t far_units(const upols_t* h) { return int64_t(h->C) * (h->B / 16); }

// windows per far phase-1 pass (far1_mac): K ~ sqrt(2 (nseg - 1)) minimizes the spectra read per
// window and column, 2 (nseg - 1) / K + K - 1; but phase 2 takes up to K - 1 extra segments in
// its one-workgroup-per-unit chain, which bounds the step where a step has few far units
// (measured: K = 3 / 4 instead of 2 at 64 / 32 units per step, C5 / C4: 13 % / 25 % slower; at
// 512, the 2048-channel headline: 3 % faster; round 5, the 4-GPU shard of the headline, 512
// channels = 128 units per step: K = 3 2-3.5 % faster, tools/gpu_shard_sweep.sh), so K = 2 below
// kFarGroupUnits units
constexpr int64_t kFarGroupUnits = 16384;  // 128 units per step

static int far_group_auto(int C, int B, int ns)
{
    if (ns < 2) return 1;
    if (int64_t(C) * (B / 16) < kFarGroupUnits) return 2;
    const int K = int(std::lround(std::sqrt(2.0 * (ns - 1))));
    return std::min(kFarKMax, std::max(2, K));
}

int far_group_for(int C, int B, int P)
{
    level_plan lp;
    plan_levels(P, lp);
    return lp.nseg ? far_group_auto(C, B, lp.nseg) : 0;
}

static int far_group(const upols_t* h)
{
    const int ns = h->lv.nseg;
    if (ns < 2 || h->far_raw) return 1;  // recomputed: every window on its own
    if (h->far_k) return h->far_k;  // neo_hip_upols_opts.far_group (tests, A/B runs)
    return far_group_auto(h->C, h->B, ns);
}

// far phase 1 over the slice units [u0, u1): mode 0 one window per group, 1 only the groups of
// class cls (K windows each), 2 every group (class cls: K windows; classes not started: one)
__host__ __device__ inline void far1_range_k(slice_args& a, int u0, int u1, int mode, int cls, int K, int fpl)
{
    a.f1u0 = u0;
    a.f1u1 = u1;
    a.f1fpl = fpl;
    a.f1mode = mode;
    a.f1cls = cls;
    a.f1nwg = 0;
    if (u1 <= u0) return;
    const int ga = u0 / kF1UG, gb = (u1 - 1) / kF1UG;  // groups holding slice units
    a.f1g0 = mode == 1 ? ga + ((cls - ga % K) % K + K) % K : ga;
    a.f1gs = mode == 1 ? K : 1;
    const int ng = a.f1g0 > gb ? 0 : (gb - a.f1g0) / a.f1gs + 1;
    a.f1nwg = ng * (kFN / (4 * fpl));
}

static void far1_range(const upols_t* h, slice_args& a, int u0, int u1, int mode, int cls)
{
    far1_range_k(a, u0, u1, mode, cls, far_group(h), far1_fpl(h));
}

// Latency mode's far level (persist_far): the far work of step n (block t0 + n, ring row w) in the
// one-launch schedule, with kFarT - 2 slices (one more step of slack: the field of window W is
// complete two steps before its first block, as the Toeplitz slabs): phase 1 of slice q and phase 2
// (far2c_role) of slice q - 1 of window W = n / kFarT + 1 at q = n mod kFarT
__host__ __device__ inline void persist_far_args(slice_args& a, int64_t n, int w, int U, int K, int fpl, cf* ff)
{
    constexpr int ns = kFarT - 2;
    const int64_t W = n / kFarT + 1;
    const int q = int(n % kFarT);
    a.f1nwg = a.f2nwg = a.f3nwg = 0;
    if (q < ns) {
        a.f1wn = int(W);
        far1_range_k(a, int(int64_t(q) * U / ns), int(int64_t(q + 1) * U / ns), K == 1 ? 0 : (W < K ? 2 : 1),
                     int(W % K), K, fpl);
    }
    if (q >= 1 && q <= ns) {
        a.f3u0 = int(int64_t(q - 1) * U / ns);
        a.f3nwg = int(int64_t(q) * U / ns) - a.f3u0;
        a.f3wn = int(W);
        a.f2grp = K > 1;
        a.f3ff = ff + (W & 1) * int64_t(a.C) * ff_cs(a.B);
        const int64_t t = (int64_t(w) + W * kFarT - n) % a.ring;
        a.f2tw = int(t < 0 ? t + a.ring : t);
        a.f2comb = 1;
    }
}

// device buffers of the level pipeline (allocated on the first streaming step), all or none
static int lvl_buffers(upols_t* h)
{
    if (h->lv_ready) return NEO_HIP_OK;
    const level_plan& lp = h->lv;
    const size_t C = size_t(h->C), B = size_t(h->B);
    std::vector<void**> got;
    auto alloc = [&](void** p, size_t bytes) {
        if (dalloc(p, bytes) != NEO_HIP_OK) return false;
        got.push_back(p);
        return true;
    };
    auto undo = [&](const char* what, size_t bytes) {
        for (void** p : got) {
            dfree(*p);
            *p = nullptr;
        }
        return fail(NEO_HIP_ENOMEM, "level pipeline: allocation of %s (%zu bytes) failed", what, bytes);
    };
    for (int l = 0; l < lp.n; ++l) {
        const size_t bytes = 2 * C * size_t(slab_cs(lp.T[l], int(B))) * sizeof(cf);
        if (!alloc(reinterpret_cast<void**>(&h->lv_slab[l]), bytes)) return undo("level slabs", bytes);
    }
    if (lp.nseg) {
        const size_t spec = C * size_t(spec_cs(lp.nseg, int(B))) * sizeof(cf);
        const size_t ffb = 2 * C * size_t(ff_cs(int(B))) * sizeof(cf);
        if (!h->far_raw) {  // the stored form: segment and row-pair spectra, phase 1 -> 2 partial sums
            if (!alloc(reinterpret_cast<void**>(&h->fv_hf), spec)) return undo("far segment spectra", spec);
            if (!alloc(reinterpret_cast<void**>(&h->fv_xf), spec)) return undo("far FDL spectra", spec);
            const size_t accb = size_t(far_group(h)) * size_t(far_units(h)) * kFN * 16 * sizeof(cf);
            if (!alloc(reinterpret_cast<void**>(&h->fv_acc), accb)) return undo("far partial sums", accb);
        }
        if (!alloc(reinterpret_cast<void**>(&h->fv_ff), ffb)) return undo("far field", ffb);
        if (shared_far_tw(&h->fv_tw) != NEO_HIP_OK) return undo("far twiddles", kFN * sizeof(cf));
        h->fv_dirty = true;
    }
    h->lv_ready = true;
    return NEO_HIP_OK;
}

void lvl_free(upols_t* h)
{
    if (h->bg) {  // slices still in flight read and write the buffers freed below
        (void)hipStreamSynchronize(h->bg);
        (void)hipStreamDestroy(h->bg);
        h->bg = nullptr;
        for (hipEvent_t* e : {&h->ev_blk, &h->ev_sl[0], &h->ev_sl[1], &h->ev_join, &h->ev_pc[0], &h->ev_pc[1]}) {
            (void)hipEventDestroy(*e);
            *e = nullptr;
        }
        h->bg_busy = false;
    }
    for (auto& p : h->lv_slab) {
        dfree(p);
        p = nullptr;
    }
    for (cf** p : {&h->fv_hf, &h->fv_xf, &h->fv_ff, &h->fv_acc}) {
        dfree(*p);
        *p = nullptr;
    }
    h->fv_tw = nullptr;  // shared (shared_far_tw)
    h->lv_ready = false;
}

// the filter changed: the far segment spectra are recomputed before the next streaming step
// (and the offline windows' before the next offline pass)
void lvl_filter_changed(upols_t* h)
{
    h->fv_dirty = true;
    h->off_dirty = true;
    h->lv_n = -1;
}

static int ring_add(int64_t r, int64_t d, int R) { return int(((r + d) % R + R) % R); }

// Toeplitz role geometry per window T (k_lvl_step's level roles): window parts per column
// group and units per workgroup. T = 32 splits its window in two where a step has fewer than
// 8 of its units (few channels: the part halves the step's longest chain).
int toep_split_for(int C, int B) { return C * (B / 16) < 8 * 32 ? 2 : 1; }

// steps per background launch of the level slices (launch_levels): 4 from kStepGroupUnits
// 16-column units (same-box A/B, ms per step at G = 1 / 4: C5 0.0183 / 0.0165, C4 0.0155 / 0.0134,
// c5full 0.1213 / 0.1215 with the host round trip per block 133 -> 63 us; at one channel, C3, the
// block launch and the cross-stream waits cost more than the overlap gives: 0.0063 / 0.0083)
constexpr int64_t kStepGroupUnits = 2048;

int bg_pad_for(int C, int B) { return int64_t(C) * (B / 16) <= 4096 ? 1024 : 0; }

int step_group_for(int C, int B, int P)
{
    (void)P;
    return int64_t(C) * (B / 16) >= kStepGroupUnits && B <= 1024 ? 4 : 1;
}

static void toep_geom(const upols_t* h, int T, int& JH, int& UPW)
{
    JH = T == kBigT ? kBigJH : (T == 32 ? (h->toep_jh ? h->toep_jh : toep_split_for(h->C, h->B)) : 1);
    UPW = T <= 8 ? 16 : (T <= 32 ? 32 / T : 1);  // toep_role<T, 2T, 1, 1>: 16 units; toep_tile: 32 / T
}

static slice_args base_args(const upols_t* h)
{
    slice_args a{};
    a.H = h->H;
    a.fdl = h->fdl;
    a.ring = h->ring;
    a.C = h->C;
    a.B = h->B;
    a.cstride = h->cstride;
    a.pstride = h->pstride;
    if (h->lv.nseg) {
        a.M = h->lv.nseg;
        a.nseg = h->lv.nseg;
        a.fsc = spec_cs(h->lv.nseg, h->B);
        a.fcs = ff_cs(h->B);
        a.fnfresh = 1;
        a.fU = int(far_units(h));
        a.fK = far_group(h);
        a.f1acc = h->fv_acc;
        a.f2acc = h->fv_acc;
        a.hf = h->fv_hf;
        a.xf = h->fv_xf;
        a.twf = h->fv_tw;
        a.P = h->P;
    }
    return a;
}

#ifdef NEO_TIMELINE
// diagnostic builds: the records of the last step-kernel launch of a handle
static void* g_tl_buf[3] = {};  // timeline records of the last launch of each part (0 step, 1 block, 2 slices)
static int64_t g_tl_nn[3] = {}, g_tl_capp[3] = {};
#endif

static unsigned launch_grid(const slice_args& a)
{
    unsigned t = unsigned(a.f3nwg + a.f2nwg + a.nblk + a.f1nwg);
    for (int l = 0; l < a.ntp; ++l) t += unsigned(a.tp[l].nwg);
    return t;
}

// kernel of a launch: part 0 the step kernel (every role), 1 the block alone, 2 the slices alone
static int launch_step_kernel(const upols_t* h, const slice_args& a_in, hipStream_t s, int part = 0,
                              int piece = 0, int pieces = 1)
{
    slice_args a = a_in;
    unsigned grid = launch_grid(a);
    if (pieces > 1) {  // workgroups [piece grid / pieces, (piece + 1) grid / pieces) of the launch
        const unsigned g0 = unsigned(uint64_t(grid) * piece / pieces), g1 = unsigned(uint64_t(grid) * (piece + 1) / pieces);
        a.bid0 = int(g0);
        grid = g1 - g0;
    }
    if (!grid) return NEO_HIP_OK;
#ifdef NEO_TIMELINE
    if (int64_t(grid) > g_tl_capp[part]) {
        (void)hipFree(g_tl_buf[part]);
        g_tl_capp[part] = int64_t(grid) * 2;
        NEO_HIP_CHECK(hipMalloc(&g_tl_buf[part], size_t(g_tl_capp[part]) * 32));
        NEO_HIP_CHECK(hipMemset(g_tl_buf[part], 0, size_t(g_tl_capp[part]) * 32));
    }
    a.tl = g_tl_buf[part];
    g_tl_nn[part] = grid;
#endif
    // pairs-only build where the window group is <= 2 (fewer VGPRs: every shape below
    // kFarGroupUnits), else the build for any group
    const bool pairs = a.fK <= 2, raw = h->far_raw;
    if (part == 1) {
        if (h->ola) {
            NEO_UPOLS_DISPATCH(h->B, if constexpr (BB <= 1024) hipLaunchKernelGGL((k_lvl_block<BB, true>), dim3(grid),
                                                                                  dim3(lstep_cfg<BB>::WG), 0, s, a))
        } else {
            NEO_UPOLS_DISPATCH(h->B, if constexpr (BB <= 1024) hipLaunchKernelGGL((k_lvl_block<BB, false>), dim3(grid),
                                                                                  dim3(lstep_cfg<BB>::WG), 0, s, a))
        }
    } else if (part == 2) {
        // 1 KB of dynamic LDS holds the slices kernel to two workgroups per CU (three by its 53.8 KB
        // of static LDS and 149 VGPRs), leaving room for block workgroups beside it: where the
        // chain of block launches bounds the step (C4: 256 ch x B = 256) they are no longer held
        // back until slice workgroups end (same-box A/B, 128 steps, two repetitions: C4 10.95 /
        // 10.97 -> 10.24 / 10.39 us per step, C5 15.9 / 15.7 -> 15.5 / 15.8, c5full 107.0 /
        // 107.7 -> 115.3 / 114.3: only at the smaller shapes, bg_pad_for)
#ifdef NEO_BG_LDS_PAD  // diagnostic builds: force the padding
        const unsigned pad = NEO_BG_LDS_PAD;
#else
        const unsigned pad = h->bg_pad;
#endif
        if (raw) hipLaunchKernelGGL((k_lvl_slices<1>), dim3(grid), dim3(256), pad, s, a);
        else if (pairs) hipLaunchKernelGGL((k_lvl_slices<2>), dim3(grid), dim3(256), pad, s, a);
        else hipLaunchKernelGGL((k_lvl_slices<kFarKMax>), dim3(grid), dim3(256), pad, s, a);
    } else {
#define NEO_LVL(OL, KM)                                                                                        \
    NEO_UPOLS_DISPATCH(h->B, if constexpr (BB <= 1024) hipLaunchKernelGGL((k_lvl_step<BB, OL, KM>), dim3(grid), \
                                                                         dim3(lstep_cfg<BB>::WG), 0, s, a))
        if (h->ola) {
            if (raw) NEO_LVL(true, 1) else if (pairs) NEO_LVL(true, 2) else NEO_LVL(true, kFarKMax)
        } else {
            if (raw) NEO_LVL(false, 1) else if (pairs) NEO_LVL(false, 2) else NEO_LVL(false, kFarKMax)
        }
#undef NEO_LVL
    }
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

// The far level's units are cut into slices per window. G = 1: kFarT - 1 slices, slice q of
// window W runs phase 1 and 2a at step q of window W - 1 (2a reads FDL rows up to the last block
// before that window) and 2b at step q + 1 (<= the window's last: the far field is complete when
// window W's first block runs). G > 1 (step groups, slice_part): kFarT / G - 2 slices, phase 1
// of slice q at step group q + 1 of window W - 1 (its launch waits only for the blocks before the
// previous group), phase 2 (far2c_role: 2a and 2b in one workgroup) at group q + 2.
static int far_nslices(const upols_t* h) { return h->sg == 1 ? kFarT - 1 : kFarT / h->sg - 2; }

static int far_u(int64_t U, int q, int ns) { return int(q * U / ns); }

// the first unit of far slice q: step groups take the planned cuts (part_plan), G = 1 equal slices
static int far_cut(const upols_t* h, int q)
{
    if (!h->fv_cut.empty()) return h->fv_cut[size_t(q)];
    return far_u(int64_t(h->C) * (h->B / 16), q, h->sg == 1 ? kFarT - 1 : kFarT / h->sg - 2);
}

// far phase 1 for slice q of window W: the unit groups of class W mod K for the windows
// W .. W + K - 1 (far1_mac); in the first windows after priming (W < K) the classes that have
// not started, for window W alone
static void far1_args(const upols_t* h, int64_t W, int q, slice_args& a)
{
    const int K = far_group(h);
    a.f1wn = int(W);
    far1_range(h, a, far_cut(h, q), far_cut(h, q + 1), K == 1 ? 0 : (W < K ? 2 : 1), int(W % K));
}

// the recomputed far level's slice q of window W (far2r_role), issued at step n (block t0 + n at
// ring row w): every unit of the slice computes the window's field from rows before t_W - 128
static void far_raw_args(const upols_t* h, int64_t W, int q, int w, int64_t n, slice_args& a)
{
    a.f3u0 = far_cut(h, q);
    a.f3nwg = far_cut(h, q + 1) - a.f3u0;
    a.f3wn = int(W);
    a.f3ff = h->fv_ff + (W & 1) * h->C * ff_cs(h->B);
    a.f2tw = ring_add(w, W * kFarT - n, h->ring);
    a.f2comb = 2;
}

// Step groups: the background levels' window offsets and part sizes. A window's first group
// carries none of its level's parts (they read the window's rows), so with every window starting at
// a multiple of its length the groups at multiples of 8 (G = 4) had no Toeplitz work at all and
// the odd ones all of the 8-block level's: background launches of 0.9 to 2.1 GB at c5full, and a
// 20-step sample of the stream 5-8 % above or below the far window's mean. So a level of window
// T >= 4 G (up to 32 blocks: its prime reads at most 16 rows further back) starts its windows half a
// window later (phi = T / 2; still at even groups, which the events need), which puts the groups it
// skips apart from every other level's (2 G: odd groups carry it, 4 G: skips 2 mod 4, 8 G: 4 mod 8,
// the far level: 0 mod kFarT / G); and each window's units are cut into parts of unequal sizes so
// that, over a cycle of groups (the far window, else the longest level window), every group's
// background bytes come as close to equal as the slots allow: min-max water filling of one window
// at a time against the rest (the far slices' bytes fixed), swept until it settles.
static int part_phi(int T, int G, bool bg) { return bg && G > 1 && T >= 4 * G && T <= 32 ? T / 2 : 0; }

struct part_level {
    int T = 0, UPW = 1;
    bool bg = false;
    int64_t U = 0;
    double wbytes = 0;  // bytes per window
};

// phi, cycle length (groups), cuts [k][j] (k < cyc / (T / G) windows of the cycle, j <= T / G - 1)
// per level and the far slices' unit cuts fcut[0 .. ns] (ns > 0); loads: the predicted background
// bytes per group of the cycle (null: not wanted). balance = false: equal parts, no offsets.
static void part_plan(const part_level* lv, int nl, int G, int64_t FU, int ns, double c1, double c2, bool far_raw,
                      bool balance, int* phi, int& cyc, std::vector<int>* cut, std::vector<int>& fcut,
                      std::vector<double>* loads)
{
    cyc = 1;
    for (int l = 0; l < nl; ++l) {
        phi[l] = balance ? part_phi(lv[l].T, G, lv[l].bg) : 0;
        cut[l].clear();
        if (lv[l].bg) cyc = std::max(cyc, lv[l].T / G);
    }
    if (ns) cyc = std::max(cyc, kFarT / G);
    // the far slices (slice_part): slice q's phase 1 at group q + 1, phase 2 at q + 2 (recomputed:
    // all of it at q + 2), s[q] units each
    std::vector<double> fs(size_t(ns), ns ? double(FU) / ns : 0.0), load(size_t(cyc), 0.0);
    auto far_add = [&](std::vector<double>& L, const std::vector<double>& sq, double sign) {
        for (int q = 0; q < ns; ++q) {
            if (!far_raw) L[size_t(q + 1)] += sign * c1 * sq[size_t(q)];
            L[size_t(q + 2)] += sign * c2 * sq[size_t(q)];
        }
    };
    far_add(load, fs, 1.0);
    struct win {
        int l, np;
        double c;
        std::vector<int> grp;
        std::vector<double> x;  // units per part
    };
    std::vector<win> ws;
    for (int l = 0; l < nl; ++l) {
        if (!lv[l].bg || lv[l].U <= 0) continue;
        const int Tg = lv[l].T / G, np = Tg - 1, s0 = ((-phi[l] / G) % Tg + Tg) % Tg;
        for (int k = 0; k < cyc / Tg; ++k) {
            win w{l, np, lv[l].wbytes / double(lv[l].U), {}, std::vector<double>(size_t(np), double(lv[l].U) / np)};
            for (int j = 1; j <= np; ++j) w.grp.push_back((s0 + k * Tg + j) % cyc);
            for (int j = 0; j < np; ++j) load[size_t(w.grp[size_t(j)])] += w.c * w.x[size_t(j)];
            ws.push_back(std::move(w));
        }
    }
    std::vector<double> base, sb, grad, y;
    for (int round = 0; round < (balance ? 4 : 0); ++round) {
        // the Toeplitz windows, one at a time against the rest: min-max water filling
        for (int sweep = 0; sweep < 32; ++sweep)
            for (auto& w : ws) {
                const int np = w.np;
                base.assign(size_t(np), 0.0);
                for (int j = 0; j < np; ++j) {
                    load[size_t(w.grp[size_t(j)])] -= w.c * w.x[size_t(j)];
                    base[size_t(j)] = load[size_t(w.grp[size_t(j)])];
                }
                sb = base;
                std::sort(sb.begin(), sb.end());
                const double total = w.c * double(lv[w.l].U);
                double h = sb[0], acc = 0;  // water level: sum of max(0, h - base) = the window's bytes
                for (int i = 0; i < np; ++i) {
                    const double next = i + 1 < np ? sb[size_t(i + 1)] : 1e300;
                    const double need = (next - sb[size_t(i)]) * (i + 1);
                    if (acc + need >= total) {
                        h = sb[size_t(i)] + (total - acc) / (i + 1);
                        break;
                    }
                    acc += need;
                }
                for (int j = 0; j < np; ++j) {
                    w.x[size_t(j)] = std::max(0.0, h - base[size_t(j)]) / w.c;
                    load[size_t(w.grp[size_t(j)])] += w.c * w.x[size_t(j)];
                }
            }
        if (!ns) break;
        // the far slices against the rest: least squares around the mean, projected gradient on
        // {s >= 0, sum s = FU} (the min-max recurrence is unstable: phase 2 bytes > phase 1's)
        double mean = 0;
        for (double v : load) mean += v;
        mean /= cyc;
        const double eta = 1.0 / (2.0 * (c1 + c2) * (c1 + c2));
        for (int it = 0; it < 400; ++it) {
            grad.assign(size_t(ns), 0.0);
            for (int q = 0; q < ns; ++q) {
                if (!far_raw) grad[size_t(q)] += 2 * c1 * (load[size_t(q + 1)] - mean);
                grad[size_t(q)] += 2 * c2 * (load[size_t(q + 2)] - mean);
            }
            far_add(load, fs, -1.0);
            y.resize(size_t(ns));
            for (int q = 0; q < ns; ++q) y[size_t(q)] = fs[size_t(q)] - eta * grad[size_t(q)];
            sb = y;  // projection onto the simplex: subtract tau, clip at 0
            std::sort(sb.begin(), sb.end(), std::greater<double>());
            double cs = 0, tau = 0;
            for (int i = 0; i < ns; ++i) {
                cs += sb[size_t(i)];
                const double t = (cs - double(FU)) / (i + 1);
                if (sb[size_t(i)] - t > 0) tau = t;
            }
            for (int q = 0; q < ns; ++q) fs[size_t(q)] = std::max(0.0, y[size_t(q)] - tau);
            far_add(load, fs, 1.0);
        }
    }
    for (int l = 0; l < nl; ++l)
        if (lv[l].bg) cut[l].assign(size_t(cyc / (lv[l].T / G) * (lv[l].T / G)), 0);
    std::vector<int> kcount(size_t(nl), 0);
    for (const auto& w : ws) {  // cuts on workgroup multiples, the last at U
        const int64_t U = lv[w.l].U, q = lv[w.l].UPW;
        int* c = cut[w.l].data() + size_t(kcount[size_t(w.l)]++) * size_t(w.np + 1);
        double cum = 0;
        c[0] = 0;
        for (int j = 1; j <= w.np; ++j) {
            cum += w.x[size_t(j - 1)];
            const int64_t r = j == w.np ? U : std::min<int64_t>(U, std::llround(cum / double(q)) * q);
            c[j] = int(std::max<int64_t>(c[j - 1], r));
        }
    }
    fcut.assign(ns ? size_t(ns + 1) : 0, 0);
    if (ns) {
        double cum = 0;
        for (int q = 1; q <= ns; ++q) {
            cum += fs[size_t(q - 1)];
            const int64_t r = q == ns ? FU : std::min<int64_t>(FU, std::llround(cum));
            fcut[size_t(q)] = int(std::max<int64_t>(fcut[size_t(q - 1)], r));
        }
    }
    if (loads) {  // from the integer cuts
        loads->assign(size_t(cyc), 0.0);
        std::vector<double> fi(static_cast<size_t>(ns));
        for (int q = 0; q < ns; ++q) fi[size_t(q)] = double(fcut[size_t(q + 1)] - fcut[size_t(q)]);
        far_add(*loads, fi, 1.0);
        std::fill(kcount.begin(), kcount.end(), 0);
        for (const auto& w : ws) {
            const int* c = cut[w.l].data() + size_t(kcount[size_t(w.l)]++) * size_t(w.np + 1);
            for (int j = 1; j <= w.np; ++j) (*loads)[size_t(w.grp[size_t(j - 1)])] += w.c * double(c[j] - c[j - 1]);
        }
    }
}

static int64_t toep_units(const upols_t* h, int T);
static bool block_level(const upols_t* h, int T);

// the handle's plan (lvl_prime): levels, far slices and their bytes as bench.algorithmic_bytes
// counts them
static void plan_handle_parts(upols_t* h, std::vector<double>* loads = nullptr, bool balance = true)
{
    const level_plan& lp = h->lv;
    part_level pl[kLvToep];
    const double CB = double(h->C) * h->B;
    for (int l = 0; l < lp.n; ++l) {
        int JH, UPW;
        toep_geom(h, lp.T[l], JH, UPW);
        pl[l].T = lp.T[l];
        pl[l].UPW = UPW;
        pl[l].bg = h->sg > 1 && !h->persist && !block_level(h, lp.T[l]);  // latency mode: its own schedule
        pl[l].U = toep_units(h, lp.T[l]);
        pl[l].wbytes = CB * 8 * (2.0 * (lp.b[l] - lp.a[l]) + 2 * lp.T[l] - 1);
    }
    const int ns = h->sg > 1 && !h->persist && lp.nseg ? far_nslices(h) : 0;
    const int64_t FU = far_units(h);
    double c1 = 0, c2 = 0;  // bytes per far unit (16 columns) of phase 1 and 2 per window
    if (ns) {
        const int K = far_group(h), nseg = lp.nseg;
        if (h->far_raw) {
            c2 = 16.0 * 8 * ((nseg + 1) * 128.0 + (h->P - 256) + 128);
        } else {
            c1 = 16.0 * 8 * (256.0 * 2 * (nseg - 1) / K + 256);     // stored spectra, partial sums out
            c2 = 16.0 * 8 * (256.0 * (3 + K - 1) + 128 + 256);       // fresh pair, products, field, sums in
        }
    }
    part_plan(pl, lp.n, h->sg, FU, ns, c1, c2, h->far_raw, balance, h->lv_phi, h->lv_cyc, h->lv_cut, h->fv_cut, loads);
}

// The block role of step n (block t0 + n at FDL ring row w) for the channels [c0, c0 + nc): its
// slab row of every Toeplitz level and its far-field row (windows finished in earlier launches)
static void block_part(const upols_t* h, int64_t n, int w, int c0, int nc, const float* in, int64_t ld_in, float* out,
                       int64_t ld_out, slice_args& a)
{
    const level_plan& lp = h->lv;
    const int B = h->B, C = h->C;
    a.nblk = nc;
    a.blk_c0 = c0;
    a.in = in;
    a.ld_in = ld_in;
    a.out = out;
    a.ld_out = ld_out;
    a.prev = h->prev;
    a.twg = h->tw;
    a.w = w;
    a.a0 = lp.a0;
    for (int l = 0; l < lp.n; ++l) {
        const int T = lp.T[l];
        const int64_t m = n + h->lv_phi[l];  // window m / T, its row m mod T
        a.sl[a.nsl] = h->lv_slab[l] + (m / T & 1) * C * slab_cs(T, B) + (m % T) * B;
        a.scs[a.nsl++] = slab_cs(T, B);
    }
    if (lp.nseg) {
        a.ff = h->fv_ff + (n / kFarT & 1) * C * ff_cs(B) + (n % kFarT) * B;
        a.fcs = ff_cs(B);
    }
}

// A Toeplitz level's slice: units [u0, u1) of window W (first block t0 + W T) into its slab buffer
static void toep_slice(const upols_t* h, int l, int64_t W, int64_t u0, int64_t u1, int64_t n, int w, slice_args& a)
{
    const int T = h->lv.T[l];
    int JH, UPW;
    toep_geom(h, T, JH, UPW);
    toep_arg& ta = a.tp[l];  // slot l = level l (the kernel dispatches on it), empty slices allowed
    ta.u0 = int(u0);
    ta.u1 = int(u1);
    ta.slab = h->lv_slab[l] + (W & 1) * h->C * slab_cs(T, h->B);
    ta.cs = slab_cs(T, h->B);
    ta.T = T;
    ta.a = h->lv.a[l];
    ta.b = h->lv.b[l];
    ta.tw = ring_add(w, W * T - n, h->ring);  // block t0 + n at row w
    ta.nwg = ta.u1 > ta.u0 ? (ta.u1 - ta.u0 + UPW - 1) / UPW : 0;
    ta.jh = JH;
    a.ntp = std::max(a.ntp, l + 1);
}

// Far phase 2 at G = 1 in one workgroup per unit (far2c_role, one step after phase 1) or in
// two (2a: the fresh transform -> its slot, beside phase 1; 2b: the products and the inverse one
// step later). One workgroup reads the fresh spectrum back from registers instead of its slot,
// fewer bytes; two halve the chain, which bounds the step where a step has few far units.
// Step groups always run one (their background launches have a group of slack).
constexpr int64_t kFarWholeUnits = 32768;  // 256 units per step

static bool far2_whole(const upols_t* h)
{
    if (h->sg > 1) return true;
    if (h->f2mode) return h->f2mode == 1;  // neo_hip_upols_opts.far_phase2
    return far_units(h) >= kFarWholeUnits;
}

static int64_t toep_units(const upols_t* h, int T)
{
    int JH, UPW;
    toep_geom(h, T, JH, UPW);
    return int64_t(h->C) * (h->B / 16) * JH;
}

// Step groups: the Toeplitz levels stepped in the block launches, 1/T of the next window per step
// (the others in the background launches, T / G - 1 parts per window). T < 2 G must (a background
// launch may not read the blocks of its own group); larger windows may (diagnostic builds).
#ifndef NEO_BLOCK_TMAX
#define NEO_BLOCK_TMAX 0
#endif
static bool block_level(const upols_t* h, int T) { return T < 2 * h->sg || T <= NEO_BLOCK_TMAX; }

// The slices the launch of step n (block t0 + n at ring row w) carries. G = 1: slice n mod T of
// window n / T + 1 of every Toeplitz level (its rows end before the window in progress, so every
// window's slabs are complete when its first block runs) and, with q = n mod 128 and W = n / 128 + 1,
// far phase 1 and 2a of slice q (q < 127) and far phase 2b of slice q - 1 (q >= 1) of window W.
// G > 1, block launches: the levels with T < 2 G, as for G = 1.
static void block_levels(const upols_t* h, int64_t n, int w, slice_args& a)
{
    for (int l = 0; l < h->lv.n; ++l) {
        const int T = h->lv.T[l];
        if (h->sg > 1 && !block_level(h, T)) break;
        const int64_t U = toep_units(h, T), st = n % T;
        toep_slice(h, l, n / T + 1, st * U / T, (st + 1) * U / T, n, w, a);
    }
    if (h->sg > 1 || !h->lv.nseg) return;
    const int64_t U = far_units(h), W = n / kFarT + 1;
    const int q = int(n % kFarT), ns = far_nslices(h);
    if (h->far_raw) {  // recomputed: slice q - 1 of window W whole (far2r_role)
        if (q >= 1 && q <= ns) far_raw_args(h, W, q - 1, w, n, a);
        return;
    }
    if (far2_whole(h)) {  // phase 1 of slice q, phase 2 (far2c_role) of slice q - 1
        if (q < ns) far1_args(h, W, q, a);
        if (q >= 1 && q <= ns) {
            a.f3u0 = far_u(U, q - 1, ns);
            a.f3nwg = far_u(U, q, ns) - a.f3u0;
            a.f3wn = int(W);
            a.f2grp = far_group(h) > 1;
            a.f3ff = h->fv_ff + (W & 1) * h->C * ff_cs(h->B);
            a.f2tw = ring_add(w, W * kFarT - n, h->ring);
            a.f2comb = 1;
        }
        return;
    }
    if (q < ns) {
        a.f2u0 = far_u(U, q, ns);
        a.f2nwg = far_u(U, q + 1, ns) - a.f2u0;
        a.f2tw = ring_add(w, W * kFarT - n, h->ring);
        a.f2wn = int(W);
        far1_args(h, W, q, a);
    }
    if (q >= 1) {
        a.f3u0 = far_u(U, q - 1, ns);
        a.f3nwg = far_u(U, q, ns) - a.f3u0;
        a.f3wn = int(W);
        a.f2grp = far_group(h) > 1;
        a.f3ff = h->fv_ff + (W & 1) * h->C * ff_cs(h->B);
    }
}

// G > 1: the background launch issued at step n0 (a multiple of G; block t0 + n0 at ring row w0).
// It may read only the blocks before n0 - G (it waits for those, not for the group before it), and
// the block launch of step n0 + G waits for it. So a level of window T >= 2 G computes window W + 1
// in T / G - 1 parts at the steps t_W + G j, j = 1 .. T / G - 1 (part j - 1; its rows end at t_W - 1),
// the last due one group before t_{W+1}; the far level's slice q (kFarT / G - 2 of them) runs
// phase 1 at group q + 1 and phase 2 (2a and 2b in one workgroup) at group q + 2 of the window before.
static void slice_part(const upols_t* h, int64_t n0, int w0, slice_args& a)
{
    const level_plan& lp = h->lv;
    const int G = h->sg;
    for (int l = 0; l < lp.n; ++l) {
        const int T = lp.T[l], Tg = T / G;
        if (block_level(h, T)) continue;  // in the block launches
        const int64_t m0 = n0 + h->lv_phi[l], j = (m0 % T) / G, W = m0 / T;  // group j of window W
        if (j < 1) continue;
        const int64_t gw = (W * T - h->lv_phi[l]) / G, cyc = h->lv_cyc;  // window W's first group
        const int k = int((gw % cyc + cyc) % cyc / Tg);
        const int* cut = h->lv_cut[l].data() + size_t(k) * size_t(Tg);  // the window's cuts [0, Tg)
        toep_slice(h, l, W + 1, cut[j - 1], cut[j], m0, w0, a);  // tw from m0: block t_{W+1} = (W + 1) T - phi
    }
    if (lp.nseg && h->far_raw) {  // recomputed: slice q - 2 of window W whole, at phase 2's time
        const int q = int(n0 % kFarT) / G;
        if (q >= 2 && q - 2 < far_nslices(h)) far_raw_args(h, n0 / kFarT + 1, q - 2, w0, n0, a);
    } else if (lp.nseg) {
        const int64_t W = n0 / kFarT + 1;
        const int q = int(n0 % kFarT) / G, ns = far_nslices(h);
        if (q >= 1 && q <= ns) far1_args(h, W, q - 1, a);  // phase 1 of slice q - 1
        if (q >= 2) {  // phase 2 of slice q - 2, 2a and 2b in one workgroup per unit (far2c_role)
            a.f3u0 = far_cut(h, q - 2);
            a.f3nwg = far_cut(h, q - 1) - a.f3u0;
            a.f3wn = int(W);
            a.f2grp = far_group(h) > 1;
            a.f3ff = h->fv_ff + (W & 1) * h->C * ff_cs(h->B);
            a.f2tw = ring_add(w0, W * kFarT - n0, h->ring);
            a.f2comb = 1;
        }
    }
}

// The block role of step n (FDL ring row w) for channel c alone: the same slabs and far-field
// row as that step, input / output blocks of channel c (ld 0: one channel); the kernel that
// ran the step's block (step groups: the block kernel)
int launch_block_only(upols_t* h, int64_t n, int w, int c, const float* in, float* out, hipStream_t s)
{
    if (c < 0 || c >= h->C || n < 0) return fail(NEO_HIP_EINVAL, "block redo: channel %d / step %lld", c, (long long)n);
    slice_args a = base_args(h);
    block_part(h, n, w, c, 1, in, 0, out, 0, a);
    return launch_step_kernel(h, a, s, h->sg > 1 ? 1 : 0);
}

int lvl_join(upols_t* h, hipStream_t s)
{
    if (!h->bg_busy) return NEO_HIP_OK;
    NEO_HIP_CHECK(hipEventRecord(h->ev_join, h->bg));
    NEO_HIP_CHECK(hipStreamWaitEvent(s, h->ev_join, 0));
    h->bg_busy = false;
    return NEO_HIP_OK;
}

// First streaming step after a reset / filter change / batched pass (block t0 at ring row w):
// window 0 of every level, starting at t0, computed whole (all units; the far level
// transforms every segment: phase 1 and 2a in the levels' launch, 2b in a second one).
// After a reset or a filter change (fdl_zero) every FDL row before t0 is zero, and so is every
// value the prime computes from them: Toeplitz windows 0 and 1 (slab[j] = sum over the band,
// p >= 2T, of H[p] X[t_W + j - p]: rows before t0), the far window's row-pair spectra, partial
// sums and field (rows t_W - 128 (q + 1) ... + 255 < t0). Then priming is zeroing the level
// buffers (all of them: a superset of what the two launches write), a fraction of their time.
static int lvl_prime(upols_t* h, hipStream_t s)
{
    const level_plan& lp = h->lv;
    const int B = h->B, C = h->C, w = h->wpos;
    if (int rc = lvl_join(h, s)) return rc;  // slices of an earlier run still in flight on bg
    if (lp.nseg && h->fv_dirty && !h->far_raw) {
        const unsigned grid = unsigned(C) * unsigned(lp.nseg) * unsigned(B / 16);
        hipLaunchKernelGGL(k_lvf_filter, dim3(grid), dim3(256), 0, s, h->H, h->fv_hf, h->fv_tw, B, h->P, lp.nseg,
                           h->cstride, h->pstride, kFarA / kFarT, spec_cs(lp.nseg, B));
        NEO_HIP_LAUNCH_CHECK();
        h->fv_dirty = false;
    }
    plan_handle_parts(h);  // window offsets and background part sizes (step groups)
    if (h->fdl_zero) {
        for (int l = 0; l < lp.n; ++l)
            NEO_HIP_CHECK(hipMemsetAsync(h->lv_slab[l], 0, 2 * size_t(C) * slab_cs(lp.T[l], B) * sizeof(cf), s));
        if (lp.nseg) {
            if (!h->far_raw) {
                const size_t spec = size_t(C) * size_t(spec_cs(lp.nseg, B)) * sizeof(cf);
                NEO_HIP_CHECK(hipMemsetAsync(h->fv_xf, 0, spec, s));
                const size_t accb = size_t(far_group(h)) * size_t(far_units(h)) * kFN * 16 * sizeof(cf);
                NEO_HIP_CHECK(hipMemsetAsync(h->fv_acc, 0, accb, s));
            }
            NEO_HIP_CHECK(hipMemsetAsync(h->fv_ff, 0, 2 * size_t(C) * ff_cs(B) * sizeof(cf), s));
        }
        return NEO_HIP_OK;
    }
    slice_args a = base_args(h), f = base_args(h);  // f: the second launch (far 2b, offset windows 1)
    bool f_any = false;
    for (int l = 0; l < lp.n; ++l) {
        int JH, UPW;
        toep_geom(h, lp.T[l], JH, UPW);
        toep_arg& ta = a.tp[a.ntp++];
        ta.jh = JH;
        ta.slab = h->lv_slab[l];
        ta.cs = slab_cs(lp.T[l], B);
        ta.T = lp.T[l];
        ta.a = lp.a[l];
        ta.b = lp.b[l];
        ta.tw = ring_add(w, -h->lv_phi[l], h->ring);  // window 0 holds step 0: it began phi steps ago
        ta.u0 = 0;
        ta.u1 = C * (B / 16) * JH;
        ta.nwg = (ta.u1 + UPW - 1) / UPW;
        if (h->lv_phi[l]) {  // and window 1 whole: its parts before step 0 never ran (the rest run again)
            toep_arg& t1 = f.tp[l];
            t1 = ta;
            t1.slab = h->lv_slab[l] + size_t(C) * slab_cs(lp.T[l], B);
            t1.tw = ring_add(w, lp.T[l] - h->lv_phi[l], h->ring);
            f.ntp = l + 1;
            f_any = true;
        }
    }
    if (lp.nseg && h->far_raw) {  // recomputed: window 0's field whole, every unit in the same launch
        a.f3u0 = 0;
        a.f3nwg = int(far_units(h));
        a.f3wn = 0;
        a.f3ff = h->fv_ff;
        a.f2tw = w;
        a.f2comb = 2;
    }
    if (lp.nseg && !h->far_raw) {  // far window 0: phase 1 and 2a of every unit beside the levels
        const int U = int(far_units(h));
        a.fnfresh = lp.nseg;  // every segment transformed
        a.f1wn = 0;
        far1_range(h, a, 0, U, 0, 0);  // zero partial sums (no stored segments)
        a.f2u0 = 0;
        a.f2nwg = U;
        a.f2tw = w;
        a.f2wn = 0;
    }
    if (int rc = launch_step_kernel(h, a, s)) return rc;
    if (lp.nseg && !h->far_raw) {  // and 2b of every unit: two launches whatever the shape
        f.fnfresh = lp.nseg;
        f.f3u0 = 0;
        f.f3nwg = int(far_units(h));
        f.f3wn = 0;
        f.f3ff = h->fv_ff;
        f_any = true;
    }
    return f_any ? launch_step_kernel(h, f, s) : NEO_HIP_OK;
}

// background stream and events of the step groups (created on the first grouped step)
static int group_streams(upols_t* h)
{
    if (h->bg) return NEO_HIP_OK;
    int lo = 0, hi = 0;
    NEO_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
#ifdef NEO_BG_PRIO_NORMAL  // diagnostic builds (A/B): the background stream at the default priority
    lo = 0;
#endif
    NEO_HIP_CHECK(hipStreamCreateWithPriority(&h->bg, hipStreamNonBlocking, lo));  // lo: the least urgent
    for (hipEvent_t* e : {&h->ev_blk, &h->ev_sl[0], &h->ev_sl[1], &h->ev_join, &h->ev_pc[0], &h->ev_pc[1]})
        NEO_HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    return NEO_HIP_OK;
}

// One streaming step (block t0 + n, n = lv_n). G = 1: one launch, the block and 1/T of every
// level's next window. G > 1: the block (with the levels of T < 2 G) is a launch of its own on the
// caller's stream; at every G-th step the background stream gets one launch of slices (slice_part),
// after the blocks before the previous group (ev_blk, recorded there), and the block waits for
// the previous group's background launch (ev_sl). With one group of slack on each side neither
// stream waits for the other in steady state. The background launch is issued when its group's
// first call comes, so a block redone before that call (upols_group.hip) is the one it reads.
int launch_levels(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s, float* snap)
{
    int rc = lvl_buffers(h);
    if (rc) return rc;
    if (h->sg > 1 && (rc = group_streams(h))) return rc;
    const bool primed = h->lv_n < 0;
    if (primed) {
        if ((rc = lvl_prime(h, s))) return rc;
        h->lv_n = 0;
        h->pace_prev = false;
        h->pace_seq = 0;
    }
    const int64_t n = h->lv_n;
    const int G = h->sg;
    slice_args a = base_args(h);
    block_part(h, n, h->wpos, 0, h->C, in, ld_in, out, ld_out, a);
    a.snap = snap;
    block_levels(h, n, h->wpos, a);
    if (G > 1 && h->paced) {
        // Paced (neo_hip_upols_set_paced): the group's background launch in np pieces (np = G:
        // one per call; np = 2: at the group's calls 0 and G / 2), piece j covering workgroups
        // [j W / np, (j + 1) W / np) of the same launch (its workgroups are independent); the
        // block of a call that issues a piece waits for the piece issued before it (for piece 0:
        // the previous group's last piece, so the previous group is complete before the group's
        // first block, as without pacing). No block waits for more than one piece of background
        // work: every call costs about the same, at the price of np cross-stream waits per group
        // (the real-time caller's view).
        const int np = h->paced == 2 ? 2 : G, per = G / np;
        const int k = int(n % G);
        const int64_t n0 = n - k;
        const int w0 = ring_add(h->wpos, -k, h->ring);
        const bool odd = (n0 / G) & 1;
        if (k == 0) {
            if (primed) NEO_HIP_CHECK(hipEventRecord(h->ev_blk, s));  // the priming launches
            if (odd || primed) NEO_HIP_CHECK(hipStreamWaitEvent(h->bg, h->ev_blk, 0));
            if (!odd) NEO_HIP_CHECK(hipEventRecord(h->ev_blk, s));  // the blocks before n: the next odd group
        }
        if (k % per == 0) {
            const int j = k / per;
            slice_args b = base_args(h);
            slice_part(h, n0, w0, b);
            if ((rc = launch_step_kernel(h, b, h->bg, 2, j, np))) return rc;
            h->bg_busy = true;
            if (j == np - 1) ++h->bg_launches;
            NEO_HIP_CHECK(hipEventRecord(h->ev_pc[h->pace_seq & 1], h->bg));
            if (h->pace_prev) NEO_HIP_CHECK(hipStreamWaitEvent(s, h->ev_pc[(h->pace_seq - 1) & 1], 0));
            h->pace_prev = true;
            ++h->pace_seq;
        }
    } else if (G > 1 && n % G == 0) {
        // Every background level has T >= 2 G, so its windows (and the far level's) start at
        // multiples of 2 G: a background launch at an odd group (n = G mod 2 G) needs the blocks
        // before n - G, one at an even group only those before n - 2 G (its predecessor on bg
        // waited for them), and only the block of an even group starts windows whose slabs the
        // previous background launch finished. So one cross-stream wait per 2 G steps each way
        // (each costs the waiting queue ~10 us of idle time on MI355X, kernel traces).
        const bool odd = (n / G) & 1;
#ifndef NEO_NO_XWAIT
#define NEO_NO_XWAIT 0  // diagnostic builds (timing only, outputs wrong): 1 drops both cross-stream waits
#endif
        if (primed) NEO_HIP_CHECK(hipEventRecord(h->ev_blk, s));  // the priming launches
        if ((odd && !NEO_NO_XWAIT) || primed) NEO_HIP_CHECK(hipStreamWaitEvent(h->bg, h->ev_blk, 0));
        slice_args b = base_args(h);
        slice_part(h, n, h->wpos, b);
        upols_t::ev_group* eb = nullptr;  // timed when it launches (the first group after a window start may be empty)
        if (launch_grid(b) && ((rc = timing_begin(h, 2, &eb)) || (rc = timing_mark(eb, 0, h->bg)))) return rc;
        if (eb) eb->part = 1;
        if ((rc = launch_step_kernel(h, b, h->bg, 2))) return rc;
        if ((rc = timing_mark(eb, 1, h->bg))) return rc;
        h->bg_busy = true;
        ++h->bg_launches;
        if (odd) {
            NEO_HIP_CHECK(hipEventRecord(h->ev_sl[0], h->bg));  // due at the next even group's block
        } else {
            NEO_HIP_CHECK(hipEventRecord(h->ev_blk, s));  // the blocks before n: the next odd group's launch
            if (!primed && !NEO_NO_XWAIT) NEO_HIP_CHECK(hipStreamWaitEvent(s, h->ev_sl[0], 0));
        }
    }
    upols_t::ev_group* ev = nullptr;  // the step's (block's) launch alone
    if ((rc = timing_begin(h, 2, &ev)) || (rc = timing_mark(ev, 0, s))) return rc;
    if ((rc = launch_step_kernel(h, a, s, G > 1 ? 1 : 0))) return rc;
    h->fdl_zero = false;
    if ((rc = timing_mark(ev, 1, s))) return rc;
    h->wpos = h->wpos + 1 >= h->ring ? 0 : h->wpos + 1;
    h->lv_n = n + 1;
    return NEO_HIP_OK;
}

size_t off_hf_bytes(const upols_t* h) { return size_t(h->C) * size_t(spec_cs(h->off_nseg, h->B)) * sizeof(cf); }

int launch_off_mac(upols_t* h, int wp, hipStream_t s)
{
    if (!h->fv_tw)
        if (int rc = shared_far_tw(&h->fv_tw)) return rc;
    if (h->off_dirty) {
        const unsigned grid = unsigned(h->C) * unsigned(h->off_nseg) * unsigned(h->B / 16);
        hipLaunchKernelGGL(k_lvf_filter, dim3(grid), dim3(256), 0, s, h->H, h->off_hf, h->fv_tw, h->B, h->P,
                           h->off_nseg, h->cstride, h->pstride, 0, spec_cs(h->off_nseg, h->B));
        NEO_HIP_LAUNCH_CHECK();
        h->off_dirty = false;
    }
    off_args a{h->fdl, h->off_hf, h->fv_tw, h->off_y, h->cstride, h->pstride, spec_cs(h->off_nseg, h->B), h->ring, h->B,
               h->off_nseg, h->wpos};
    const unsigned grid = unsigned(h->C) * unsigned(h->B / 16);
    if (wp == 2) hipLaunchKernelGGL(k_off_mac<2>, dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_off_mac<1>, dim3(grid), dim3(256), 0, s, a);
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

int lvl_setup_prime(upols_t* h)
{
    if (!h->ahead || h->grouped || h->lv_n >= 0) return NEO_HIP_OK;
    if (int rc = lvl_buffers(h)) return rc;
    if (int rc = lvl_prime(h, h->stream)) return rc;
    h->lv_n = 0;
    h->pace_prev = false;
    h->pace_seq = 0;
    return NEO_HIP_OK;
}

// ---------------------------------------------------------------------------------------
// Latency mode (neo_hip_upols_set_persistent): ONE persistent kernel per handle runs every step
// of a latency-bound shape (few channels, no far level, one launch per step otherwise: C3). The
// host writes step n's record (its blocks' device addresses) to the mapped mailbox and spins on
// mb->done; no launch, no stream wait. Workgroups by role, fixed for the launch:
//   block    one per channel: waits for the slices of step n - 2 (agent acquire, issued before
//            the record arrives), polls the record, runs block_role, publishes (system-scope
//            release: the output and the FDL row), and the last of them signals the host
//   slices   per Toeplitz level: part j = n mod T (j < T - 1) of the NEXT window in T - 1 parts
//            (step groups' schedule: a window's slabs are complete two steps before its first
//            block, so a block never waits for the slices of the step before), after block
//            n - 1 published (agent acquire), then publish (agent release) and sl_done = n
// Every wait has a deadline (mb->err, then every workgroup leaves); the block workgroups leave
// after ps_idle_ms without a record, and the host relaunches at the next block.
// persist_ctl (upols_handle.hpp): the mailbox, flags, step times and limits; n0 = the launch's
// first step (the levels primed at step 0)
struct persist_args : persist_ctl {
    slice_args base;                // handle constants (H, FDL, ring, strides, prev, twiddles, a0)
    cf* slab[kLvToep];
    int T[kLvToep], LT[kLvToep], A[kLvToep], Bd[kLvToep], JH[kLvToep], UPW[kLvToep], U[kLvToep];  // LT = log2 T
    int wg0[kLvToep + 1];           // slice workgroups of level l: [wg0[l], wg0[l + 1])
    int nlev, nblk;
    int far, fU, fK, ffpl;          // far level (persist_far): on, units, window group, phase-1 f rows per lane
    int wgf0, wgf1;                 // its workgroups: slice workgroups [wgf0, wgf1) (after the Toeplitz levels')
    cf* ff;                         // far field [2][C][kFarT][B]
};

__device__ __forceinline__ int ps_ring_row(const persist_args& pa, int64_t n)
{
    const int64_t r = (int64_t(pa.w0) + (n - pa.n0)) % pa.base.ring;
    return int(r < 0 ? r + pa.base.ring : r);
}

template<int B, bool OLA>
__device__ __forceinline__ void persist_block(const persist_args& pa, int c, char* smem)
{
    __shared__ uint64_t io[2];
    __shared__ int go;
    const int nsl = pa.wgf1;  // the Toeplitz levels' slice workgroups and the far level's
    unsigned long long t_seen = 0;  // thread 0: when the record of the step was read (stored with its done time)
    int w = pa.w0;                  // ring row of step n
    for (int64_t n = pa.n0;; ++n, w = w + 1 == pa.base.ring ? 0 : w + 1) {
        // the step's arguments but its blocks, while thread 0 waits (T are powers of two)
        slice_args a = pa.base;
        a.w = w;
        a.nsl = pa.nlev;
        a.ff = nullptr;
        if (pa.far) {  // this block's far-field row (window n / kFarT, complete two steps before)
            a.ff = pa.ff + ((n / kFarT) & 1) * a.C * ff_cs(a.B) + (n % kFarT) * a.B;
            a.fcs = ff_cs(a.B);
        }
#pragma unroll
        for (int l = 0; l < kLvToep; ++l) {  // static indices: the slice_args stay in registers
            if (l < pa.nlev) {
                const int T = pa.T[l];
                a.sl[l] = pa.slab[l] + ((n >> pa.LT[l]) & 1) * a.C * slab_cs(T, a.B) + (n & (T - 1)) * a.B;
                a.scs[l] = slab_cs(T, a.B);
            }
        }
        if (threadIdx.x == 0) {
            // the window's slabs: every slice workgroup past step n - 2
            bool ok = ps_wait(pa, [&] {
                for (int s = 0; s < nsl; ++s)
                    if (ps_ld(pa.flags + kPsFlagSlices + s) < n - 2) return false;
                return true;
            });
            // a window of some level starts (every level's T is a multiple of the first's): its slab
            // rows were written by other workgroups since this CU last read that buffer
            if (ok && (n == pa.n0 || (n & (pa.T[0] - 1)) == 0)) ps_acquire();
            ok = ps_record(pa, n, c == 0, pa.nblk > 1, ok, io, t_seen);
            go = ok;
        }
        __syncthreads();
        if (!go) break;
        a.in = reinterpret_cast<const float*>(io[0]);
        a.out = reinterpret_cast<float*>(io[1]);
#ifdef NEO_PS_PROBE
        a.tl = pa.tl + 2 * kPsRing + 8 * (n % kPsRing);  // probe records [kPsRing][8] after the step times
        NEO_PS_MARK(a, 0);
#endif
        block_role<B, OLA, true>(a, c, smem);  // the output block write-through (system scope)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            // 1. the output: its write-through stores are complete, so the host may read it now
            int64_t* arr = pa.flags + kPsFlagArrive + n % kPsArr;
            if (__hip_atomic_fetch_add(arr, int64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pa.nblk - 1) {
                ps_st(arr, 0);  // free for step n + kPsArr (no channel gets there before blk_done moves on)
                const unsigned long long t_done = wall_clock64();
                __hip_atomic_store(&pa.mb->done, n + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                pa.tl[2 * (n % kPsRing) + 1] = t_done;  // plain: written back by the release below
            }
            if (c == 0) pa.tl[2 * (n % kPsRing)] = t_seen;  // workgroup 0 read the record
            // 2. the FDL row for the slice workgroups (off the host's path): agent release, blk_done
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            int64_t* arf = pa.flags + kPsFlagArriveFdl + n % kPsArr;
            if (__hip_atomic_fetch_add(arf, int64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pa.nblk - 1) {
                ps_st(arf, 0);
                ps_st(pa.flags + 0, n);
            }
        }
    }
    if (threadIdx.x == 0 && c == 0) __hip_atomic_store(&pa.mb->alive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void persist_slices(const persist_args& pa, int s, char* smem)
{
    __shared__ int go;
    int l = 0;
    while (l + 1 < pa.nlev && s >= pa.wg0[l + 1]) ++l;
    const int i = s - pa.wg0[l], T = pa.T[l], U = pa.U[l], UPW = pa.UPW[l];
    for (int64_t n = pa.n0 - 1;; ++n) {
        if (threadIdx.x == 0) {
            // FDL rows up to block n - 1 (the relaunch's first round redoes step n0 - 1: rows of
            // earlier launches, ordered by the kernel boundary)
            bool ok = n < pa.n0 || ps_wait(pa, [&] { return ps_ld(pa.flags + 0) >= n - 1; });
            if (ok && n >= pa.n0) ps_acquire();
            go = ok;
        }
        __syncthreads();
        if (!go) break;
        const int64_t cur = n / T;
        const int j = int(n % T);
        if (n >= 0 && j < T - 1) {
            const int u0 = int(int64_t(j) * U / (T - 1)), u1 = int(int64_t(j + 1) * U / (T - 1));
            const int nwg = (u1 - u0 + UPW - 1) / UPW;
            if (i < nwg) {
                slice_args a = pa.base;
                a.nblk = 0;
                a.ntp = l + 1;
                toep_arg ta{};
                ta.slab = pa.slab[l] + ((cur + 1) & 1) * int64_t(a.C) * slab_cs(T, a.B);
                ta.cs = slab_cs(T, a.B);
                ta.T = T;
                ta.a = pa.A[l];
                ta.b = pa.Bd[l];
                int tw = int((int64_t(ps_ring_row(pa, n)) + (cur + 1) * T - n) % a.ring);
                ta.tw = tw < 0 ? tw + a.ring : tw;
                ta.u0 = u0;
                ta.u1 = u1;
                ta.nwg = nwg;
                ta.jh = pa.JH[l];
#pragma unroll
                for (int L = 0; L < kLvToep; ++L) {  // static indices
                    if (L < l) a.tp[L].nwg = 0;
                    if (L == l) a.tp[L] = ta;
                }
                int bid = i;
                if (!toep_level<0>(a, bid, smem) && !toep_level<1>(a, bid, smem) && !toep_level<2>(a, bid, smem))
                    (void)toep_level<3>(a, bid, smem);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ps_st(pa.flags + kPsFlagSlices + s, n);
        }
    }
}

// far workgroup i of the far level (slice workgroup s): per step n, after block n - 1 published its
// FDL row AND every far workgroup finished step n - 1 (phase 2 of slice q - 1 reads the partial sums
// phase 1 wrote at step n - 1), the far work of step n (persist_far_args); then publish, sl_done = n
__device__ __forceinline__ void persist_far(const persist_args& pa, int s, int i, char* smem)
{
    __shared__ int go;
    for (int64_t n = pa.n0 - 1;; ++n) {
        if (threadIdx.x == 0) {
            // the relaunch's first round redoes step n0 - 1 (its inputs are an earlier launch's)
            bool ok = n < pa.n0 || ps_wait(pa, [&] {
                if (ps_ld(pa.flags + 0) < n - 1) return false;
                for (int f = pa.wgf0; f < pa.wgf1; ++f)
                    if (ps_ld(pa.flags + kPsFlagSlices + f) < n - 1) return false;
                return true;
            });
            if (ok && n >= pa.n0) ps_acquire();
            go = ok;
        }
        __syncthreads();
        if (!go) break;
        if (n >= 0) {
            slice_args a = pa.base;
            a.nblk = 0;
            a.ntp = 0;
            persist_far_args(a, n, ps_ring_row(pa, n), pa.fU, pa.fK, pa.ffpl, pa.ff);
            int bid = i;
            if (bid < a.f3nwg) {
                far2c_role<2>(a, bid, smem);
            } else if ((bid -= a.f3nwg) < a.f1nwg) {
                if (a.f1fpl == 4) far1_role<4, 2>(a, bid);
                else if (a.f1fpl == 2) far1_role<2, 2>(a, bid);
                else far1_role<1, 2>(a, bid);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ps_st(pa.flags + kPsFlagSlices + s, n);
        }
    }
}

template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_lvl_persist(persist_args pa)
{
    __shared__ __attribute__((aligned(16))) char smem[kSliceLds];
    const int s = int(blockIdx.x) - pa.nblk;
    if (s < 0) persist_block<B, OLA>(pa, int(blockIdx.x), smem);
    else if (s < pa.wgf0) persist_slices(pa, s, smem);
    else persist_far(pa, s, s - pa.wgf0, smem);
}

const char* persist_ineligible(const upols_t* h)
{
    if (h->v2) return "upola_convolver_v2 takes sub-block input";
    if (h->C > 16) return "more than 16 channels (the latency mode is for latency-bound shapes)";
    if (!h->ahead)  // the plain step's workgroups, all resident (one per CU at B = 4096)
        return h->C * h->S > 256 ? "the plain step's channels x splits above 256 workgroups" : nullptr;
    if (h->lv.n && h->lv.T[h->lv.n - 1] == kBigT) return "the 128-block Toeplitz form of the far band (far_level 0)";
    if (h->lv.nseg && h->far_raw) return "the recomputed far level (far_level 2)";
    if (h->lv.nseg && far_group(h) > 2) return "a far window group above 2 (neo_hip_upols_opts.far_group)";
    if (h->B > 512) return "blocks above 512 samples with the streaming levels";
    return nullptr;
}

// the slice workgroups of level l: the most any part of its T - 1 needs
static int persist_level_wgs(const upols_t* h, int l, int& U, int& UPW, int& JH)
{
    const int T = h->lv.T[l];
    toep_geom(h, T, JH, UPW);
    U = int(toep_units(h, T));
    int most = 0;
    for (int j = 0; j + 1 < T; ++j) {
        const int u0 = int(int64_t(j) * U / (T - 1)), u1 = int(int64_t(j + 1) * U / (T - 1));
        most = std::max(most, (u1 - u0 + UPW - 1) / UPW);
    }
    return most;
}

// the levels' part of the latency mode's arguments (window 0 of every level primed first when
// the schedule restarts)
static int persist_levels(upols_t* h, persist_args& pa, int64_t ld_in, int64_t ld_out)
{
    if (int rc = lvl_buffers(h)) return rc;
    if (h->lv_n == 0 && h->fdl_zero) {  // primed by a setup call (lvl_setup_prime), nothing stepped since
        h->ps_valid = true;
    } else if (!h->ps_valid || h->lv_n < 0) {  // window 0 of every level, from this block on
        if (int rc = lvl_join(h, h->ps_stream)) return rc;
        h->lv_n = -1;
        if (int rc = lvl_prime(h, h->ps_stream)) return rc;
        h->lv_n = 0;
        h->ps_valid = true;
    }
    pa.base = base_args(h);
    pa.base.prev = h->prev;
    pa.base.twg = h->tw;
    pa.base.a0 = h->lv.a0;
    pa.base.ld_in = ld_in;
    pa.base.ld_out = ld_out;
    pa.nlev = h->lv.n;
    pa.nblk = h->C;
    pa.wg0[0] = 0;
    for (int l = 0; l < h->lv.n; ++l) {
        pa.slab[l] = h->lv_slab[l];
        pa.T[l] = h->lv.T[l];
        pa.LT[l] = __builtin_ctz(unsigned(h->lv.T[l]));
        pa.A[l] = h->lv.a[l];
        pa.Bd[l] = h->lv.b[l];
        pa.wg0[l + 1] = pa.wg0[l] + persist_level_wgs(h, l, pa.U[l], pa.UPW[l], pa.JH[l]);
    }
    pa.wgf0 = pa.wgf1 = pa.wg0[h->lv.n];
    if (h->lv.nseg) {  // the far level: as many workgroups as its busiest step needs (any window, any slice)
        pa.far = 1;
        pa.fU = int(far_units(h));
        pa.fK = far_group(h);
        pa.ffpl = far1_fpl(h);
        pa.ff = h->fv_ff;
        int most = 1;
        for (int64_t W = 1; W <= 2 * pa.fK + 1; ++W)
            for (int q = 0; q < kFarT; ++q) {
                slice_args t = pa.base;
                persist_far_args(t, (W - 1) * kFarT + q, 0, pa.fU, pa.fK, pa.ffpl, pa.ff);
                most = std::max(most, t.f1nwg + t.f3nwg);
            }
        pa.wgf1 = pa.wgf0 + most;
    }
    return NEO_HIP_OK;
}

bool persist_room(upols_t* h, const void* f, int grid)
{
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (!resident_admit(h->device, grid, per_cu * cus * 3 / 4)) return false;
    h->ps_wgs = grid;
    return true;
}

static int persist_launch(upols_t* h, int64_t ld_in, int64_t ld_out)
{
    if (!h->ps_stream) {
        // the most urgent priority: such a stream gets a hardware queue of its own. At the default
        // priority it shares one of the process's GPU_MAX_HW_QUEUES (4) with other streams, whose
        // work then queues behind the resident kernel until it leaves (idle limit): measured on
        // MI355X, the third new torch stream waited 1.4 s behind a 1.5 s idle limit
        // (tools/dbg_hwq.py; none waited with this priority)
        int lo = 0, hi = 0;
        NEO_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        NEO_HIP_CHECK(hipStreamCreateWithPriority(&h->ps_stream, hipStreamNonBlocking, hi));
        if (int rc = halloc(reinterpret_cast<void**>(&h->ps_mb), reinterpret_cast<void**>(&h->ps_mb_dev), sizeof(persist_mb)))
            return rc;
        std::memset(h->ps_mb, 0, sizeof(persist_mb));
        if (int rc = dalloc(&h->ps_tl, 10 * kPsRing * sizeof(unsigned long long))) return rc;
        NEO_HIP_CHECK(hipMemsetAsync(h->ps_tl, 0, 10 * kPsRing * sizeof(unsigned long long), h->ps_stream));
    }
    persist_args pa{};
    if (h->ahead) {
        if (int rc = persist_levels(h, pa, ld_in, ld_out)) return rc;
    } else if (!h->ps_valid || h->lv_n < 0) {  // the plain step continues from the FDL ring: nothing to prime
        h->lv_n = 0;
        h->ps_valid = true;
    }
    const int nsl = h->ahead ? pa.wgf1 : 0;
    if (h->ps_nslices < nsl || !h->ps_flags) {
        dfree(h->ps_flags);
        h->ps_flags = nullptr;
        if (int rc = dalloc(&h->ps_flags, size_t(kPsFlagSlices + nsl) * sizeof(int64_t))) return rc;
        h->ps_nslices = nsl;
    }
    pa.n0 = h->lv_n;
    pa.w0 = h->wpos;
    pa.mb = h->ps_mb_dev;
    pa.flags = h->ps_flags;
    pa.tl = h->ps_tl;
    pa.idle_ticks = (long long)(h->ps_idle_ms * 1e5);  // wall_clock64: 100 MHz
    // 2 s past the idle limit: a wait that long is a fault, not a schedule (the slice and later
    // block workgroups wait for the host's next record too, up to the idle limit)
    pa.dead_ticks = pa.idle_ticks + 200000000LL;
    std::vector<int64_t> init(size_t(kPsFlagSlices + nsl), 0);  // quit, arrivals, records: 0
    init[0] = pa.n0 - 1;                                          // blk_done
    init[kPsFlagGo] = pa.n0 - 1;
    for (int k = 0; k < nsl; ++k) init[size_t(kPsFlagSlices + k)] = pa.n0 - 2;  // sl_done
    NEO_HIP_CHECK(hipMemcpyAsync(h->ps_flags, init.data(), init.size() * sizeof(int64_t), hipMemcpyHostToDevice,
                                 h->ps_stream));
    NEO_HIP_CHECK(hipStreamSynchronize(h->ps_stream));  // the prime and the flags before the first record
    // no record of an earlier launch may match a step of this one: a restarted schedule (n0 = 0
    // after a reset, filter change or mode toggle) reuses the lap tags of the run before, so every
    // slot is cleared to tag 0, which no step carries (ps_tag is 1..15). The kernel is not running
    // and the host writes step n0's record only after this.
    for (auto& r : h->ps_mb->rec) {
        __atomic_store_n(&r.in, uint64_t(0), __ATOMIC_RELAXED);
        __atomic_store_n(&r.out, uint64_t(0), __ATOMIC_RELAXED);
    }
    h->ps_mb->stop = 0;
    h->ps_mb->err = 0;
    h->ps_mb->done = pa.n0;
    h->ps_mb->alive = 1;
    const unsigned grid = unsigned(h->C + nsl);
    bool launched = false;
    if (!h->ahead) {
        if (int rc = plain_persist_launch(h, pa, ld_in, ld_out, &launched)) return rc;
    } else if (h->ola) {
        NEO_UPOLS_DISPATCH(h->B, if constexpr (BB <= 512) {
            if ((launched = persist_room(h, reinterpret_cast<const void*>(&k_lvl_persist<BB, true>), int(grid))))
                hipLaunchKernelGGL((k_lvl_persist<BB, true>), dim3(grid), dim3(256), 0, h->ps_stream, pa);
        })
    } else {
        NEO_UPOLS_DISPATCH(h->B, if constexpr (BB <= 512) {
            if ((launched = persist_room(h, reinterpret_cast<const void*>(&k_lvl_persist<BB, false>), int(grid))))
                hipLaunchKernelGGL((k_lvl_persist<BB, false>), dim3(grid), dim3(256), 0, h->ps_stream, pa);
        })
    }
    if (!launched) {  // no room for every workgroup at once: the caller runs normal steps (persist_process)
        h->ps_mb->alive = 0;
        return NEO_HIP_OK;
    }
    if (hipGetLastError() != hipSuccess) {
        resident_release(h->device, h->ps_wgs);
        h->ps_wgs = 0;
        return fail(NEO_HIP_ERUNTIME, "persistent kernel launch failed");
    }
    h->ps_running = true;
    h->ps_ld_in = ld_in;
    h->ps_ld_out = ld_out;
    h->ps_n0 = pa.n0;
    ++h->ps_launches;
    return NEO_HIP_OK;
}

// a step that was handed to the kernel may not have completed: the FDL ring and the level slabs
// no longer follow the schedule, so the next call re-primes from its own block (persist_stop's
// semantics) instead of continuing with a missing row
static void persist_invalidate(upols_t* h)
{
    h->ps_valid = false;
    h->lv_n = -1;
}

// the running kernel (if any) leaves; ps_valid stays: a relaunch continues the schedule (unless
// the kernel failed)
static int persist_join(upols_t* h)
{
    if (!h->ps_running) return NEO_HIP_OK;
    __atomic_store_n(&h->ps_mb->stop, 1, __ATOMIC_SEQ_CST);
    const hipError_t e = hipStreamSynchronize(h->ps_stream);
    h->ps_running = false;
    resident_release(h->device, h->ps_wgs);
    h->ps_wgs = 0;
    if (e != hipSuccess) {
        persist_invalidate(h);
        return fail(NEO_HIP_ERUNTIME, "persistent kernel: %s", hipGetErrorString(e));
    }
    if (__atomic_load_n(&h->ps_mb->err, __ATOMIC_SEQ_CST)) {
        persist_invalidate(h);
        return fail(NEO_HIP_ERUNTIME, "persistent kernel: a wait passed its deadline");
    }
    if (__atomic_load_n(&h->ps_mb->done, __ATOMIC_SEQ_CST) < h->lv_n) {
        persist_invalidate(h);  // left (stop, idle limit) with records not yet stepped
        return fail(NEO_HIP_ERUNTIME, "persistent kernel left before step %lld", (long long)h->lv_n - 1);
    }
    return NEO_HIP_OK;
}

int persist_stop(upols_t* h)
{
    const int rc = persist_join(h);
    if (h->ps_valid) {
        h->ps_valid = false;
        h->lv_n = -1;  // the normal schedule re-primes the levels
    }
    return rc;
}

int persist_process(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int64_t nblocks)
{
    if (const char* why = persist_ineligible(h)) return fail(NEO_HIP_EINVAL, "latency mode: %s", why);
    if (h->ps_running && (h->lv_n < 0 || !h->ps_valid))
        if (int rc = persist_join(h)) return rc;  // the schedule restarts: relaunch after the prime
    if (h->C > 1 && (ld_in != h->ps_ld_in || ld_out != h->ps_ld_out) && h->ps_running)
        if (int rc = persist_join(h)) return rc;  // another channel stride: relaunch with it
    if (h->ps_running && !__atomic_load_n(&h->ps_mb->alive, __ATOMIC_ACQUIRE))
        if (int rc = persist_join(h)) return rc;  // left after its idle limit (or failed)
    if (!h->ps_running) {
        if (int rc = persist_launch(h, ld_in, ld_out)) return rc;
        if (!h->ps_running) {
            // no room on the device for the persistent grid (other persistent kernels of this
            // process hold it): this call's blocks run as normal steps, complete on return; the
            // schedules differ, so the levels re-prime (and again when a later call relaunches)
            ++h->ps_fallbacks;
            if (int rc = persist_stop(h)) return rc;
            for (int64_t k = 0; k < nblocks; ++k)
                if (int rc = launch_step_normal(h, in + k * h->B, ld_in, out + k * h->B, ld_out, h->stream)) return rc;
            return spin_sync(h->stream);
        }
    }
    persist_mb* mb = h->ps_mb;  // allocated by the first launch
    const int B = h->B;
    for (int64_t k = 0; k < nblocks; ++k) {
        const int64_t n = h->lv_n;
        while (__atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) < n - (kPsRing - 2)) {  // a free slot
            if (!__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE)) {
                const int rc = persist_join(h);
                return rc ? rc : fail(NEO_HIP_ERUNTIME, "persistent kernel left");
            }
        }
        const uint64_t tag = ps_tag(n);
        persist_rec& r = mb->rec[n % kPsRing];
        __atomic_store_n(&r.in, reinterpret_cast<uint64_t>(in + k * B) | tag, __ATOMIC_RELEASE);
        __atomic_store_n(&r.out, reinterpret_cast<uint64_t>(out + k * B) | tag, __ATOMIC_RELEASE);
        h->fdl_zero = false;
        h->lv_n = n + 1;
        h->wpos = h->wpos + 1 >= h->ring ? 0 : h->wpos + 1;
    }
    // complete on return (the block's deadline: spin, do not yield); the kernel's own waits give
    // up 2 s past its idle limit (dead_ticks), so a host wait 3 s past it means the kernel is not
    // running at all
    const auto t0 = std::chrono::steady_clock::now();
    const auto limit = std::chrono::duration<double, std::milli>(h->ps_idle_ms + 3000.0);
    for (unsigned it = 0; __atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) < h->lv_n; ++it) {
        if (!__atomic_load_n(&mb->alive, __ATOMIC_ACQUIRE) && __atomic_load_n(&mb->done, __ATOMIC_ACQUIRE) < h->lv_n) {
            const int rc = persist_join(h);
            return rc ? rc : fail(NEO_HIP_ERUNTIME, "persistent kernel left before step %lld", (long long)h->lv_n);
        }
        if ((it & 4095) == 0 && std::chrono::steady_clock::now() - t0 > limit) {
            __atomic_store_n(&mb->stop, 1, __ATOMIC_SEQ_CST);
            persist_invalidate(h);  // the next call joins the kernel and re-primes
            return fail(NEO_HIP_ERUNTIME, "persistent kernel: no progress for %.0f ms", limit.count());
        }
    }
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

// The step groups' background plan of a (channels, block, partitions) convolver with default
// options and step group G (0: the automatic one), for tests (no device needed): phi[l] per
// Toeplitz level; the cycle (groups); the cuts of every background level in level order, each
// cycle / (T / G) windows of T / G cuts, into cuts[cuts_cap] (*ncuts written); the predicted
// background bytes per group of the cycle into loads[loads_cap]; uniform != 0: equal parts and
// no offsets (the plan step groups had before the balancing, for comparison).
extern "C" NEO_HIP_API int neo_hip_upols_part_plan(int channels, int block, int partitions, int step_group, int uniform,
                                                   int* phi, int* cycle, int* cuts, int cuts_cap, int* ncuts,
                                                   double* loads, int loads_cap)
{
    if (channels < 1 || block < 16 || partitions < 1 || step_group < 0)
        return neo_hip::fail(NEO_HIP_EINVAL, "part plan: bad shape");
    neo_hip_upols h{};
    h.C = channels;
    h.B = block;
    h.P = partitions;
    neo_hip::plan_levels(partitions, h.lv);
    h.sg = step_group ? step_group : neo_hip::step_group_for(channels, block, partitions);
    std::vector<double> ld;
    neo_hip::plan_handle_parts(&h, &ld, !uniform);
    if (phi)
        for (int l = 0; l < h.lv.n; ++l) phi[l] = h.lv_phi[l];
    if (cycle) *cycle = h.lv_cyc;
    int n = 0;
    for (int l = 0; l < h.lv.n; ++l)
        for (int v : h.lv_cut[l]) {
            if (cuts && n < cuts_cap) cuts[n] = v;
            ++n;
        }
    if (ncuts) *ncuts = n;
    if (loads)
        for (int g = 0; g < std::min(loads_cap, int(ld.size())); ++g) loads[g] = ld[size_t(g)];
    return NEO_HIP_OK;
}

// The far level's phase-1 window group of a handle (far_group: auto or forced by
// neo_hip_upols_opts.far_group); 0 without a far transform level.
extern "C" NEO_HIP_API int neo_hip_upols_get_far_group(neo_hip_upols* h, int* windows)
{
    if (!h || !windows) return neo_hip::fail(NEO_HIP_EINVAL, "null handle or output");
    *windows = h->lv.nseg ? neo_hip::far_group(h) : 0;
    return NEO_HIP_OK;
}

extern "C" NEO_HIP_API int neo_hip_upols_get_far_form(neo_hip_upols* h, int* form)
{
    if (!h || !form) return neo_hip::fail(NEO_HIP_EINVAL, "null handle or output");
    *form = h->lv.nseg ? (h->far_raw ? 2 : 1) : (h->lv.n && h->lv.T[h->lv.n - 1] == neo_hip::kBigT ? 3 : 0);
    return NEO_HIP_OK;
}

extern "C" NEO_HIP_API int neo_hip_upols_get_step_group(neo_hip_upols* h, int* steps)
{
    if (!h || !steps) return neo_hip::fail(NEO_HIP_EINVAL, "null handle or output");
    *steps = h->sg;
    return NEO_HIP_OK;
}

extern "C" NEO_HIP_API int neo_hip_upols_join_background(neo_hip_upols* h, void* stream)
{
    if (!h) return neo_hip::fail(NEO_HIP_EINVAL, "null handle");
    neo_hip::device_guard g(h->device);
    if (g.rc) return g.rc;
    return neo_hip::lvl_join(h, static_cast<hipStream_t>(stream));
}

#ifdef NEO_PS_PROBE
// diagnostic builds only (not in include/neo_hip.h): the latency mode's per-step probe records,
// [kPsRing][2] {seen, done} then [kPsRing][8] block-role points (wall clock, 100 MHz)
extern "C" NEO_HIP_API int neo_hip_diag_persist_probe(neo_hip_upols* h, unsigned long long* out)
{
    if (!h || !h->ps_tl) return neo_hip::fail(NEO_HIP_EINVAL, "no latency-mode records");
    NEO_HIP_CHECK(hipMemcpy(out, h->ps_tl, 10 * neo_hip::kPsRing * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return NEO_HIP_OK;
}
#endif

#ifdef NEO_TIMELINE
// diagnostic builds only (not in include/neo_hip.h): copy the last step launch's per-workgroup
// records {start, end, role | cu << 32 | xcc << 56, mid} (wall_clock64 ticks; mid 0 where the
// role stamps none) into out, up to cap workgroups
extern "C" NEO_HIP_API int neo_hip_diag_timeline(unsigned long long* out, int64_t cap, int64_t* count)
{
    NEO_HIP_CHECK(hipDeviceSynchronize());
    const int64_t n = std::min(cap, neo_hip::g_tl_nn[0]);
    if (n > 0) NEO_HIP_CHECK(hipMemcpy(out, neo_hip::g_tl_buf[0], size_t(n) * 32, hipMemcpyDeviceToHost));
    if (count) *count = neo_hip::g_tl_nn[0];
    return NEO_HIP_OK;
}

// the same for the last launch of part 1 (step groups' block launch) or 2 (their slices launch)
extern "C" NEO_HIP_API int neo_hip_diag_timeline_part(int part, unsigned long long* out, int64_t cap, int64_t* count)
{
    if (part < 0 || part > 2) return neo_hip::fail(NEO_HIP_EINVAL, "part");
    NEO_HIP_CHECK(hipDeviceSynchronize());
    const int64_t n = std::min(cap, neo_hip::g_tl_nn[part]);
    if (n > 0) NEO_HIP_CHECK(hipMemcpy(out, neo_hip::g_tl_buf[part], size_t(n) * 32, hipMemcpyDeviceToHost));
    if (count) *count = neo_hip::g_tl_nn[part];
    return NEO_HIP_OK;
}
#endif
