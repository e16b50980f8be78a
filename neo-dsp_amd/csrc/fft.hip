// fft.hip — batched c2c / r2c / c2r FFT plans for MI355X (gfx950), C-ABI part.
//
// Replaces neo's fft_plan (c2c_dit2_plan, src/neo/fft/reference/c2c_dit2_plan.hpp:21-104)
// and rfft_plan (fallback_rfft_plan, src/neo/fft/fallback/fallback_rfft_plan.hpp:14-61).
//
// Sizes N <= 4096 (c2c) / N <= 8192 (real): one kernel, one pass over HBM — each
// workgroup loads whole transforms into registers (lane t owns t + m*T, coalesced),
// runs the Stockham passes through LDS and stores the natural-order result.
// Larger sizes: ceil(log2 N / 10) global Stockham passes of radix 64..1024 whose DFTs
// run in LDS over groups of adjacent columns (ping-pong scratch); 2-2.4x faster than
// the radix-16 register passes of the first version.
#include "common.hpp"
#include "fft_device_real.hpp"

#include <algorithm>
#include <cstring>
#include <memory>

namespace neo_hip {

constexpr int kMaxOrder = 27;   // c2c_dit2_plan.hpp:58-61
constexpr int kLdsMaxOrder = 12;  // N <= 4096 complex points per LDS transform
#ifndef NEO_FFT_PASS_BITS
#define NEO_FFT_PASS_BITS 10
#endif
constexpr int kPassBits = NEO_FFT_PASS_BITS;  // large transforms: passes of at most 2^kPassBits points

__host__ __device__ constexpr int pick_e(int n) { return n >= 16 ? 16 : (n < 1 ? 1 : n); }

// ---------------------------------------------------------------------------
// c2c, whole transforms in LDS. FPB transforms per 256-lane block for small N.
// ---------------------------------------------------------------------------
template<int N, int DIR, class C = cf>
__global__ __launch_bounds__(256) void k_c2c_lds(const C* __restrict__ in, C* __restrict__ out,
                                                 const C* __restrict__ twg, int64_t batch)
{
    constexpr int E = pick_e(N), T = N / E, FPB = T >= 256 ? 1 : 256 / T;
    constexpr int TWL = twiddle_len<N>(), LL = lds_len(N);
    __shared__ C smem[FPB * LL + TWL];
    C* tw = smem + FPB * LL;
    const int tid = threadIdx.x, f = tid / T, t = tid % T;
    for (int i = tid; i < TWL; i += FPB * T) tw[i] = twg[i];
    const int64_t g = int64_t(blockIdx.x) * FPB + f;
    const bool active = g < batch;
    C v[E];
    if (active) {
        const C* src = in + g * N;
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = ld_nt(src + t + m * T);
    }
    __syncthreads();
    stockham<N, E, DIR>(v, smem + f * LL, tw, t, active);
    if (active) {
        C* dst = out + g * N;
#pragma unroll
        for (int m = 0; m < E; ++m) st_nt(dst + t + m * T, v[m]);
    }
}

// ---------------------------------------------------------------------------
// r2c / c2r of N = 2M reals, whole transforms in LDS (unpacked N/2+1 bins).
// ---------------------------------------------------------------------------
template<int M, class C = cf>
__global__ __launch_bounds__(256) void k_r2c_lds(const real_of<C>* __restrict__ in, C* __restrict__ out,
                                                 const C* __restrict__ twg, int64_t batch)
{
    using R = real_of<C>;
    constexpr int E = pick_e(M), T = M / E, FPB = T >= 256 ? 1 : 256 / T;
    constexpr int TW1 = twiddle_len<M>(), TW2 = twiddle_len<2 * M>(), LL = lds_len(M);
    __shared__ C smem[FPB * LL + TW1 + TW2];
    C* tw1 = smem + FPB * LL;
    C* tw2 = tw1 + TW1;
    const int tid = threadIdx.x, f = tid / T, t = tid % T;
    for (int i = tid; i < TW1 + TW2; i += FPB * T) tw1[i] = twg[i];
    const int64_t g = int64_t(blockIdx.x) * FPB + f;
    const bool active = g < batch;
    C* lds = smem + f * LL;
    C v[E];
    if (active) {
        const C* src = reinterpret_cast<const C*>(in + g * 2 * M);  // z[n] = x[2n] + i x[2n+1]
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = ld_nt(src + t + m * T);
    }
    __syncthreads();
    stockham<M, E, -1>(v, lds, tw1, t, active);
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) lds[lpad(t + m * T)] = v[m];
    }
    __syncthreads();
    if (active) {
        C* dst = out + g * (M + 1);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = t + m * T;
            const C x = r2c_split<M>(lds, tw2, k);
            if (k == 0) {
                dst[0] = {x.x, R(0)};
                dst[M] = {x.y, R(0)};
            } else {
                dst[k] = x;
            }
        }
    }
}

template<int M, class C = cf>
__global__ __launch_bounds__(256) void k_c2r_lds(const C* __restrict__ in, real_of<C>* __restrict__ out,
                                                 const C* __restrict__ twg, int64_t batch)
{
    constexpr int E = pick_e(M), T = M / E, FPB = T >= 256 ? 1 : 256 / T;
    constexpr int TW1 = twiddle_len<M>(), TW2 = twiddle_len<2 * M>(), LL = lds_len(M + 1);
    __shared__ C smem[FPB * LL + TW1 + TW2];
    C* tw1 = smem + FPB * LL;
    C* tw2 = tw1 + TW1;
    const int tid = threadIdx.x, f = tid / T, t = tid % T;
    for (int i = tid; i < TW1 + TW2; i += FPB * T) tw1[i] = twg[i];
    const int64_t g = int64_t(blockIdx.x) * FPB + f;
    const bool active = g < batch;
    C* lds = smem + f * LL;
    if (active) {
        const C* src = in + g * (M + 1);
        for (int k = t; k <= M; k += T) lds[lpad(k)] = src[k];
    }
    __syncthreads();
    C v[E];
    if (active) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int k = t + m * T;
            v[m] = c2r_join<M>(lds[lpad(k)], lds[lpad(k == 0 ? M : M - k)], tw2, k);
        }
    }
    __syncthreads();
    stockham<M, E, +1>(v, lds, tw1, t, active);
    if (active) {
        C* dst = reinterpret_cast<C*>(out + g * 2 * M);
#pragma unroll
        for (int m = 0; m < E; ++m) st_nt(dst + t + m * T, v[m]);
    }
}

// order-0 real transforms (N = 1): X[0] = x[0]; x[0] = Re X[0]
template<class C>
__global__ void k_r2c_order0(const real_of<C>* in, C* out, int64_t batch)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < batch) out[i] = {in[i], 0};
}
template<class C>
__global__ void k_c2r_order0(const C* in, real_of<C>* out, int64_t batch)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < batch) out[i] = in[i].x;
}

// ---------------------------------------------------------------------------
// Large transforms: two-level twiddle W_n^e from the split table (e = hi * 2^lo_bits + lo).
// ---------------------------------------------------------------------------
template<class C>
__device__ __forceinline__ C split_twiddle(const C* tw, int lo_bits, int64_t e)
{
    const int64_t mask = (int64_t(1) << lo_bits) - 1;
    return cmul(tw[(int64_t(1) << lo_bits) + (e >> lo_bits)], tw[e & mask]);
}

// One global Stockham pass of a large radix R (64..512) with the R-point DFTs done in LDS
// (the same stockham<> building block as the one-pass kernel): a workgroup takes G
// consecutive columns j, reads in[j + r*(n/R)] (G contiguous elements per r: coalesced),
// twiddles by W_n^(r * jm * n/(ns*R)), runs G R-point FFTs and writes
// out[(j/ns)*ns*R + jm + r*ns]. Large transforms take ceil(log2(n)/9) such passes
// instead of ceil(log2(n)/4) radix-16 ones.
template<int R>
__host__ __device__ constexpr int pass_cols() { return 8192 / R; }  // G: G*R = 8192 points per workgroup

template<int R, int DIR, class C>
__global__ __launch_bounds__(256, (sizeof(C) == 8 ? 2 : 1)) void k_pass_lds(const C* __restrict__ in, C* __restrict__ out,
                                                  const C* __restrict__ tw, int lo_bits, const C* __restrict__ twr,
                                                  int64_t n, int64_t ns, int64_t batch)
{
    constexpr int G = pass_cols<R>(), E = pick_e(R), TR = R / E, LL = lds_len(R), FPR = 256 / TR;
    constexpr int TWL = twiddle_len<R>();
    static_assert(G % FPR == 0, "whole rounds of transforms");
    __shared__ C data[G * LL];
    __shared__ C twl[TWL];
    const int tid = threadIdx.x;
    for (int i = tid; i < TWL; i += 256) twl[i] = twr[i];
    const int64_t nb = n / R, gpb = nb / G;
    const int64_t b = blockIdx.x / gpb, j0 = (blockIdx.x - b * gpb) * G;
    in += b * n;
    out += b * n;
    const int64_t step = n / (ns * R);
    constexpr int PER = G * R / 256, HALF = 16, NH = PER / HALF;  // elements per thread, batches of 16
    // all loads of a batch are issued before any is used (no per-element wait)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        C v[HALF];
#pragma unroll
        for (int k = 0; k < HALF; ++k) {
            const int idx = tid + (h * HALF + k) * 256, r = idx / G, jj = idx - r * G;
            v[k] = ld_nt(in + (j0 + jj) + r * nb);
        }
#pragma unroll
        for (int k = 0; k < HALF; ++k) {
            const int idx = tid + (h * HALF + k) * 256, r = idx / G, jj = idx - r * G;
            if (ns > 1 && r) {
                C w = split_twiddle(tw, lo_bits, int64_t(r) * ((j0 + jj) & (ns - 1)) * step);
                if (DIR > 0) w.y = -w.y;
                v[k] = cmul(v[k], w);
            }
            data[jj * LL + lpad(r)] = v[k];
        }
    }
    __syncthreads();
#pragma unroll 1
    for (int f0 = 0; f0 < G; f0 += FPR) {
        const int f = f0 + tid / TR, t = tid - (tid / TR) * TR;
        C v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = data[f * LL + lpad(t + m * TR)];
        __syncthreads();  // every lane of a transform has its inputs before the passes write
        stockham<R, E, DIR>(v, data + f * LL, twl, t, true);
#pragma unroll
        for (int m = 0; m < E; ++m) data[f * LL + lpad(t + m * TR)] = v[m];
        __syncthreads();
    }
    if (ns == 1) {  // out[j*R + r]: contiguous in r
        for (int idx = tid; idx < G * R; idx += 256) {
            const int jj = idx / R, r = idx - jj * R;
            st_nt(out + (j0 + jj) * R + r, data[jj * LL + lpad(r)]);
        }
    } else {  // contiguous in j within an ns-block
        for (int idx = tid; idx < G * R; idx += 256) {
            const int r = idx / G, jj = idx - r * G;
            const int64_t j = j0 + jj, jm = j & (ns - 1);
            st_nt(out + (j / ns) * ns * R + jm + r * ns, data[jj * LL + lpad(r)]);
        }
    }
}

// r2c split / c2r join for large sizes (global memory, one bin per lane).
template<class C>
__global__ void k_r2c_split_global(const C* __restrict__ z, C* __restrict__ out, const C* __restrict__ tw,
                                   int lo_bits, int64_t m, int64_t batch)
{
    using Rl = real_of<C>;
    const int64_t gid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (gid >= batch * m) return;
    const int64_t b = gid / m, k = gid - b * m;
    const C* zr = z + b * m;
    C* dst = out + b * (m + 1);
    const C zk = zr[k];
    if (k == 0) {
        dst[0] = {zk.x + zk.y, Rl(0)};
        dst[m] = {zk.x - zk.y, Rl(0)};
        return;
    }
    const C zc = cconj(zr[m - k]);
    const C fe = cscale(cadd(zk, zc), Rl(0.5));
    const C d = csub(zk, zc);
    const C fo = {Rl(0.5) * d.y, Rl(-0.5) * d.x};
    dst[k] = cadd(fe, cmul(split_twiddle(tw, lo_bits, k), fo));
}

template<class C>
__global__ void k_c2r_join_global(const C* __restrict__ x, C* __restrict__ z, const C* __restrict__ tw,
                                  int lo_bits, int64_t m, int64_t batch)
{
    const int64_t gid = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (gid >= batch * m) return;
    const int64_t b = gid / m, k = gid - b * m;
    const C* xr = x + b * (m + 1);
    C a, c;
    if (k == 0) {
        a = {xr[0].x, 0};
        c = {xr[m].x, 0};
    } else {
        a = xr[k];
        c = cconj(xr[m - k]);
    }
    C w = split_twiddle(tw, lo_bits, k);
    w.y = -w.y;
    const C fe = cadd(a, c);
    const C fo = cmul(csub(a, c), w);
    z[b * m + k] = {fe.x - fo.y, fe.y + fo.x};
}

}  // namespace neo_hip

using namespace neo_hip;

struct neo_hip_fft_plan {
    int order = 0, kind = 0, device = 0;
    bool f64 = false;        // complex<double> / double plans (NEO_HIP_F64)
    int64_t batch = 0, n = 0;
    hipStream_t stream = nullptr;
    void* d_tw = nullptr;    // LDS path: table(n) [c2c] or table(M) ++ table(2M) [real]
    void* d_split = nullptr; // large path: split table of the inner c2c size
    int lo_bits = 0;
    void* d_split2 = nullptr;  // large real path: split table of size 2M (join/split twiddles)
    int lo_bits2 = 0;
    void* d_scratch[3] = {nullptr, nullptr, nullptr};
    std::vector<int> radix;  // large path: pass radices (64..512 in LDS, or 2..16 in registers)
    void* d_ptw = nullptr;   // large path: R-point twiddle tables of the LDS passes, concatenated
    std::vector<size_t> ptw_off;
    void* d_in = nullptr;    // staging for neo_hip_fft_execute_host
    void* d_out = nullptr;
    size_t in_bytes = 0, out_bytes = 0;
    neo_hip::stream_set used;  // streams the plan's executes ran on (destroy joins them, not the device)
};

namespace {

using plan_t = neo_hip_fft_plan;

// inner complex FFT order of a plan (c2c: order, real: order-1)
int inner_order(const plan_t* p) { return p->kind == NEO_HIP_C2C ? p->order : p->order - 1; }

template<int DIR, class C>
int launch_c2c_lds(int order, const C* in, C* out, const C* tw, int64_t batch, hipStream_t s)
{
#define NEO_C2C_CASE(ORD)                                                                            \
    case ORD: {                                                                                      \
        constexpr int N = 1 << ORD, E = pick_e(N), T = N / E, FPB = T >= 256 ? 1 : 256 / T;          \
        const int64_t blocks = (batch + FPB - 1) / FPB;                                              \
        hipLaunchKernelGGL((k_c2c_lds<N, DIR, C>), dim3(unsigned(blocks)), dim3(FPB * T), 0, s, in, out, tw, \
                           batch);                                                                   \
        break;                                                                                       \
    }
    switch (order) {
        NEO_C2C_CASE(0) NEO_C2C_CASE(1) NEO_C2C_CASE(2) NEO_C2C_CASE(3) NEO_C2C_CASE(4) NEO_C2C_CASE(5)
        NEO_C2C_CASE(6) NEO_C2C_CASE(7) NEO_C2C_CASE(8) NEO_C2C_CASE(9) NEO_C2C_CASE(10) NEO_C2C_CASE(11)
        NEO_C2C_CASE(12)
        default: return fail(NEO_HIP_EINVAL, "c2c lds: bad order %d", order);
    }
#undef NEO_C2C_CASE
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

template<class C>
int launch_real_lds(int kind, int m_order, const void* in, void* out, const C* tw, int64_t batch, hipStream_t s)
{
    using R = real_of<C>;
#define NEO_REAL_CASE(ORD)                                                                            \
    case ORD: {                                                                                       \
        constexpr int M = 1 << ORD, E = pick_e(M), T = M / E, FPB = T >= 256 ? 1 : 256 / T;           \
        const int64_t blocks = (batch + FPB - 1) / FPB;                                               \
        if (kind == NEO_HIP_R2C)                                                                      \
            hipLaunchKernelGGL((k_r2c_lds<M, C>), dim3(unsigned(blocks)), dim3(FPB * T), 0, s,         \
                               static_cast<const R*>(in), static_cast<C*>(out), tw, batch);           \
        else                                                                                          \
            hipLaunchKernelGGL((k_c2r_lds<M, C>), dim3(unsigned(blocks)), dim3(FPB * T), 0, s,         \
                               static_cast<const C*>(in), static_cast<R*>(out), tw, batch);           \
        break;                                                                                        \
    }
    switch (m_order) {
        NEO_REAL_CASE(0) NEO_REAL_CASE(1) NEO_REAL_CASE(2) NEO_REAL_CASE(3) NEO_REAL_CASE(4) NEO_REAL_CASE(5)
        NEO_REAL_CASE(6) NEO_REAL_CASE(7) NEO_REAL_CASE(8) NEO_REAL_CASE(9) NEO_REAL_CASE(10)
        NEO_REAL_CASE(11) NEO_REAL_CASE(12)
        default: return fail(NEO_HIP_EINVAL, "real lds: bad order %d", m_order);
    }
#undef NEO_REAL_CASE
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
}

// Large c2c: radix-16 passes (remainder radix last), ping-pong through scratch
// so that `in == out` is safe; the last pass writes `out`.
template<class C>
int run_c2c_global(const plan_t* p, int order, const C* in, C* out, int dir, hipStream_t s)
{
    const int64_t n = int64_t(1) << order;
    const int K = int(p->radix.size());
    const C* src = in;
    const C* split = static_cast<const C*>(p->d_split);
    int64_t ns = 1;
    for (int i = 0; i < K; ++i) {
        C* dst = (i == K - 1) ? out : static_cast<C*>(p->d_scratch[i & 1]);
        const int R = p->radix[size_t(i)];
        const C* twr = static_cast<const C*>(p->d_ptw) + p->ptw_off[size_t(i)];
#define NEO_LPASS(RR)                                                                                      \
    {                                                                                                      \
        const unsigned blocks = unsigned(p->batch * (n / RR) / pass_cols<RR>());                           \
        if (dir < 0)                                                                                       \
            hipLaunchKernelGGL((k_pass_lds<RR, -1, C>), dim3(blocks), dim3(256), 0, s, src, dst, split,     \
                               p->lo_bits, twr, n, ns, p->batch);                                          \
        else                                                                                               \
            hipLaunchKernelGGL((k_pass_lds<RR, +1, C>), dim3(blocks), dim3(256), 0, s, src, dst, split,     \
                               p->lo_bits, twr, n, ns, p->batch);                                          \
    }
        switch (R) {
            case 64: NEO_LPASS(64) break;
            case 128: NEO_LPASS(128) break;
            case 256: NEO_LPASS(256) break;
            case 512: NEO_LPASS(512) break;
            case 1024: NEO_LPASS(1024) break;
            default: return fail(NEO_HIP_ERUNTIME, "bad pass radix %d", R);
        }
#undef NEO_LPASS
        NEO_HIP_LAUNCH_CHECK();
        src = dst;
        ns *= R;
    }
    return NEO_HIP_OK;
}

template<class C>
int upload(void** dst, const std::vector<C>& v)
{
    if (int rc = dalloc(dst, v.size() * sizeof(C))) return rc;  // pooled (dmem.hip)
    NEO_HIP_CHECK(hipMemcpy(*dst, v.data(), v.size() * sizeof(C), hipMemcpyHostToDevice));
    return NEO_HIP_OK;
}

void free_plan(plan_t* p)
{
    if (!p) return;
    // pooled (dmem.hip): freeing waits for nothing, so the plan's streams are joined first
    (void)p->used.join();
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    dfree(p->d_tw);
    dfree(p->d_split);
    dfree(p->d_split2);
    dfree(p->d_ptw);
    for (auto* s : p->d_scratch) dfree(s);
    dfree(p->d_in);
    dfree(p->d_out);
    // p->stream is one of the device's shared streams (dmem.hip)
    delete p;
}

template<class C>
int setup_tables(plan_t* p)
{
    const int io = inner_order(p);
    int rc = NEO_HIP_OK;
    if (io >= 0 && io <= kLdsMaxOrder) {
        std::vector<C> t = make_twiddle_table<C>(int64_t(1) << io);
        if (p->kind != NEO_HIP_C2C) {
            std::vector<C> t2 = make_twiddle_table<C>(int64_t(2) << io);
            t.insert(t.end(), t2.begin(), t2.end());
        }
        if ((rc = upload(&p->d_tw, t))) return rc;
    } else if (io > kLdsMaxOrder) {
        p->lo_bits = (io + 1) / 2;
        if ((rc = upload(&p->d_split, make_split_table<C>(io, p->lo_bits)))) return rc;
        // ceil(io/kPassBits) passes, bits spread evenly (R = 64..1024, in LDS)
        const int passes = (io + kPassBits - 1) / kPassBits;
        std::vector<C> ptw;
        for (int i = 0, left = io; i < passes; ++i) {
            const int bits = (left + (passes - i) - 1) / (passes - i);
            left -= bits;
            p->radix.push_back(1 << bits);
            p->ptw_off.push_back(ptw.size());
            const std::vector<C> t = make_twiddle_table<C>(int64_t(1) << bits);
            ptw.insert(ptw.end(), t.begin(), t.end());
        }
        if ((rc = upload(&p->d_ptw, ptw))) return rc;
        const int64_t inner = int64_t(1) << io;
        const int nscratch = p->kind == NEO_HIP_C2C ? 2 : 3;
        for (int i = 0; i < nscratch; ++i)
            if (dalloc(&p->d_scratch[i], size_t(inner * p->batch) * sizeof(C)))
                return fail(NEO_HIP_ENOMEM, "scratch allocation failed");
        if (p->kind != NEO_HIP_C2C) {
            p->lo_bits2 = (io + 2) / 2;
            if ((rc = upload(&p->d_split2, make_split_table<C>(io + 1, p->lo_bits2)))) return rc;
        }
    }
    return NEO_HIP_OK;
}

template<class C>
int execute(neo_hip_fft_plan* p, const void* in, void* out, int direction, hipStream_t s)
{
    using R = real_of<C>;
    const int io = inner_order(p);
    const C* tw = static_cast<const C*>(p->d_tw);
    if (p->kind == NEO_HIP_C2C) {
        const C* ci = static_cast<const C*>(in);
        C* co = static_cast<C*>(out);
        if (io <= kLdsMaxOrder)
            return direction < 0 ? launch_c2c_lds<-1>(io, ci, co, tw, p->batch, s)
                                 : launch_c2c_lds<+1>(io, ci, co, tw, p->batch, s);
        return run_c2c_global(p, io, ci, co, direction, s);
    }
    if (io < 0) {  // order 0 real transform
        const unsigned blocks = unsigned((p->batch + 255) / 256);
        if (p->kind == NEO_HIP_R2C)
            hipLaunchKernelGGL((k_r2c_order0<C>), dim3(blocks), dim3(256), 0, s, static_cast<const R*>(in),
                               static_cast<C*>(out), p->batch);
        else
            hipLaunchKernelGGL((k_c2r_order0<C>), dim3(blocks), dim3(256), 0, s, static_cast<const C*>(in),
                               static_cast<R*>(out), p->batch);
        NEO_HIP_LAUNCH_CHECK();
        return NEO_HIP_OK;
    }
    if (io <= kLdsMaxOrder) return launch_real_lds<C>(p->kind, io, in, out, tw, p->batch, s);
    const int64_t m = int64_t(1) << io, total = m * p->batch;
    const unsigned blocks = unsigned((total + 255) / 256);
    C* z = static_cast<C*>(p->d_scratch[2]);
    const C* split2 = static_cast<const C*>(p->d_split2);
    if (p->kind == NEO_HIP_R2C) {
        int rc = run_c2c_global(p, io, static_cast<const C*>(in), z, -1, s);
        if (rc) return rc;
        hipLaunchKernelGGL((k_r2c_split_global<C>), dim3(blocks), dim3(256), 0, s, z, static_cast<C*>(out), split2,
                           p->lo_bits2, m, p->batch);
        NEO_HIP_LAUNCH_CHECK();
        return NEO_HIP_OK;
    }
    hipLaunchKernelGGL((k_c2r_join_global<C>), dim3(blocks), dim3(256), 0, s, static_cast<const C*>(in), z, split2,
                       p->lo_bits2, m, p->batch);
    NEO_HIP_LAUNCH_CHECK();
    return run_c2c_global(p, io, static_cast<const C*>(z), static_cast<C*>(out), +1, s);
}

}  // namespace

extern "C" {

NEO_HIP_API int neo_hip_fft_max_order(void) { return kMaxOrder; }

NEO_HIP_API int neo_hip_fft_plan_create(int order, int64_t batch, int kind, int device, neo_hip_fft_plan** out)
{
    if (!out) return fail(NEO_HIP_EINVAL, "plan pointer is null");
    *out = nullptr;
    const bool f64 = (kind & NEO_HIP_F64) != 0;
    kind &= ~NEO_HIP_F64;
    if (order < 0 || order > kMaxOrder)
        return fail(NEO_HIP_EINVAL, "unsupported order '%d' (max_order %d)", order, kMaxOrder);
    if (batch < 1) return fail(NEO_HIP_EINVAL, "batch must be >= 1");
    if (kind != NEO_HIP_C2C && kind != NEO_HIP_R2C && kind != NEO_HIP_C2R)
        return fail(NEO_HIP_EINVAL, "bad fft kind %d", kind);
    device_guard g(device);
    if (g.rc) return g.rc;
    auto* p = new plan_t{};
    p->order = order;
    p->kind = kind;
    p->f64 = f64;
    p->batch = batch;
    p->n = int64_t(1) << order;
    (void)hipGetDevice(&p->device);
    auto bail = [&](int code) {
        free_plan(p);
        return code;
    };
    if (int rc = shared_stream(&p->stream)) return bail(rc);
    if (int rc = f64 ? setup_tables<cd>(p) : setup_tables<cf>(p)) return bail(rc);
    const size_t rs = f64 ? sizeof(double) : sizeof(float), cs = 2 * rs;
    const size_t cbytes = size_t(p->n) * cs, rbytes = size_t(p->n) * rs;
    const size_t hbytes = size_t(p->n / 2 + 1) * cs;
    p->in_bytes = size_t(batch) * (kind == NEO_HIP_C2C ? cbytes : kind == NEO_HIP_R2C ? rbytes : hbytes);
    p->out_bytes = size_t(batch) * (kind == NEO_HIP_C2C ? cbytes : kind == NEO_HIP_R2C ? hbytes : rbytes);
    *out = p;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_fft_plan_destroy(neo_hip_fft_plan* p)
{
    if (!p) return NEO_HIP_OK;
    device_guard g(p->device);
    free_plan(p);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_fft_execute(neo_hip_fft_plan* p, const void* in, void* out, int direction, void* stream)
{
    if (!p || !in || !out) return fail(NEO_HIP_EINVAL, "null plan or buffer");
    if (p->kind == NEO_HIP_C2C && direction != -1 && direction != 1)
        return fail(NEO_HIP_EINVAL, "direction must be -1 (forward) or +1 (backward)");
    device_guard g(p->device);
    if (g.rc) return g.rc;
    hipStream_t s = as_stream(stream);  // NULL = the HIP null stream (torch's default stream)
    if (int rc = p->used.note(s)) return rc;
    return p->f64 ? execute<cd>(p, in, out, direction, s) : execute<cf>(p, in, out, direction, s);
}

NEO_HIP_API int neo_hip_fft_execute_host(neo_hip_fft_plan* p, const void* in, void* out, int direction)
{
    if (!p || !in || !out) return fail(NEO_HIP_EINVAL, "null plan or buffer");
    device_guard g(p->device);
    if (g.rc) return g.rc;
    if ((!p->d_in && dalloc(&p->d_in, p->in_bytes)) || (!p->d_out && dalloc(&p->d_out, p->out_bytes)))
        return fail(NEO_HIP_ENOMEM, "fft staging allocation failed");
    NEO_HIP_CHECK(hipMemcpyAsync(p->d_in, in, p->in_bytes, hipMemcpyHostToDevice, p->stream));
    int rc = neo_hip_fft_execute(p, p->d_in, p->d_out, direction, p->stream);
    if (rc) return rc;
    NEO_HIP_CHECK(hipMemcpyAsync(out, p->d_out, p->out_bytes, hipMemcpyDeviceToHost, p->stream));
    NEO_HIP_CHECK(hipStreamSynchronize(p->stream));
    return NEO_HIP_OK;
}

}  // extern "C"
