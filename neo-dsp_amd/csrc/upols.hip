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
//
// This file: the single-block step (MAC + finish, or one launch with the last-arriver
// tail), the upola_convolver_v2 piece kernel, the handle and the neo_hip_upols_* C-ABI.
// upols_batch.hip: T blocks per pass (process_blocks). upols_setup.hip: partitioning
// and normalization. upols_device.hpp / upols_handle.hpp: what they share.
#include "upols_device.hpp"
#include "upols_handle.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace neo_hip {

// One whole block step for every channel (grid C x S, 256 lanes). Workgroup (c, s)
// accumulates partitions [p0, p1) into a partial spectrum; split 0 first runs the
// window r2c and inserts FDL row w. Each workgroup publishes its slab, and the last
// of a channel's S workgroups to arrive (agent-scope release -> counter -> acquire,
// cdna_hip_programming.md §6 G16 / split-K seam) sums the slabs in the fixed order
// s = 0..S-1 and runs the c2r: one launch per block, deterministic results.
// TAIL (upola_convolver_v2 sub-block pieces): no window / insert, partitions p >= 1 only
// (overlap_add_convolver.hpp:96-108), slabs summed by k_upola2_piece.
// latency-mode probe builds (NEO_PS_PROBE): thread 0 stamps point i of the plain step into mk
#ifdef NEO_PS_PROBE
#define NEO_STEP_MARK(i)                                    \
    do {                                                    \
        if (mk && threadIdx.x == 0) mk[i] = wall_clock64(); \
    } while (0)
#else
#define NEO_STEP_MARK(i) \
    do {                 \
    } while (0)
#endif

// the LDS of one step workgroup (k_upols_step, k_plain_persist)
template<int B>
struct step_lds {
    using K = upols_cfg<B>;
    __attribute__((aligned(16))) cf xnew[B];  // new spectrum; later the summed spectrum
    cf fft[K::LL];
    cf tw[K::TW1 + K::TW2];
    __attribute__((aligned(16))) float4 red[K::RPI > 1 ? 256 * 2 * K::VPT : 1];
    int last;
};

// The step of workgroup (c, s): returns true in the workgroup that ran the channel's tail (FUSED:
// the last split to arrive). WT (the latency mode's persistent plain step): the input block read
// at system scope and the output stored write-through.
template<int B, bool FUSED, bool OLA, bool TAIL, int UNROLL, bool WT = false>
__device__ __forceinline__ bool upols_step_wg(step_lds<B>& L, int c, int s,
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, cf* __restrict__ part, int* __restrict__ arrivals,
    const cf* __restrict__ twg, int P, int ring, int S, int rows, int w, int64_t cstride, int64_t pstride, int pc,
    unsigned long long* mk = nullptr)
{
    (void)mk;
    using K = upols_cfg<B>;
    static_assert(!(TAIL && FUSED), "the v2 tail is summed by k_upola2_piece");
    cf* xnew = L.xnew;
    cf* fft = L.fft;
    cf* tw = L.tw;
    float4* red = L.red;
    int& last = L.last;

    const int tid = threadIdx.x;
    const int p0 = s * rows, p1 = min(P, p0 + rows);
    const int64_t crow = int64_t(c) * cstride;  // channel base in H / FDL (complex units); row p at + p * pstride
    const int64_t ps4 = pstride / 2;            // row stride in float4 units

    if (!TAIL && s == 0) {
        const float* in_c = in + int64_t(c) * ld_in;
        float* prev_c = prev + int64_t(c) * B;
        window_fft<B, OLA, (B / 8 <= 256 ? 8 : B / 256), WT>(prev_c, in_c, fft, tw, tid, twg);
        NEO_STEP_MARK(1);
        cf* row = fdl + crow + int64_t(w) * pstride;
        for (int k = tid; k < B; k += 256) {
            const cf x = r2c_split<B>(fft, tw + K::TW1, k);
            xnew[k] = x;
            row[k] = x;
        }
        if constexpr (!OLA && !WT) {  // the window's second half becomes the next call's first half (WT: window_fft)
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
    // main loop over [pbeg, pend): UNROLL row-groups in flight, no bounds checks inside.
    // Filter rows below `pc` use the default (cacheable) policy so they can stay resident
    // in the 256 MiB Infinity Cache across steps; everything else streams nontemporally.
    auto mac_rows = [&]<bool NTH>(int pbeg, int pend) {
        int p = pbeg + rs;
        for (; p + (UNROLL - 1) * K::RPI < pend; p += UNROLL * K::RPI) {
            float4 hv[UNROLL][K::VPT], xv[UNROLL][K::VPT];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int pp = p + u * K::RPI;
                const int fr = w >= pp ? w - pp : w - pp + ring;  // fdl_index.hpp:28-31 ring
#pragma unroll
                for (int v = 0; v < K::VPT; ++v) {
                    const int q = q0 + v * K::QT;
                    hv[u][v] = ld4<NTH>(H4 + int64_t(pp) * ps4 + q);
                    xv[u][v] = ld4_nt(F4 + int64_t(fr) * ps4 + q);
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                for (int v = 0; v < K::VPT; ++v) mac2(a[2 * v], a[2 * v + 1], hv[u][v], xv[u][v]);
        }
        for (; p < pend; p += K::RPI) {
            const int fr = w >= p ? w - p : w - p + ring;
#pragma unroll
            for (int v = 0; v < K::VPT; ++v) {
                const int q = q0 + v * K::QT;
                mac2(a[2 * v], a[2 * v + 1], ld4<NTH>(H4 + int64_t(p) * ps4 + q), ld4_nt(F4 + int64_t(fr) * ps4 + q));
            }
        }
    };
    const int pmid = min(p1, max(pstart, pc));
    if (pmid > pstart) mac_rows.template operator()<false>(pstart, pmid);
    if (p1 > pmid) mac_rows.template operator()<true>(pmid, p1);
    if (s < 2) NEO_STEP_MARK(2 + s);  // MAC loop issued (its loads land at the first use below)

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
        c2r_tail<B, OLA, (B / 4 <= 256 ? 4 : B / 256), false, false, WT>(xnew, fft, tw, out_c, prev + int64_t(c) * B, tid);
        return true;
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
    if constexpr (!FUSED) return false;  // k_upols_finish sums the slabs in the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep the release's wait (G16 pitfall)
        const int before = __hip_atomic_fetch_add(arrivals + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = before == S - 1;
    }
    __syncthreads();
    if (!last) return false;  // uniform per workgroup
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(arrivals + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next step
    }
    NEO_STEP_MARK(4);  // the tail: every split arrived
    if (s != 0)
        for (int i = tid; i < K::TW1 + K::TW2; i += 256) tw[i] = twg[i];
    __syncthreads();

    // sum the S slabs in order s = 0..S-1, 8 loads in flight
    const float4* p4 = reinterpret_cast<const float4*>(part + int64_t(c) * S * B);
    if constexpr (K::Q > 256) {
        // B >= 1024: QI float4 per lane and slab; every lane's loads of SB slabs in flight at once
        // (one trip to memory per SB slabs instead of one per float4: the latency-bound one-channel
        // step at B = 4096), the same order per bin
        constexpr int QI = K::Q / 256, SB = QI >= 8 ? 2 : 16 / QI;
        float4 sum[QI];
#pragma unroll
        for (int i = 0; i < QI; ++i) sum[i] = p4[tid + i * 256];
        int t = 1;
        for (; t + SB - 1 < S; t += SB) {
            float4 r[SB][QI];
#pragma unroll
            for (int u = 0; u < SB; ++u)
#pragma unroll
                for (int i = 0; i < QI; ++i) r[u][i] = p4[int64_t(t + u) * K::Q + tid + i * 256];
#pragma unroll
            for (int u = 0; u < SB; ++u)
#pragma unroll
                for (int i = 0; i < QI; ++i) {
                    sum[i].x += r[u][i].x; sum[i].y += r[u][i].y; sum[i].z += r[u][i].z; sum[i].w += r[u][i].w;
                }
        }
        for (; t < S; ++t) {
            float4 r[QI];
#pragma unroll
            for (int i = 0; i < QI; ++i) r[i] = p4[int64_t(t) * K::Q + tid + i * 256];
#pragma unroll
            for (int i = 0; i < QI; ++i) {
                sum[i].x += r[i].x; sum[i].y += r[i].y; sum[i].z += r[i].z; sum[i].w += r[i].w;
            }
        }
#pragma unroll
        for (int i = 0; i < QI; ++i) reinterpret_cast<float4*>(xnew)[tid + i * 256] = sum[i];
    } else
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
    NEO_STEP_MARK(5);  // slabs summed
    c2r_tail<B, OLA, (B / 4 <= 256 ? 4 : B / 256), false, false, WT>(xnew, fft, tw, out_c, prev + int64_t(c) * B, tid);
    NEO_STEP_MARK(6);  // output stores issued
    return true;
}

template<int B, bool FUSED, bool OLA, bool TAIL = false, int UNROLL = upols_cfg<B>::U>
__global__ __launch_bounds__(256, (B <= 1024 ? 8 : 2)) void k_upols_step(
    const float* __restrict__ in, int64_t ld_in, float* __restrict__ out, int64_t ld_out, float* __restrict__ prev,
    const cf* __restrict__ H, cf* __restrict__ fdl, cf* __restrict__ part, int* __restrict__ arrivals,
    const cf* __restrict__ twg, int P, int ring, int S, int rows, int w, int64_t cstride, int64_t pstride, int pc)
{
    __shared__ step_lds<B> L;
    const int c = blockIdx.x / S, s = blockIdx.x - c * S;
    (void)upols_step_wg<B, FUSED, OLA, TAIL, UNROLL>(L, c, s, in, ld_in, out, ld_out, prev, H, fdl, part, arrivals, twg,
                                                     P, ring, S, rows, w, cstride, pstride, pc);
}

// Latency mode of a handle without streaming levels (fewer than 64 partitions, or the levels off;
// blocks up to 4096: the reference benchmark's shape, extra/benchmark/src/convolution.cpp:47-55):
// the fused plain step's C x S workgroups stay resident across steps. Per step n every workgroup
// waits for step n - 1 to be complete (blk_done: every channel's tail summed its slabs, reset its
// split counter and wrote its output; split 0 wrote the FDL row and the previous block), takes the
// record (workgroup 0 polls the mailbox, ps_record) and runs its split (upols_step_wg, the input
// read and the output stored at system scope). The tail of each channel counts the channel in; the
// last one tells the host (mb->done) and the workgroups (blk_done).
struct plain_persist_args : persist_ctl {
    const cf* H;
    cf* fdl;
    cf* part;
    int* arrivals;
    float* prev;
    const cf* twg;
    int64_t ld_in, ld_out, cstride, pstride;
    int C, P, ring, S, rows, pc;
};

template<int B, bool OLA>
__global__ __launch_bounds__(256) void k_plain_persist(plain_persist_args pa)
{
    __shared__ step_lds<B> L;
    __shared__ uint64_t io[2];
    __shared__ int go;
    const int c = int(blockIdx.x) / pa.S, s = int(blockIdx.x) - c * pa.S;
    const bool lead = blockIdx.x == 0;
    unsigned long long t_seen = 0;  // thread 0 of workgroup 0: when the step's record was read
    int w = pa.w0;                  // ring row of step n
    for (int64_t n = pa.n0;; ++n, w = w + 1 == pa.ring ? 0 : w + 1) {
        if (threadIdx.x == 0) {
            bool ok = ps_wait(pa, [&] { return ps_ld(pa.flags + 0) >= n - 1; });
            if (ok) ps_acquire();  // the slabs, FDL row and previous block of step n - 1 (other workgroups')
            go = ps_record(pa, n, lead, gridDim.x > 1, ok, io, t_seen);
        }
        __syncthreads();
        if (!go) break;
        // two rows in flight at B >= 2048 (one row is 8 or 16 float4 per lane: a trip to memory per row)
        const bool tail = upols_step_wg<B, true, OLA, false, (upols_cfg<B>::VPT >= 4 ? 2 : upols_cfg<B>::U), true>(
            L, c, s, reinterpret_cast<const float*>(io[0]), pa.ld_in, reinterpret_cast<float*>(io[1]), pa.ld_out,
            pa.prev, pa.H, pa.fdl, pa.part, pa.arrivals, pa.twg, pa.P, pa.ring, pa.S, pa.rows, w, pa.cstride,
            pa.pstride, pa.pc,
#ifdef NEO_PS_PROBE
            c == 0 ? pa.tl + 2 * kPsRing + 8 * (n % kPsRing) : nullptr
#else
            nullptr
#endif
        );
        if (tail) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the output's write-through stores complete
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                int64_t* arr = pa.flags + kPsFlagArrive + n % kPsArr;
                if (__hip_atomic_fetch_add(arr, int64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == pa.C - 1) {
                    ps_st(arr, 0);  // free for step n + kPsArr
                    const unsigned long long t_done = wall_clock64();
                    __hip_atomic_store(&pa.mb->done, n + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    pa.tl[2 * (n % kPsRing) + 1] = t_done;
                    ps_acquire();  // the other channels' releases, passed on by the one below
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    ps_st(pa.flags + 0, n);
                }
            }
        }
        if (lead && threadIdx.x == 0) pa.tl[2 * (n % kPsRing)] = t_seen;
    }
    if (lead && threadIdx.x == 0) __hip_atomic_store(&pa.mb->alive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int plain_persist_launch(upols_t* h, const persist_ctl& ctl, int64_t ld_in, int64_t ld_out, bool* launched)
{
    *launched = false;
    if (h->C * h->S > 256) return fail(NEO_HIP_EINVAL, "latency mode: %d x %d plain step workgroups", h->C, h->S);
    plain_persist_args pa{};
    static_cast<persist_ctl&>(pa) = ctl;
    pa.H = h->H;
    pa.fdl = h->fdl;
    pa.part = h->part;
    pa.arrivals = h->arrivals;
    pa.prev = h->prev;
    pa.twg = h->tw;
    pa.ld_in = ld_in;
    pa.ld_out = ld_out;
    pa.cstride = h->cstride;
    pa.pstride = h->pstride;
    pa.C = h->C;
    pa.P = h->P;
    pa.ring = h->ring;
    pa.S = h->S;
    pa.rows = h->rows;
    pa.pc = h->pc;
    const unsigned grid = unsigned(h->C) * unsigned(h->S);
    bool room = false;
    if (h->ola) {
        NEO_UPOLS_DISPATCH(h->B, room = persist_room(h, reinterpret_cast<const void*>(&k_plain_persist<BB, true>), int(grid));
                           if (room) hipLaunchKernelGGL((k_plain_persist<BB, true>), dim3(grid), dim3(256), 0, h->ps_stream, pa))
    } else {
        NEO_UPOLS_DISPATCH(h->B, room = persist_room(h, reinterpret_cast<const void*>(&k_plain_persist<BB, false>), int(grid));
                           if (room) hipLaunchKernelGGL((k_plain_persist<BB, false>), dim3(grid), dim3(256), 0, h->ps_stream, pa))
    }
    if (!room) return NEO_HIP_OK;
    *launched = true;
    NEO_HIP_LAUNCH_CHECK();
    return NEO_HIP_OK;
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

}  // namespace neo_hip

using namespace neo_hip;


int neo_hip::setup_join(upols_t* h, bool device_input)
{
    if (int rc = h->used.join()) return rc;
    if (device_input)
        if (int rc = null_join()) return rc;
    if (int rc = lvl_join(h, h->stream)) return rc;
    NEO_HIP_CHECK(hipStreamSynchronize(h->stream));
    return NEO_HIP_OK;
}

namespace {

int reset_state(upols_t* h, hipStream_t s)
{
    if (int rc = lvl_join(h, s)) return rc;
    NEO_HIP_CHECK(hipMemsetAsync(h->fdl, 0, size_t(h->C) * h->ring * h->B * sizeof(cf), s));
    NEO_HIP_CHECK(hipMemsetAsync(h->prev, 0, size_t(h->C) * h->B * sizeof(float), s));
    NEO_HIP_CHECK(hipMemsetAsync(h->arrivals, 0, size_t(h->C) * sizeof(int), s));
    if (h->v2) {
        NEO_HIP_CHECK(hipMemsetAsync(h->window, 0, size_t(h->C) * 2 * h->B * sizeof(float), s));
        NEO_HIP_CHECK(hipMemsetAsync(h->tmp, 0, size_t(h->C) * h->B * sizeof(cf), s));
    }
    h->wpos = 0;
    h->in_pos = 0;
    h->lv_n = -1;  // streaming levels re-prime at the next step (zeroing: lvl_prime)
    h->fdl_zero = true;
    return NEO_HIP_OK;
}

void destroy(upols_t* h)
{
    if (!h) return;
    (void)persist_stop(h);
    if (h->ps_stream) (void)hipStreamDestroy(h->ps_stream);
    hfree(h->ps_mb);
    dfree(h->ps_flags);
    dfree(h->ps_tl);
    for (auto& g : h->events)
        for (auto& e : g.e) (void)hipEventDestroy(e);
    lvl_free(h);  // joins the background stream first
    // device buffers back to the pool (dmem.hip): no device-wide synchronization; the caller
    // joined every stream that used them
    dfree(h->H);  // the FDL shares H's allocation (rows [nrows, 2 nrows))
    dfree(h->part);
    dfree(h->prev);
    dfree(h->arrivals);
    dfree(h->window);
    dfree(h->tmp);
    hfree(h->io_host);  // h->io is its device mapping
    dfree(h->samples_dev);
    dfree(h->part_b);
    dfree(h->tail);
    dfree(h->off_hf);
    dfree(h->off_y);
    dfree(h->off_tail);
    hfree(h->samples_host);
    delete h;  // h->stream is shared (a group's, or one of the device's four: dmem.hip)
}

int launch_step(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s)
{
    if (int rc = note_stream(h, s)) return rc;
    if (h->persist) return persist_process(h, in, ld_in, out, ld_out, 1);  // synchronous: s is not used
    return launch_step_normal(h, in, ld_in, out, ld_out, s);
}

}  // namespace

int neo_hip::launch_step_normal(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s)
{
    if (h->ahead) return launch_levels(h, in, ld_in, out, ld_out, s);
    if (int rc = lvl_join(h, s)) return rc;
    upols_t::ev_group* ev = nullptr;
    if (int rc = timing_begin(h, 2, &ev)) return rc;
    if (int rc = timing_mark(ev, 0, s)) return rc;
    const unsigned grid = unsigned(h->C) * unsigned(h->S);
#define NEO_STEP(FU, OL)                                                                                      \
    NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_step<BB, FU, OL>), dim3(grid), dim3(256), 0, s, in, ld_in, \
                                                out, ld_out, h->prev, h->H, h->fdl, h->part, h->arrivals, h->tw,   \
                                                h->P, h->ring, h->S, h->rows, h->wpos, h->cstride, h->pstride,  \
                                                h->pc))
    if (h->fused) {
        if (h->ola) NEO_STEP(true, true) else NEO_STEP(true, false)
    } else {
        if (h->ola) NEO_STEP(false, true) else NEO_STEP(false, false)
    }
#undef NEO_STEP
    NEO_HIP_LAUNCH_CHECK();
    h->fdl_zero = false;
    if (int rc = timing_mark(ev, 1, s)) return rc;
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
    h->lv_n = -1;
    return NEO_HIP_OK;
}

namespace {

// One v2 piece of n samples at block position h->in_pos (n <= B - in_pos).
int launch_piece(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int n, hipStream_t s)
{
    const int sum_first = h->in_pos == 0;
    if (int rc = lvl_join(h, s)) return rc;
    h->lv_n = -1;
    h->fdl_zero = false;
    if (sum_first) {  // tail MAC over partitions p >= 1 into the split slabs
        const unsigned grid = unsigned(h->C) * unsigned(h->S);
        NEO_UPOLS_DISPATCH(h->B, hipLaunchKernelGGL((k_upols_step<BB, false, true, true>), dim3(grid), dim3(256), 0, s,
                                                    in, ld_in, out, ld_out, h->prev, h->H, h->fdl, h->part,
                                                    h->arrivals, h->tw, h->P, h->ring, h->S, h->rows, h->wpos,
                                                    h->cstride, h->pstride, h->pc))
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
    if (int rc = note_stream(h, s)) return rc;
    const int B = h->B;
    const int T = h->batch ? batch_blocks(h) : 1;
    const bool a16 = !((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) &&
                     !((ld_in | ld_out) & 3);
    if (h->persist) {  // latency mode: every block through the persistent kernel, complete on return
        if (n % B || !a16) return fail(NEO_HIP_EINVAL, "latency mode: whole 16-byte aligned blocks");
        return persist_process(h, in, ld_in, out, ld_out, n / B);
    }
    if (!h->v2) {
        if (n % B) return fail(NEO_HIP_EINVAL, "upols/upola convolvers take whole blocks (%lld samples, block %d)",
                               (long long)n, B);
        if (!a16) return fail(NEO_HIP_EINVAL, "device I/O must be 16-byte aligned (ld multiple of 4)");
    }
    // Streaming levels: a batched pass leaves them to re-prime at the next single-block step
    // (window 0 of every level computed whole, 2 x 128 far launches), so with the levels on
    // only whole T-block batches run (the rest stream, one prime per call at most), and a
    // call of fewer than kStreamKeep batches' blocks on primed levels streams them all.
    constexpr int kStreamKeep = 4;
    const bool stream_all = h->ahead && h->lv_n >= 0 && n < int64_t(kStreamKeep) * T * B;
    int64_t done = 0;
    while (done < n) {
        const float* ip = in + done;
        float* op = out + done;
        int rc;
        // offline windows: 256 or 128 whole blocks left, every block known (batching on)
        const int64_t left = (n - done) / B;
        if (h->off && h->batch && !stream_all && h->in_pos == 0 && a16 && done % 4 == 0 && left >= kFarT) {
            const int wp = left >= int64_t(kFarT) * kOffMaxWP ? kOffMaxWP : 1;
            if ((rc = launch_offline(h, ip, ld_in, op, ld_out, wp, s))) return rc;
            done += int64_t(wp) * kFarT * B;
            continue;
        }
        // the largest power-of-two batch (<= T) of whole blocks left, one pass over H + FDL
        int tb = 1;
        while (!stream_all && tb * 2 <= T && n - done >= int64_t(tb) * 2 * B) tb *= 2;
        if (h->ahead && tb < T) tb = 1;
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


// The offline windows' ring, 128 (nseg + 2) rows, is a multiple of 256 rows: a channel stride of
// 5 x 2^20 bytes at B = 512 made the streaming step 4 % slower at c5full (same-box A/B: 9.29-9.49
// vs 9.68-9.74 Gsamples/s at 20 steps, as with the ring of P + 31 rows); one more row keeps it odd
// and restores it (9.58-9.83). profiles/r6_ab_ring.json
#ifndef NEO_OFF_RING_PAD
#define NEO_OFF_RING_PAD 1  // diagnostic builds (A/B): 0 = the even ring
#endif
namespace {
int create_convolver(int channels, int block, int partitions, int device, bool ola, bool v2,
                     const neo_hip_upols_opts* opt, neo_hip_upols** out, hipStream_t borrow = nullptr)
{
    if (!out) return fail(NEO_HIP_EINVAL, "handle pointer is null");
    const neo_hip_upols_opts o = opt ? *opt : neo_hip_upols_opts{-1, 0, 0, 0, -1, -1, 0, 0, 0, 0};
    if (o.fused < -1 || o.fused > 1 || o.levels < -1 || o.levels > 1 || o.far_level < -1 || o.far_level > 2 ||
        o.split_workgroups < 0 ||
        (o.batch_blocks && (o.batch_blocks < 2 || o.batch_blocks > kMaxBatch || (o.batch_blocks & (o.batch_blocks - 1)))) ||
        o.batch_bins < 0 || o.batch_bins > 2 || o.far_group < 0 || o.far_group > 4 || o.toep_split < 0 || o.toep_split > 2 ||
        (o.step_group != 0 && o.step_group != 1 && o.step_group != 2 && o.step_group != 4 && o.step_group != 8) ||
        o.far_phase2 < 0 || o.far_phase2 > 2)
        return fail(NEO_HIP_EINVAL, "invalid convolver options");
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
    plan_levels(partitions, h->lv, o.far_level);
    h->far_k = o.far_group;
    h->toep_jh = o.toep_split;
    h->f2mode = o.far_phase2;
    h->sg = o.step_group ? o.step_group : step_group_for(channels, block, partitions);
    h->bg_pad = bg_pad_for(channels, block);
    // the far level's form: the stored spectra (phase 1 + 2) by default; recomputed every window
    // (far2r_role) on request -- fewer bytes (C5: 15 instead of 23 rows per column and step) but
    // 2 nseg + 1 transforms per unit and window: same-box A/B with step groups, stored vs
    // recomputed, us per step: c5full 107-109 vs 115-124 (VALU), C5 15.9 vs 15.8-16.4, C4 12.4 vs
    // 18-20 (the 27-transform chain of 13 segments bounds the background launch)
    h->far_raw = h->lv.nseg && o.far_level == 2;
    if (h->lv.nseg) h->ring = std::max(h->ring, kFarRing);  // far slices read 383 blocks back
    // recomputed: a window's slices read the band's rows back to t_W - 128 (nseg + 2) > t_W - P - 128
    // while blocks up to t_W + 3 may be written beside them (step groups)
    if (h->far_raw) h->ring = std::max(h->ring, partitions + 2 * kFarT);
    // offline windows (k_off_mac): a pass of 128 wp blocks reads rows back to t_W - 128 nseg while
    // writing rows t_W .. t_W + 128 wp - 1
    h->off = !v2 && partitions >= kOffMinP;
    h->off_nseg = (partitions + kFarT - 1) / kFarT;
    if (h->off) h->ring = std::max(h->ring, kFarT * (h->off_nseg + kOffMaxWP) + NEO_OFF_RING_PAD);
    h->ola = ola || v2;
    h->v2 = v2;
    h->fused = 2.0 * 8.0 * double(channels) * double(partitions) * double(block) < double(kFusedMaxBytes);
    if (o.fused >= 0) h->fused = o.fused != 0;
    if (o.batch_blocks) h->bT = o.batch_blocks;
    if (o.batch_bins) h->bNB = o.batch_bins;
    // filter rows kept resident in the Infinity Cache across steps: the first pc rows of
    // every channel are read with the default policy, ~216 MiB in all (A/B on MI355X: C5
    // 0.302 -> 0.286 ms per MAC at 220 rows, C4 0.295 -> 0.282 at 400; past ~250 MiB
    // the cached rows start evicting each other)
    h->pc = int(std::min<double>(partitions, kCacheBudgetBytes / (double(channels) * block * sizeof(cf))));
    h->cstride = int64_t(h->ring) * block;
    h->pstride = block;
    // splits per channel: aim for ~1024 workgroups (4 per CU, all resident at 8 waves/SIMD;
    // A/B on MI355X: 1024 beat 512/768/2048/4096 at C4 and C5), <= 64 partial slabs
    const int target = o.split_workgroups ? o.split_workgroups : 1024;
    // >= 8 rows per split keeps the slab sum short at small C; the one-launch (latency) form
    // takes >= 16 (C3: 12 splits, 9.6 vs 10.6 us per block with 24)
    // (an explicit workgroup target is taken as given)
    // (an explicit workgroup target is taken as given); above B = 512 the one-launch form takes
    // >= 8 rows: a split's rows stream through one CU (~130 GB/s), the tail sums the slabs alone.
    // One channel, P = 32, us per step with 2 / 4 / 8 splits (normal; latency mode): B = 4096
    // 25.1 / 22.6 / 22.3 (22.5 / 21.2 / 23.4), B = 2048 16.3 / 15.2 / 15.2 (12.8 / 11.9 / 12.4),
    // B = 1024 12.5 / 12.2 / 12.7 (10.0 / 9.3 / 9.6) (tools/plain_split_sweep.py)
    const int min_rows = o.split_workgroups ? 1 : h->fused ? (block > 512 ? 8 : 16) : 8;
    int S = std::max(1, std::min({(target + channels - 1) / channels, (partitions + min_rows - 1) / min_rows, 64}));
    h->rows = (partitions + S - 1) / S;
    h->S = (partitions + h->rows - 1) / h->rows;
    // batched passes: same workgroup target, >= 2T partitions per split so the sliding FDL
    // window's warm-up (T - 1 extra rows per split) stays under half the split's rows
    h->bufload = (int64_t(h->ring - 1) * h->pstride + block) * int64_t(sizeof(cf)) < (int64_t(1) << 31);
    h->pcb = int(std::min<double>(partitions, kBatchCacheBudgetBytes / (double(channels) * block * sizeof(cf))));
    // batched MAC: 256-lane workgroups at 2 waves/SIMD -> 2 resident per CU, so 512 fills the
    // chip once with no second round (A/B, bmac_var 3: C5 0.409 -> 0.367 ms per pass, C4 0.369
    // -> 0.379 ms, within run-to-run spread)
    const int btarget = 512;
    const int bt = batch_t(block, h->bNB, h->bT);
    // workgroups per (channel, split): the batched MAC has one lane per bin, <= 256 lanes
    const int bgroups = std::max(1, block / h->bNB / 256);
    int Sb = std::max(1, std::min({(btarget + channels * bgroups - 1) / (channels * bgroups), partitions / (2 * bt), 64}));
    if (h->ring - partitions < bt - 1) h->batch = false;  // ring too short for a batch
    // streaming levels (upols_levels.hip) instead of one pass over filter + FDL per block,
    // from 64 partitions, blocks up to 1024; short filters keep the plain step, whose one pass
    // is already small (its working set sits in the Infinity Cache)
    h->ahead = !v2 && block <= 1024 && (o.levels >= 0 ? o.levels != 0 : partitions >= 64);
    h->rows_b = ((partitions + Sb - 1) / Sb + kMaxBatch - 1) / kMaxBatch * kMaxBatch;  // whole chunks of any T
    h->Sb = (partitions + h->rows_b - 1) / h->rows_b;
    const size_t rowbytes = size_t(block) * sizeof(cf);
    const size_t nrows = size_t(channels) * size_t(h->ring);  // H uses the first P rows of each channel
    auto bail = [&](int code) {
        destroy(h);
        return code;
    };
    // a group member runs its setup and host-I/O work on its group's stream (upols_group.hip),
    // every other handle on one of its device's four shared streams (dmem.hip shared_stream: a
    // stream of its own would cost ~4 ms to create and ~3 ms to destroy; the first four handles on
    // a device create them)
    h->stream = borrow;
    if (!borrow) {
#ifdef NEO_OWN_STREAM  // diagnostic builds (A/B): a stream of its own per handle, as before round 5 (never destroyed)
        if (hipStreamCreateWithFlags(&h->stream, hipStreamDefault) != hipSuccess)
            return bail(fail(NEO_HIP_ERUNTIME, "hipStreamCreate failed"));
#else
        if (int rc = shared_stream(&h->stream)) return bail(rc);
#endif
    }
    // filter and FDL in ONE allocation (FDL = rows [nrows, 2 nrows)): the LDS-DMA batched MAC
    // reaches both of a channel through a single buffer descriptor
    if (dalloc(&h->H, 2 * nrows * rowbytes) || dalloc(&h->part, size_t(channels) * h->S * rowbytes) ||
        dalloc(&h->prev, size_t(channels) * block * sizeof(float)) || dalloc(&h->arrivals, size_t(channels) * sizeof(int)) ||
        (v2 && (dalloc(&h->window, size_t(channels) * 2 * block * sizeof(float)) ||
                dalloc(&h->tmp, size_t(channels) * rowbytes))))
        return bail(fail(NEO_HIP_ENOMEM, "device allocation of %zu bytes failed", 2 * nrows * rowbytes));
    h->fdl = h->H + nrows * size_t(block);
    int rc = shared_tw(&h->tw, block);
    if (rc) return bail(rc);
    // stream-ordered zeroing, one wait at the end (the caller's later work may run on any stream)
    if (hipMemsetAsync(h->H, 0, nrows * rowbytes, h->stream) != hipSuccess)
        return bail(fail(NEO_HIP_ERUNTIME, "memset failed"));
    if ((rc = reset_state(h, h->stream))) return bail(rc);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return bail(fail(NEO_HIP_ERUNTIME, "sync failed"));
    *out = h;
    return NEO_HIP_OK;
}
}  // namespace

int neo_hip::create_handle(int channels, int block, int partitions, int device, int method, hipStream_t stream,
                           neo_hip_upols** out)
{
    const int rc = create_convolver(channels, block, partitions, device, method >= 1, method == 2, nullptr, out, stream);
    if (!rc) (*out)->grouped = true;
    return rc;
}

extern "C" {

NEO_HIP_API int neo_hip_upols_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, false, false, nullptr, out);
}

NEO_HIP_API int neo_hip_upola_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, true, false, nullptr, out);
}

NEO_HIP_API int neo_hip_upola2_create(int channels, int block, int partitions, int device, neo_hip_upols** out)
{
    return create_convolver(channels, block, partitions, device, true, true, nullptr, out);
}

NEO_HIP_API int neo_hip_upols_create_ex(int channels, int block, int partitions, int device, int method,
                                        const neo_hip_upols_opts* opts, neo_hip_upols** out)
{
    if (method < 0 || method > 2) return fail(NEO_HIP_EINVAL, "method must be 0 (upols), 1 (upola) or 2 (upola v2)");
    return create_convolver(channels, block, partitions, device, method >= 1, method == 2, opts, out);
}

NEO_HIP_API int neo_hip_upols_destroy(neo_hip_upols* h)
{
    if (!h) return NEO_HIP_OK;
    device_guard g(h->device);
    (void)persist_stop(h);
    (void)setup_join(h);
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
    if (int rc = persist_stop(h)) return rc;
    if (int rc = setup_join(h)) return rc;  // after this handle's steps on any stream
    int rc = reset_state(h, h->stream);
    if (!rc) rc = lvl_setup_prime(h);  // the next call is an ordinary streaming step
    if (rc) return rc;
    NEO_HIP_CHECK(hipStreamSynchronize(h->stream));
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_filter(neo_hip_upols* h, const void* filter, int is_device)
{
    if (!h || !filter) return fail(NEO_HIP_EINVAL, "null handle or filter");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    if (int rc = persist_stop(h)) return rc;
    if (int rc = setup_join(h, is_device != 0)) return rc;  // after this handle's steps (and a device filter's producer)
    const int64_t rows = int64_t(h->C) * h->P;
    const size_t bytes = size_t(rows) * size_t(h->B + 1) * sizeof(cf);
    const cf* src = static_cast<const cf*>(filter);
    cf* tmp = nullptr;
    if (!is_device) {
        if (int rc = dalloc(&tmp, bytes)) return rc;
        NEO_HIP_CHECK(hipMemcpyAsync(tmp, filter, bytes, hipMemcpyHostToDevice, h->stream));
        src = tmp;
    }
    int rc = pack_filter(h, src, h->stream);
    lvl_filter_changed(h);
    if (!rc) rc = reset_state(h, h->stream);
    // the reference's filter() rebuilds the convolver's state (uniform_partitioned_convolver.hpp:37-45)
    // and its next call is an ordinary block step (:47-65): the levels' setup runs here, not there
    if (!rc) rc = lvl_setup_prime(h);
    if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    dfree(tmp);  // the stream was joined above
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
    if (int rc = persist_stop(h)) return rc;
    if (int rc = setup_join(h, is_device != 0)) return rc;  // after this handle's steps (and a device IR's producer)
    const size_t bytes = size_t(h->C) * size_t(length) * sizeof(float);
    float* d = nullptr;
    if (int rc = dalloc(&d, bytes)) return rc;
    int rc = NEO_HIP_OK;
    if (hipMemcpyAsync(d, ir, bytes, is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->stream) !=
        hipSuccess)
        rc = fail(NEO_HIP_ERUNTIME, "impulse copy failed");
    if (!rc && normalize) rc = normalize_device(d, h->C, length, h->stream);
    if (!rc) rc = partition_device(d, h->C, length, h->B, true, h->H, h->tw, h->stream, h->cstride, h->pstride);
    lvl_filter_changed(h);
    if (!rc) rc = reset_state(h, h->stream);
    // the reference's filter() rebuilds the convolver's state (uniform_partitioned_convolver.hpp:37-45)
    // and its next call is an ordinary block step (:47-65): the levels' setup runs here, not there
    if (!rc) rc = lvl_setup_prime(h);
    if (hipStreamSynchronize(h->stream) != hipSuccess && !rc) rc = fail(NEO_HIP_ERUNTIME, "sync failed");
    dfree(d);
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
    // Host buffers (the plugin's processFrame pattern, DenseConvolution.cpp:62-74): the step
    // kernel reads the block from host memory and writes the output back itself over PCIe
    // (zero-copy, no DMA launches). Page-locked memory (neo_hip_host_register, hipHostMalloc)
    // is used in place; any other buffer goes through the handle's mapped pinned staging.
    float* dio = host_mapped(io);
    const bool staged = !dio || (reinterpret_cast<uintptr_t>(dio) & 15);
    if (staged) {
        if (!h->io_host) {
            if (int rc = halloc(reinterpret_cast<void**>(&h->io_host), reinterpret_cast<void**>(&h->io), bytes)) return rc;
        }
        std::memcpy(h->io_host, io, bytes);
        dio = h->io;
    }
    int rc = h->v2 ? process_samples(h, dio, h->B, dio, h->B, h->B, s) : launch_step(h, dio, h->B, dio, h->B, s);
    if (rc) return rc;
    if ((rc = spin_sync(s))) return rc;  // the block's deadline: poll, do not yield the thread
    if (staged) std::memcpy(io, h->io_host, bytes);
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
        NEO_HIP_CHECK(hipStreamSynchronize(s));  // no queued work on the old staging
        dfree(h->samples_dev);
        hfree(h->samples_host);
        h->samples_dev = nullptr;
        h->samples_host = nullptr;
        h->samples_cap = 0;
        if (int rc = dalloc(&h->samples_dev, count * sizeof(float))) return rc;
        void* dmap = nullptr;  // not used: the samples go by DMA
        if (int rc = halloc(reinterpret_cast<void**>(&h->samples_host), &dmap, count * sizeof(float))) return rc;
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

NEO_HIP_API int neo_hip_upols_set_offline(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enable && (h->v2 || h->P < kOffMinP))
        return fail(NEO_HIP_EINVAL, "offline windows take whole-block handles of >= %d partitions", kOffMinP);
    h->off = enable != 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_get_offline(neo_hip_upols* h, int* enabled, int* segments)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enabled) *enabled = h->off;
    if (segments) *segments = h->off_nseg;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_ahead(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enable && h->v2) return fail(NEO_HIP_EINVAL, "streaming levels are for whole-block upols / upola handles");
    if (enable && h->B > 1024) return fail(NEO_HIP_EINVAL, "streaming levels take blocks up to 1024");
    device_guard g(h->device);
    if (int rc = persist_stop(h)) return rc;
    if (!enable) h->persist = false;  // the latency mode runs the levels
    h->ahead = enable != 0;
    h->lv_n = -1;  // the FDL is complete at any block boundary: the next step primes the levels
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_paced(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    if (enable < 0 || enable > 2) return fail(NEO_HIP_EINVAL, "paced: 0 off, 1 a piece per call, 2 two pieces per group");
    if (enable == h->paced) return NEO_HIP_OK;
    if (int rc = persist_stop(h)) return rc;  // a resident latency-mode kernel leaves first (lv_n restarts)
    if (int rc = lvl_join(h, h->stream)) return rc;
    NEO_HIP_CHECK(hipStreamSynchronize(h->stream));
    h->paced = enable;
    h->lv_n = -1;  // the levels re-prime: no group is half issued in the other form
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_persistent(neo_hip_upols* h, int enable, double idle_ms)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    device_guard g(h->device);
    if (g.rc) return g.rc;
    if (enable) {
        if (const char* why = persist_ineligible(h)) return fail(NEO_HIP_EINVAL, "latency mode: %s", why);
        if (!(idle_ms > 0.0 && idle_ms <= 10000.0)) return fail(NEO_HIP_EINVAL, "idle_ms must be in (0, 10000]");
        if (int rc = setup_join(h)) return rc;  // this handle's steps queued on any stream come first
        h->ps_idle_ms = idle_ms;
        h->persist = true;
        h->ps_valid = false;  // the persistent schedule primes the levels at its first block
        return NEO_HIP_OK;
    }
    h->persist = false;
    return persist_stop(h);
}

NEO_HIP_API int neo_hip_upols_get_persistent(neo_hip_upols* h, int* enabled, int* running, int64_t* launches)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enabled) *enabled = h->persist;
    if (running) *running = h->ps_running && h->ps_mb && __atomic_load_n(&h->ps_mb->alive, __ATOMIC_ACQUIRE);
    if (launches) *launches = h->ps_launches;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_persist_step_times(neo_hip_upols* h, double* us, int64_t cap, int64_t* count)
{
    if (!h || (cap > 0 && !us)) return fail(NEO_HIP_EINVAL, "null handle or output");
    if (count) *count = 0;
    if (!h->ps_tl || h->lv_n <= h->ps_n0 || !h->ps_valid) return NEO_HIP_OK;
    device_guard g(h->device);
    if (g.rc) return g.rc;
    std::vector<unsigned long long> tl(2 * kPsRing);
    NEO_HIP_CHECK(hipMemcpy(tl.data(), h->ps_tl, tl.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // the last min(kPsRing - 1, steps of this launch) steps, oldest first
    const int64_t last = h->lv_n - 1, k = std::min<int64_t>({int64_t(kPsRing) - 1, last - h->ps_n0 + 1, cap});
    for (int64_t i = 0; i < k; ++i) {
        const int64_t n = last - k + 1 + i, slot = n % kPsRing;
        us[i] = double(tl[size_t(2 * slot + 1)] - tl[size_t(2 * slot)]) * 1e-2;  // 100 MHz ticks -> us
    }
    if (count) *count = k;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_get_ahead(neo_hip_upols* h, int* enabled, int* phase, int* window, int* splits)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enabled) *enabled = h->ahead;
    if (phase) *phase = int(h->lv_n < 0 ? 0 : h->lv_n % kFarT);
    if (window) *window = h->lv.nseg ? kFarT : (h->lv.n ? h->lv.T[h->lv.n - 1] : 1);
    if (splits) *splits = h->lv.n + (h->lv.nseg ? 1 : 0);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_set_timing(neo_hip_upols* h, int enable)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    if (enable < 0) return fail(NEO_HIP_EINVAL, "timing stride %d < 0", enable);
    h->timing = enable;
    h->tick = 0;
    return NEO_HIP_OK;
}

// fold the recorded event groups into the per-part sums and the per-group totals
static int drain_events(upols_t* h)
{
    for (size_t i = 0; i < h->events_used; ++i) {
        const auto& e = h->events[i];
        NEO_HIP_CHECK(hipEventSynchronize(e.e[e.n - 1]));
        float tot = 0.f;
        NEO_HIP_CHECK(hipEventElapsedTime(&tot, e.e[0], e.e[e.n - 1]));
        if (e.part == 0) h->group_ms.push_back(tot);  // step times: the caller's stream only
        for (int k = 0; k + 1 < e.n; ++k) {
            float t = 0.f;
            NEO_HIP_CHECK(hipEventElapsedTime(&t, e.e[k], e.e[k + 1]));
            h->part_ms[k + e.part] += t;
            ++h->part_n[k + e.part];
        }
        if (e.n >= 3) {
            h->part_ms[3] += tot;
            ++h->part_n[3];
        }
    }
    h->events_used = 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_timing_detail(neo_hip_upols* h, double* ms, int64_t* launches)
{
    if (!h) return fail(NEO_HIP_EINVAL, "null handle");
    device_guard g(h->device);
    if (int rc = drain_events(h)) return rc;
    h->group_ms.clear();
    for (int k = 0; k < 4; ++k) {
        if (ms) ms[k] = h->part_ms[k];
        if (launches) launches[k] = h->part_n[k];
        h->part_ms[k] = 0.0;
        h->part_n[k] = 0;
    }
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_step_times(neo_hip_upols* h, double* ms, int64_t cap, int64_t* count)
{
    if (!h || (cap > 0 && !ms)) return fail(NEO_HIP_EINVAL, "null handle or buffer");
    device_guard g(h->device);
    if (int rc = drain_events(h)) return rc;
    const int64_t n = int64_t(h->group_ms.size());
    for (int64_t i = 0; i < std::min(n, cap); ++i) ms[i] = h->group_ms[size_t(i)];
    if (count) *count = n;
    h->group_ms.clear();
    for (int k = 0; k < 4; ++k) {
        h->part_ms[k] = 0.0;
        h->part_n[k] = 0;
    }
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_timing(neo_hip_upols* h, double* mac_ms, int64_t* launches)
{
    double ms[4];
    int64_t n[4];
    int rc = neo_hip_upols_timing_detail(h, ms, n);
    if (rc) return rc;
    const int k = n[3] ? 3 : 0;  // streaming-level steps: the whole step; else the MAC kernel
    if (mac_ms) *mac_ms = ms[k];
    if (launches) *launches = n[k];
    return NEO_HIP_OK;
}

}  // extern "C"
