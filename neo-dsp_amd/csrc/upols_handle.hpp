// upols_handle.hpp — the UPOLS convolver handle (neo_hip_upols) and the host helpers
// shared by the translation units that implement it (upols.hip, upols_batch.hip,
// upols_setup.hip).
#pragma once

#include "common.hpp"

#include <cstdint>
#include <deque>
#include <utility>
#include <vector>

namespace neo_hip {
constexpr int kMaxBatch = 32;                          // most blocks one batched MAC pass consumes
constexpr double kFusedMaxBytes = 64.0 * 1024 * 1024;  // filter + FDL bytes below which a step is one launch
constexpr double kCacheBudgetBytes = 216.0 * 1024 * 1024;  // filter bytes read cacheable (256 MiB Infinity Cache)
// the batched passes leave more of the Infinity Cache to the slabs (same-box A/B at C5, 4 runs
// each: 168 MiB 17.8 us/step, 216 MiB 18.3, 126 MiB 18.1)
constexpr double kBatchCacheBudgetBytes = 168.0 * 1024 * 1024;
// streaming levels (upols_levels.hip)
constexpr int kLvA0 = 8;     // partitions the block itself MACs (p < kLvA0)
constexpr int kLvToep = 5;   // Toeplitz level slots: l < 4 window kLvT0 << l; slot 4 the big level
constexpr int kLvT0 = 4;
constexpr int kBigT = 128;   // big Toeplitz level: window, band [2 kBigT, P) instead of the far level (opt-in:
                             // 26.9 vs 19.2 us per C5 step, its 89 M complex MACs per step are VALU / LDS bound)
constexpr int kFarT = 128;   // far level: blocks per window (256-point partition-axis transform)
constexpr int kFarA = 256;   // far level: first partition (2 kFarT)
constexpr int kFarRing = 2 * kFarA;  // far level: FDL ring rows needed (a slice reads back 383 blocks)
// offline windows (k_off_mac): batched calls of >= 128 blocks take windows of kFarT blocks through
// partition-axis transforms of every 128-partition segment, from this many partitions
#ifndef NEO_OFF_MIN_P
#define NEO_OFF_MIN_P 128  // diagnostic builds (A/B)
#endif
constexpr int kOffMinP = NEO_OFF_MIN_P;
constexpr int kOffMaxWP = 2;  // windows per pass

// Latency mode (neo_hip_upols_set_persistent, upols_levels.hip): one persistent kernel per handle
// polls a mailbox in mapped host memory. Step n's record (device addresses of its input and
// output blocks) goes to slot n mod kPsRing; both words carry the slot's lap tag in their low 4
// bits (the blocks are 16-B aligned), so a record read while the host rewrites it shows two
// different tags and is read again.
constexpr int kPsRing = 64;
__host__ __device__ inline uint64_t ps_tag(int64_t n) { return uint64_t((n / kPsRing) % 15 + 1); }
struct persist_rec {
    uint64_t in, out;
};
struct persist_mb {
    persist_rec rec[kPsRing];
    int64_t done;   // kernel -> host: steps completed (n + 1 of the last one)
    int32_t stop;   // host -> kernel: leave
    int32_t alive;  // kernel -> host: 0 once the kernel leaves (stop, idle timeout, error)
    int32_t err;    // kernel -> host: a wait passed its deadline
    int32_t pad;
};

// What both persistent kernels (k_lvl_persist, upols_levels.hip; k_plain_persist, upols.hip) share:
// the mailbox, the device flags (kPsFlag*), the step times, the idle limit and the deadline.
struct persist_ctl {
    persist_mb* mb;                 // the mapped mailbox (device address)
    int64_t* flags;                 // blk_done, quit, arrivals, records, sl_done (kPsFlag*)
    unsigned long long* tl;         // [kPsRing][2] record seen / done
    long long idle_ticks, dead_ticks;
    int64_t n0;                     // first step of this launch
    int w0;                         // its ring row
};
// device flags of the persistent kernels (int64 words): blk_done, quit, the per-step arrival
// counters of the block workgroups (a ring: a channel may run up to three steps ahead of another),
// the last step whose record block workgroup 0 handed on and those records (a ring), then
// sl_done per slice workgroup
constexpr int kPsArr = 8;
constexpr int kPsFlagArrive = 2, kPsFlagArriveFdl = kPsFlagArrive + kPsArr, kPsFlagGo = kPsFlagArriveFdl + kPsArr;
constexpr int kPsFlagIo = kPsFlagGo + 1;
constexpr int kPsFlagSlices = kPsFlagIo + 2 * kPsArr;

__device__ __forceinline__ int64_t ps_ld(const int64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_st(int64_t* p, int64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ps_acquire()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// thread 0: wait until cond() (quit and the deadline checked every round); false = leave
template<class F>
__device__ __forceinline__ bool ps_wait(const persist_ctl& pc, F cond)
{
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        if (cond()) return true;
        if (ps_ld(pc.flags + 1)) return false;
        if ((long long)(wall_clock64() - t0) > pc.dead_ticks) {
            __hip_atomic_store(&pc.mb->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ps_st(pc.flags + 1, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// thread 0 of a block workgroup, ok = its own waits passed: step n's record into io[2]. Workgroup 0
// (lead) polls the mailbox slot (both words tagged with the step's lap; the host's stop, quit and
// the idle limit checked every 16th poll) and, with more than one block workgroup (share), hands
// the record on through the flags; the others wait for it there. false = leave.
__device__ __forceinline__ bool ps_record(const persist_ctl& pc, int64_t n, bool lead, bool share, bool ok,
                                          uint64_t* io, unsigned long long& t_seen)
{
    if (lead) {
        const int slot = int(n % kPsRing);
        const uint64_t tag = ps_tag(n);
        const unsigned long long t0 = wall_clock64();
        for (unsigned it = 0; ok; ++it) {
            const uint64_t r0 = __hip_atomic_load(&pc.mb->rec[slot].in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint64_t r1 = __hip_atomic_load(&pc.mb->rec[slot].out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((r0 & 15) == tag && (r1 & 15) == tag) {
                io[0] = r0 & ~uint64_t(15);
                io[1] = r1 & ~uint64_t(15);
                t_seen = wall_clock64();
                if (share) {
                    int64_t* r = pc.flags + kPsFlagIo + 2 * (n % kPsArr);
                    ps_st(r, int64_t(io[0]));
                    ps_st(r + 1, int64_t(io[1]));
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    ps_st(pc.flags + kPsFlagGo, n);
                }
                return true;
            }
            if ((it & 15) == 15 &&
                (__hip_atomic_load(&pc.mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || ps_ld(pc.flags + 1) ||
                 (long long)(wall_clock64() - t0) > pc.idle_ticks)) {
                ps_st(pc.flags + 1, 1);
                return false;
            }
        }
        return false;
    }
    if (!ok || !ps_wait(pc, [&] { return ps_ld(pc.flags + kPsFlagGo) >= n; })) return false;
    ps_acquire();
    const int64_t* r = pc.flags + kPsFlagIo + 2 * (n % kPsArr);
    io[0] = uint64_t(ps_ld(r));
    io[1] = uint64_t(ps_ld(r + 1));
    return true;
}

struct level_plan {
    int a0 = 1;                      // the block step takes partitions [0, a0)
    int n = 0;                       // Toeplitz levels
    int T[kLvToep] = {}, a[kLvToep] = {}, b[kLvToep] = {};  // window (blocks) and partition band [a, b) per level
    int nseg = 0;                    // far segments of kFarT partitions from kFarA (0: no far level)
};
}  // namespace neo_hip

struct neo_hip_upols {
    int device = 0, C = 0, B = 0, P = 0, S = 1, rows = 1;
    int ring = 0;  // FDL ring rows R = P + kMaxBatch - 1 (at least kFarRing with a far level)
    hipStream_t stream = nullptr;
    neo_hip::cf* H = nullptr;
    neo_hip::cf* fdl = nullptr;
    neo_hip::cf* part = nullptr;
    float* prev = nullptr;
    int* arrivals = nullptr;  // per-channel split arrival counters (zero between steps)
    int wpos = 0;             // FDL write position (fdl_index.hpp:35-37), host-side
    neo_hip::cf* tw = nullptr;
    float* io = nullptr;       // device staging for host-pointer process()
    float* io_host = nullptr;  // pinned staging
    bool batch = true;      // process_blocks runs T blocks per MAC pass (neo_hip_upols_set_batch)
    int Sb = 1, rows_b = 1; // batched-pass splits per channel and partitions per split
    int bT = 32, bNB = 1;   // batched pass: blocks per pass (capped by batch_t), bins per lane-vector
    int pcb = 0;            // filter rows per channel the batched MAC loads cacheable (kBatchCacheBudgetBytes)
    bool bufload = true;    // batched MAC with buffer loads (one channel's rows span < 2 GiB)
    neo_hip::cf* part_b = nullptr;   // batched partial spectra [C][Sb][T][B]
    // streaming levels (upols_levels.hip): on for HBM-bound shapes (neo_hip_upols_set_ahead)
    bool ahead = false;
    neo_hip::level_plan lv;
    int64_t lv_n = -1;              // blocks since the levels were primed (-1: prime at the next step)
    bool fdl_zero = false;          // FDL ring all zero, nothing stepped since (reset_state): every level
                                    // window the prime computes is zero, so priming is zeroing
    bool grouped = false;           // created by a convolver group (create_handle): no eager priming
    bool lv_ready = false;          // level buffers allocated
    neo_hip::cf* lv_slab[neo_hip::kLvToep] = {};  // Toeplitz level slabs [2][C][T][B]
    // step groups (upols_levels.hip part_plan, set when the levels prime): per Toeplitz level the
    // window offset phi (windows start at t0 + W T - phi) and the unit cuts of its background parts
    // per window of a cycle of lv_cyc groups
    int lv_phi[neo_hip::kLvToep] = {};
    int lv_cyc = 1;
    std::vector<int> lv_cut[neo_hip::kLvToep];
    std::vector<int> fv_cut;  // step groups: the far slices' first units (ns + 1 cuts; empty: equal slices)
    neo_hip::cf* fv_hf = nullptr;   // far segment spectra [C][nseg][256][B]
    neo_hip::cf* fv_xf = nullptr;   // far FDL row-pair spectra, ring of nseg slots [C][nseg][256][B]
    neo_hip::cf* fv_ff = nullptr;   // far field [2][C][128][B]
    neo_hip::cf* fv_tw = nullptr;   // 256-point twiddles
    neo_hip::cf* fv_acc = nullptr;  // far phase-1 partial sums [K][units][256][16] (K = far_group)
    bool fv_dirty = true;           // far segment spectra to recompute (filter changed)
    int far_k = 0;                  // far phase-1 windows per pass forced by neo_hip_upols_opts.far_group (0: auto)
    int toep_jh = 0;                // T = 32 window parts forced by neo_hip_upols_opts.toep_split (0: auto)
    int f2mode = 0;                 // far phase 2 at G = 1 forced by neo_hip_upols_opts.far_phase2 (0: auto)
    bool far_raw = false;           // far level recomputed every window from the filter and FDL rows
                                    // (neo_hip_upols_opts.far_level 2; far2r_role): no fv_hf / fv_xf / fv_acc
    // step groups (neo_hip_upols_opts.step_group, G = sg): G = 1 runs a step as ONE launch (the
    // block and 1/T of every level's next window); G > 1 runs the block of every call alone on the
    // caller's stream and the level slices of G steps as one launch on the handle's background
    // stream bg, one step group ahead (events ev_blk / ev_sl order the two; upols_levels.hip)
    int sg = 1;
    int bg_pad = 0;  // dynamic LDS bytes of the slices launches (bg_pad_for): 1024 holds them to 2 workgroups per CU
    hipStream_t bg = nullptr;
    hipEvent_t ev_blk = nullptr, ev_sl[2] = {}, ev_join = nullptr;
    int paced = 0;                 // neo_hip_upols_set_paced: the group's background launch in G per-call pieces
                                   // (1) or in two pieces, at the group's calls 0 and G / 2 (2)
    bool pace_prev = false;        // a piece was issued before (its event ev_pc[(pace_seq - 1) & 1])
    int64_t pace_seq = 0;          // pieces issued since the levels primed
    hipEvent_t ev_pc[2] = {};
    bool bg_busy = false;  // slices enqueued on bg since the last join
    int64_t bg_launches = 0;
    float* tail = nullptr;  // batched OLA tails [C][T][B]
    // offline windows (k_off_mac, launch_offline): batched calls take 128 or 256 blocks per pass
    bool off = false;                // eligible (P >= kOffMinP, whole-block handles) and on (neo_hip_upols_set_offline)
    int off_nseg = 0;                // 128-partition segments from p = 0
    neo_hip::cf* off_hf = nullptr;   // the filter's segment spectra [C][off_nseg][256][B]
    bool off_dirty = true;           // off_hf to recompute (filter changed)
    neo_hip::cf* off_y = nullptr;    // a pass's output spectra [C][128 kOffMaxWP][B]
    float* off_tail = nullptr;       // OLA: a pass's tails [C][128 kOffMaxWP][B]
    float* samples_dev = nullptr;   // process_samples host staging (device side)
    float* samples_host = nullptr;  // process_samples host staging (pinned)
    size_t samples_cap = 0;
    int timing = 0;          // 0: off; n: HIP events around every n-th launch group
    int64_t tick = 0;        // launch groups seen while timing
    bool ola = false;  // upola_convolver (overlap-add stage) instead of upols (overlap-save)
    bool v2 = false;   // upola_convolver_v2: sub-block input (implies ola)
    int in_pos = 0;    // v2: samples of the current block already consumed (_input_pos)
    float* window = nullptr;  // v2: real window [C][2B]
    neo_hip::cf* tmp = nullptr;        // v2: tail accumulator [C][B] packed (_tmp_accumulator)
    // one launch per block (last-arriver tail) instead of MAC + finish: on for small filter
    // + FDL working sets, where the step is launch-bound (C3: 10.6 vs 12.4 us per block),
    // off for HBM-bound ones (C5: 0.342 vs 0.303 ms); NEO_HIP_FUSED=0/1 overrides
    bool fused = false;
    // H / FDL layout: row p of channel c at c * cstride + p * pstride (complex units).
    // Default [C][P][B]; NEO_HIP_LAYOUT=pcb selects partition-major [P][C][B] (A/B).
    int64_t cstride = 0, pstride = 0;
    int pc = 0;  // filter rows per channel read with the cacheable policy (kCacheBudgetBytes; NEO_HIP_CACHE_ROWS)
    struct ev_group {
        hipEvent_t e[4] = {};
        int n = 0;
        int part = 0;  // first part index its intervals add to (1: a step group's slice launch on bg)
    };
    std::deque<ev_group> events;   // pool, reused across timing windows (stable addresses while growing)
    size_t events_used = 0;
    double part_ms[4] = {};        // drained event time per part (see neo_hip_upols_timing_detail)
    int64_t part_n[4] = {};
    std::vector<float> group_ms;   // whole-group durations, in order (neo_hip_upols_step_times)
    // latency mode (neo_hip_upols_set_persistent): a persistent step kernel on ps_stream
    bool persist = false;          // requested
    bool ps_running = false;       // a persistent kernel was launched and not yet joined
    bool ps_valid = false;         // the level slabs follow the persistent schedule (relaunch without priming)
    hipStream_t ps_stream = nullptr;
    neo_hip::persist_mb* ps_mb = nullptr;      // mapped pinned mailbox (host address)
    neo_hip::persist_mb* ps_mb_dev = nullptr;  // its device address
    int64_t* ps_flags = nullptr;               // device: blk_done, quit, arrive, sl_done[]
    unsigned long long* ps_tl = nullptr;       // device: per ring slot {record seen, done} (wall clock, 100 MHz)
    int ps_nslices = 0;                        // slice workgroups of the persistent kernel
    int64_t ps_ld_in = 0, ps_ld_out = 0;       // channel strides of the running kernel
    int64_t ps_n0 = 0;                         // first step of the running kernel
    int64_t ps_launches = 0;                   // persistent launches so far (idle timeouts relaunch)
    int ps_wgs = 0;                            // workgroups of the running kernel (resident_admit)
    int64_t ps_fallbacks = 0;                  // calls run as normal steps: no room for the grid
    double ps_idle_ms = 50.0;                  // the kernel leaves after this long without a block
    // streams the step calls ran on since the last setup call (setup_join waits for these, not for
    // the device: another handle's resident latency-mode kernel must not stall a setup call); a
    // stream given to a step call must stay valid until the handle's next setup call or destroy
    neo_hip::stream_set used;
};


namespace neo_hip {

using upols_t = neo_hip_upols;

inline int note_stream(upols_t* h, hipStream_t s) { return h->used.note(s); }
// order a setup call (filter change, reset, mode switch, destroy) after every step of this handle:
// the streams its step calls ran on, its background stream, its own stream; device_input: also
// after work on the null stream (a device-resident filter or impulse produced there)
int setup_join(upols_t* h, bool device_input = false);

inline bool valid_block(int b) { return b >= 16 && b <= 4096 && (b & (b - 1)) == 0; }

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

inline int64_t partitions_for(int64_t L, int B)
{
    // stft.hpp:21-25 with overlap 0: idiv(L - B, B) + 1 (= ceil(L/B) for L >= B);
    // the reference underflows for L < B, we clamp to one partition.
    if (L <= B) return 1;
    return (L - B + B - 1) / B + 1;
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

inline int batch_blocks(const upols_t* h) { return batch_t(h->B, h->bNB, h->bT); }

// a handle with default options whose setup and host-I/O work runs on `stream` (a group's; not
// destroyed with the handle) instead of one of the device's shared streams (upols.hip)
int create_handle(int channels, int block, int partitions, int device, int method, hipStream_t stream,
                  neo_hip_upols** out);
// upols_batch.hip: T whole blocks in one pass over the filter and the FDL
int launch_batch(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int T, hipStream_t s);
// Timing (neo_hip_upols_set_timing): the next event group of nev events if this launch
// group is a timed one (every h->timing-th), else nullptr; mark(g, i, s) records event i.
inline int timing_begin(upols_t* h, int nev, upols_t::ev_group** out)
{
    *out = nullptr;
    if (!h->timing || h->tick++ % h->timing != 0) return NEO_HIP_OK;
    if (h->events_used == h->events.size()) {
        upols_t::ev_group g;
        for (auto& e : g.e) NEO_HIP_CHECK(hipEventCreate(&e));
        h->events.push_back(g);
    }
    *out = &h->events[h->events_used++];
    (*out)->n = nev;
    (*out)->part = 0;
    return NEO_HIP_OK;
}
inline int timing_mark(upols_t::ev_group* g, int i, hipStream_t s)
{
    if (g) NEO_HIP_CHECK(hipEventRecord(g->e[i], s));
    return NEO_HIP_OK;
}

// upols_levels.hip: one streaming block step (level slabs + the newest partitions) and 1/T
// of every level's next window; the level plan; buffers; filter-change hook
// (snap: also copy each channel's input block, as read, to snap [C][B])
int launch_levels(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s,
                  float* snap = nullptr);
// far: -1 auto (= 1), 0 the big Toeplitz level, 1 the far level
void plan_levels(int P, level_plan& lp, int far = -1);
// the block role of streaming step n (FDL ring row w) again for channel c alone, with another
// input block (upols_group.hip: a speculatively stepped channel whose caller's block differed);
// the step's slabs and far field must not have been overwritten since
int launch_block_only(upols_t* h, int64_t n, int w, int c, const float* in, float* out, hipStream_t s);
// the automatic far phase-1 window group / T = 32 window parts a handle of C channels would use
int far_group_for(int C, int B, int P);
int toep_split_for(int C, int B);
int step_group_for(int C, int B, int P);
int bg_pad_for(int C, int B);
// latency mode: whole blocks through the persistent kernel, synchronous (upols_levels.hip)
int persist_process(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int64_t nblocks);
// latency mode of a handle without streaming levels: the plain step's persistent kernel on
// h->ps_stream (upols.hip), its control (mailbox, flags, first step) set up by the caller
// (no room for its grid beside the process's other persistent kernels: *launched false, nothing
// enqueued, persist_room)
int plain_persist_launch(upols_t* h, const persist_ctl& ctl, int64_t ld_in, int64_t ld_out, bool* launched);
// room on the device for a persistent grid of `grid` workgroups of kernel f (256 lanes): all of them
// resident at once beside the persistent kernels this process already runs there, within three
// quarters of the device's slots for f (occupancy x CUs); reserved in h->ps_wgs on success
bool persist_room(upols_t* h, const void* f, int grid);
// the normal (non-persistent) block step (launch_step without the latency-mode branch)
int launch_step_normal(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s);
// stop the persistent kernel (if any) and leave the levels to re-prime on the next normal step
int persist_stop(upols_t* h);
// why a handle cannot run the latency mode (nullptr: it can)
const char* persist_ineligible(const upols_t* h);
// order everything enqueued on the background stream (step-group slices) before later work on s;
// every path that writes the FDL ring or the level buffers other than a streaming step calls it
int lvl_join(upols_t* h, hipStream_t s);
void lvl_free(upols_t* h);
void lvl_filter_changed(upols_t* h);
// offline windows: the segment spectra (if the filter changed) and k_off_mac for wp windows of
// 128 blocks at h->wpos into h->off_y (buffers allocated by the caller, launch_offline)
int launch_off_mac(upols_t* h, int wp, hipStream_t s);
size_t off_hf_bytes(const upols_t* h);  // the offline windows' segment spectra (padded channel stride)
// upols_batch.hip: wp windows of 128 blocks of every channel in one pass (window r2c of every
// block, k_off_mac, per-block finish), h->wpos advanced
int launch_offline(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int wp, hipStream_t s);
// a setup call's last step (set_filter, set_impulse, reset; FDL just zeroed): the level buffers,
// the far segment spectra and window 0 of every level, on h->stream, so the next call is an
// ordinary streaming step (no-op without levels and for group handles)
int lvl_setup_prime(upols_t* h);
// upols_setup.hip: twiddles, uniform_partition and normalize_impulse on the device
int upload_tw(cf** d, int B);
int partition_device(const float* d_ir, int C, int64_t L, int B, bool packed, cf* out, const cf* tw, hipStream_t s,
                     int64_t cstride = 0, int64_t pstride = 0);
int normalize_device(float* d_ir, int C, int64_t L, hipStream_t s);
// filter [C][P][B+1] (reference layout, device) -> packed H rows of the handle
int pack_filter(upols_t* h, const cf* src, hipStream_t s);

}  // namespace neo_hip
