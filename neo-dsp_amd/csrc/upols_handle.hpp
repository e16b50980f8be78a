// upols_handle.hpp — the UPOLS convolver handle (neo_hip_upols) and the host helpers
// shared by the translation units that implement it (upols.hip, upols_batch.hip,
// upols_setup.hip).
#pragma once

#include "common.hpp"

#include <cstdint>
#include <utility>
#include <vector>

namespace neo_hip {
constexpr int kMaxBatch = 32;                          // most blocks one batched MAC pass consumes
constexpr int kFarT = 128;                             // two-level lookahead: blocks per far-field window
constexpr int kFarAutoP = 512;                         // partitions from which it is on by default
constexpr double kFusedMaxBytes = 64.0 * 1024 * 1024;  // filter + FDL bytes below which a step is one launch
constexpr double kCacheBudgetBytes = 216.0 * 1024 * 1024;  // filter bytes read cacheable (256 MiB Infinity Cache)
// the lookahead / batched passes leave more of the Infinity Cache to the block steps' rows and
// slabs (same-box A/B at C5, 4 runs each: 168 MiB 17.8 us/step, 216 MiB 18.3, 126 MiB 18.1)
constexpr double kBatchCacheBudgetBytes = 168.0 * 1024 * 1024;
}  // namespace neo_hip

struct neo_hip_upols {
    int device = 0, C = 0, B = 0, P = 0, S = 1, rows = 1;
    int ring = 0;  // FDL ring rows R = P + kMaxBatch - 1
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
    int pcb = 0;            // filter rows per channel the batched MAC loads cacheable (kBatchCacheBudgetBytes; NEO_HIP_BATCH_CACHE_ROWS)
    int bprio = 11;         // batched MAC: co-resident workgroups trade issue priority every 2^bprio
                            // 10-ns ticks (NEO_HIP_BATCH_PRIO=0 off)
    bool snt = false;       // lookahead passes store their slabs nontemporally (NEO_HIP_SLAB_NT)
    int b8var = 3;          // 8-block passes: bmac_var 3 (buffer loads, D = 8) or 0 (NEO_HIP_BATCH8_VAR)
    int bvar = 3;           // batched MAC variant at T = 32, B = 256/512 (bmac_var in upols_batch.hip; NEO_HIP_BATCH_VAR)
    neo_hip::cf* part_b = nullptr;   // batched partial spectra [C][Sb][T][B]
    // streaming lookahead (k_upols_ahead): one batched pass per T blocks, phase = block of
    // the current window; on for HBM-bound shapes (not fused), NEO_HIP_AHEAD / set_ahead
    bool ahead = false;
    bool asub = true;     // lookahead sub-windows (k_upols_ahead2 only; NEO_HIP_AHEAD_SUB=0 disables)
    bool ssplit = false;  // sub-window passes: one split per chunk (NEO_HIP_SUB_SPLIT=1; A/B on one box: slower)
    int subw = 8;         // lookahead sub-window (blocks): 16 at B >= 512 (rocprof totals: C5 -1.7 %), 8 below
                          // (C4 +1 % with 16); NEO_HIP_SUBWINDOW=8/16
    neo_hip::cf* part_s = nullptr;  // sub-window pass slabs [C][ssub][subw][B], ssub * subw <= kMaxBatch
    // direct-head block step k_upols_ahead3 (OLS): 1 = at B = 256 (same-box A/B: C4 +3.5 %; at
    // B = 512 the 512 x 512-tap convolution costs what it saves), 2 = at B = 256 and 512,
    // 0 = off (NEO_HIP_AHEAD_DIRECT=1 / 0)
    int adirect = 1;
    bool direct_ok = false; // partition 0's time-domain head is B taps (update_head)
    float* h0t = nullptr;   // head taps [C][B] (k_head_taps)
    float* h0tail = nullptr;
    int akern = 2;  // per-block lookahead kernel: 2 = k_upols_ahead2 (B <= 1024), 1 = k_upols_ahead (NEO_HIP_AHEAD_KERNEL)
    int phase = 0;
    // two-level lookahead (upols_far.hip, NEO_HIP_FAR=1): partitions >= kFarT by a partition-axis
    // transform once per kFarT blocks; the level-1 pass then walks partitions < kFarT only
    bool far = false;
    int fwin = -1;                 // level-1 windows done in the current far window (-1: recompute)
    int fbase = 0;                 // first block of the current level-1 window within the far window
    neo_hip::cf* hf = nullptr;     // segment spectra [C][Q-1][2 kFarT][B]
    neo_hip::cf* hf0 = nullptr;    // bin 0's second coefficient [C][Q-1][2 kFarT]
    neo_hip::cf* ff = nullptr;     // far field of the current window [C][kFarT][B]
    neo_hip::cf* twf = nullptr;    // 2 kFarT-point twiddles
    float* tail = nullptr;  // batched OLA tails [C][T][B]
    float* samples_dev = nullptr;   // process_samples host staging (device side)
    float* samples_host = nullptr;  // process_samples host staging (pinned)
    size_t samples_cap = 0;
    int timing = 0;          // 0: off; n: HIP events around every n-th MAC launch
    int64_t tick = 0;        // MAC launches seen while timing
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
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // pool, reused across timing windows
    size_t events_used = 0;
    double mac_ms = 0.0;
    int64_t launches = 0;
};


namespace neo_hip {

using upols_t = neo_hip_upols;

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

// upols_batch.hip: T whole blocks in one pass over the filter and the FDL
int launch_batch(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, int T, hipStream_t s);
// upols_batch.hip: one streaming block step in lookahead mode
int launch_ahead(upols_t* h, const float* in, int64_t ld_in, float* out, int64_t ld_out, hipStream_t s);
// upols_far.hip: two-level lookahead (segment spectra after every filter change; one far
// window per kFarT blocks)
bool far_usable(const upols_t* h);
int far_filter(upols_t* h, hipStream_t s);
int far_window(upols_t* h, hipStream_t s);
// upols_setup.hip: twiddles, uniform_partition and normalize_impulse on the device
int upload_tw(cf** d, int B);
int partition_device(const float* d_ir, int C, int64_t L, int B, bool packed, cf* out, const cf* tw, hipStream_t s,
                     int64_t cstride = 0, int64_t pstride = 0);
int normalize_device(float* d_ir, int C, int64_t L, hipStream_t s);
// filter [C][P][B+1] (reference layout, device) -> packed H rows of the handle
int pack_filter(upols_t* h, const cf* src, hipStream_t s);
// time-domain head taps of partition 0 for the direct-head block step (after every filter change)
int update_head(upols_t* h, hipStream_t s);

}  // namespace neo_hip
