// upols_group.hip — many single-channel upols_convolver instances stepped as ONE multichannel
// launch per frame, with each instance's own semantics kept exactly.
//
// The reference's plugin holds std::vector<upols_convolver> and calls them one after the other
// on the channels of a frame, each call in place and complete on return
// (extra/plugin/src/dsp/DenseConvolution.hpp:35, DenseConvolution.cpp:62-74). Each of those
// calls as a GPU round trip of its own costs a launch and a wait per channel. A group holds the
// instances of one shape (block, partitions, method, device):
//   independent mode  every member has its own one-channel handle; calls run immediately. The
//                     group watches the calls: once two consecutive frames (every live member
//                     called exactly once, all with the same block count, each on the buffer it
//                     used in the frame before, the buffers distinct) went by, the members'
//                     states move into ONE shared handle (coalesced mode).
//   coalesced mode    the first call of a frame (the leader) steps ALL members in one launch: its
//                     own block, and for every other member the contents of the buffer it passed
//                     in the previous frame (speculation: the plugin's AudioBlock channels are
//                     filled before the loop over the convolvers). The leader reads ONLY buffers
//                     the group's owner registered (neo_hip_upols_group_register: the owner
//                     promises they stay allocated until it unregisters them), never a caller
//                     pointer it was merely handed once: a member whose buffer is not (or no
//                     longer) registered keeps the group in independent mode. A later member's call compares
//                     its block with the block speculated for it: equal -> its output is already
//                     computed; different -> its channel's block step runs again with the real
//                     block (previous block restored: the step's other roles never read the
//                     current block's FDL row, so the redo reproduces the one-channel step bit
//                     for bit). A member called twice before the others (or joining, leaving,
//                     changing its filter) ends coalescing: the states move back into one-channel
//                     handles (a speculatively stepped member one block back) before the call.
// So every output is the instance's own sequential step; the launch count per frame drops from
// one per channel to one while the caller keeps the plugin's call pattern. Each handle takes the
// code-path choices of its own shape (a member alone: one channel, one launch per block; the
// shared handle: its channel count's step groups, far window group, Toeplitz window parts), and a
// mode switch re-primes the streaming levels at that block: outputs equal a standalone
// single-channel convolver's up to float summation order (tests: bit for bit where the levels
// whose order depends on the shape do not contribute yet, against the oracle over long runs).
#include "upols_handle.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#ifdef NEO_GROUP_PROBE  // diagnostic builds (tools/build_variant.sh): where a coalesced frame's time goes
#include <chrono>
#include <cstdio>
namespace {
struct group_probe {
    // leader: copy in, prev backup, launch, wait, copy out; member: compare, copy out, redo;
    // whole call (coalesced); per-sample medians
    static constexpr int K = 13;
    std::vector<double> v[K];
    ~group_probe()
    {
        const char* names[K] = {"lead_copy_in", "lead_prev_backup", "lead_launch", "lead_wait", "lead_copy_out",
                                "member_cmp", "member_copy", "member_redo", "call_total", "split_members",
                                "split_sync", "split_free_shared", "coalesce_total"};
        std::fprintf(stderr, "{\"group_probe_us\": {");
        for (int k = 0; k < K; ++k) {
            auto& x = v[k];
            std::sort(x.begin(), x.end());
            const double med = x.empty() ? 0.0 : x[x.size() / 2], p90 = x.empty() ? 0.0 : x[x.size() * 9 / 10];
            std::fprintf(stderr, "%s\"%s\": [%.3f, %.3f, %zu]", k ? ", " : "", names[k], med, p90, x.size());
        }
        std::fprintf(stderr, "}}\n");
    }
} g_probe;
inline double probe_now() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace
#define NEO_GP_T(v) const double v = probe_now()
#define NEO_GP_ADD(k, t0) g_probe.v[k].push_back(probe_now() - (t0))
#else
#define NEO_GP_T(v)
#define NEO_GP_ADD(k, t0)
#endif

namespace {
using neo_hip::cf;
using neo_hip::fail;

struct member {
    bool live = false;
    neo_hip_upols* own = nullptr;  // independent mode: the member's one-channel handle
    bool filtered = false;
    int64_t steps = 0;             // blocks processed since the filter was set
    const float* io_last = nullptr;
    const float* io_prev = nullptr;  // the buffer of the frame before (coalescing needs stable buffers)
    bool pending = false;          // coalesced: stepped by the frame's leader, call not yet seen
    bool seen = false;             // independent: called in the frame being observed
    int slot = -1;                 // coalesced: channel in the shared handle
};
}  // namespace

struct neo_hip_upols_group {
    int device = 0, B = 0, P = 0, method = 0;
    std::mutex mu;
    std::vector<member> m;
    bool coalesced = false;
    neo_hip_upols* shared = nullptr;
    std::vector<int> slot_member;     // shared handle channel -> member
    struct range {
        uintptr_t lo, hi;  // owner-registered host range [lo, hi) the leader may read (page-locked: pin_range)
        int flags;         // NEO_HIP_GROUP_FRAME_STABLE: not written during a frame but by the members' own calls;
                           // NEO_HIP_GROUP_FRAME_INPLACE: also read by the owner only through them, each member on
                           // the same block every frame (the step writes every output in place)
    };
    bool trust = false;        // this frame was read in place from a stable range: members commit without comparing
    bool out_inplace = false;  // and its outputs were written in place (FRAME_INPLACE): members have nothing to copy
    std::vector<range> reg;
    float* in_pin = nullptr;          // mapped pinned [C][B]: the frame's input blocks
    float* out_pin = nullptr;         // mapped pinned [C][B]: the frame's output blocks
    float* in_dev = nullptr;          // their device addresses
    float* out_dev = nullptr;
    float* prev_bak = nullptr;        // device [C][B]: the previous blocks before the frame's step
    float* stage_pin = nullptr;       // independent mode: one member's block, mapped pinned
    float* stage_dev = nullptr;
    int64_t step_n = 0;               // the frame step's level index and FDL ring row (for redos)
    int step_w = 0;
    int npending = 0;
    int nseen = 0, good_frames = 0;
    int64_t stat_steps = 0, stat_calls = 0, stat_redos = 0, stat_switches = 0;
    hipStream_t stream = nullptr;
};

namespace {
using group_t = neo_hip_upols_group;

int live_count(const group_t* g)
{
    int n = 0;
    for (const auto& x : g->m) n += x.live;
    return n;
}

// one channel's state (filter rows, FDL ring, previous block) from (src, cs) to (dst, cd); both
// handles have the same block, partitions and ring
int copy_channel(neo_hip_upols* dst, int cd, const neo_hip_upols* src, int cs, const float* prev_src, hipStream_t s)
{
    const size_t rows = size_t(src->ring) * size_t(src->B) * sizeof(cf);
    NEO_HIP_CHECK(hipMemcpyAsync(dst->H + int64_t(cd) * dst->cstride, src->H + int64_t(cs) * src->cstride,
                                 size_t(src->P) * size_t(src->B) * sizeof(cf), hipMemcpyDeviceToDevice, s));
    NEO_HIP_CHECK(hipMemcpyAsync(dst->fdl + int64_t(cd) * dst->cstride, src->fdl + int64_t(cs) * src->cstride, rows,
                                 hipMemcpyDeviceToDevice, s));
    NEO_HIP_CHECK(hipMemcpyAsync(dst->prev + int64_t(cd) * dst->B, prev_src + int64_t(cs) * src->B,
                                 size_t(src->B) * sizeof(float), hipMemcpyDeviceToDevice, s));
    dst->fdl_zero = false;  // a stepped ring: the next streaming step primes in full
    return NEO_HIP_OK;
}

void free_shared(group_t* g)
{
    if (g->shared) neo_hip_upols_destroy(g->shared);
    g->shared = nullptr;
    neo_hip::hfree(g->in_pin);
    neo_hip::hfree(g->out_pin);
    neo_hip::dfree(g->prev_bak);
    g->in_pin = g->out_pin = g->in_dev = g->out_dev = g->prev_bak = nullptr;
    g->slot_member.clear();
}

int make_own(group_t* g, member& x)
{
    if (x.own) return NEO_HIP_OK;
    return neo_hip::create_handle(1, g->B, g->P, g->device, g->method, g->stream, &x.own);  // on the group's stream
}

// the B samples at p lie in a range the owner registered
bool registered(const group_t* g, const float* p)
{
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + size_t(g->B) * sizeof(float);
    for (const auto& r : g->reg)
        if (lo >= r.lo && hi <= r.hi) return true;
    return false;
}

// Page-locked, device-mapped registered ranges, process-wide and counted (an owner registers its
// frame buffer with the group of every shape it holds): the coalesced step reads the members'
// blocks in place instead of the leader copying them (DenseConvolution.cpp:62-74: the frame's
// channels are filled before the loop over the convolvers). hipHostRegister page-locks 4 MB in
// ~33 us (tests/cpp/bench_hipcost), once per registration.
struct pin_entry {
    int refs;
    bool ours;      // registered by us (else it was page-locked already: its owner unregisters it)
    bool borrowed;  // not ours and overlapping a range locked here: that range's last unregister
                    // (another group, another thread) may unlock it while a step reads it in place
};
std::mutex g_pin_mu;
std::map<std::pair<uintptr_t, uintptr_t>, pin_entry> g_pins;  // [lo, hi) -> entry

void pin_range(uintptr_t lo, uintptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_pin_mu);
    if (auto it = g_pins.find({lo, hi}); it != g_pins.end()) {
        ++it->second.refs;
        return;
    }
    pin_entry e{1, false, false};
    void* p = reinterpret_cast<void*>(lo);
    if (hipHostRegister(p, size_t(hi - lo), hipHostRegisterMapped) == hipSuccess) {
        e.ours = true;
    } else {
        (void)hipGetLastError();  // already page-locked (by its owner, or overlapping a range locked here)
        for (const auto& [k, v] : g_pins)
            if (v.ours && k.first < hi && lo < k.second) e.borrowed = true;
    }
    g_pins.emplace(std::make_pair(lo, hi), e);
}

// a registered range whose page lock lasts while its registration does (ours, or its owner's own
// page-locked memory), so a step may read it in place
bool pin_stable(uintptr_t lo, uintptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.find({lo, hi});
    return it != g_pins.end() && !it->second.borrowed;
}

void unpin_range(uintptr_t lo, uintptr_t hi)
{
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.find({lo, hi});
    if (it == g_pins.end() || --it->second.refs > 0) return;
    if (it->second.ours) {
        if (hipHostUnregister(reinterpret_cast<void*>(lo)) != hipSuccess) (void)hipGetLastError();
    }
    g_pins.erase(it);
}

// The leader's frame read in place: every live member's block (the leader's own io, the others'
// buffers of the last frame) at p0 + slot * ld in ONE registered, device-mapped range, 16-byte
// aligned. Then *in_dev / *ld describe it for the step kernel; false: the leader copies.
bool inplace_frame(const group_t* g, const member& lead, const float* io, const float** in_dev, int64_t* ld,
                   int* flags)
{
    *flags = 0;
    const int C = int(g->slot_member.size());
    auto ptr = [&](int slot) {
        const member& y = g->m[size_t(g->slot_member[size_t(slot)])];
        return &y == &lead ? io : y.io_last;
    };
    const float* p0 = ptr(0);
    const int64_t d = C > 1 ? ptr(1) - p0 : g->B;
    if (d < g->B || (d & 3) || (reinterpret_cast<uintptr_t>(p0) & 15)) return false;
    for (int s = 2; s < C; ++s)
        if (ptr(s) != p0 + int64_t(s) * d) return false;
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p0),
                    hi = reinterpret_cast<uintptr_t>(p0 + int64_t(C - 1) * d + g->B);
    for (const auto& r : g->reg)
        if (lo >= r.lo && hi <= r.hi && pin_stable(r.lo, r.hi)) {
            // its device mapping as of now (a range another registration page-locked may have been
            // unlocked since); none: the leader copies
            const float* dev = neo_hip::host_mapped(const_cast<float*>(p0));
            if (!dev) return false;
            *in_dev = dev;
            *ld = d;
            *flags = r.flags;
            return true;
        }
    return false;
}

// independent -> coalesced: every live member's state into one shared handle
int coalesce(group_t* g)
{
    NEO_GP_T(tc0);
    const int C = live_count(g);
    int rc = neo_hip::create_handle(C, g->B, g->P, g->device, g->method, g->stream, &g->shared);
    if (rc) return rc;
    const size_t io = size_t(C) * size_t(g->B) * sizeof(float);
    if ((rc = neo_hip::halloc(reinterpret_cast<void**>(&g->in_pin), reinterpret_cast<void**>(&g->in_dev), io)) ||
        (rc = neo_hip::halloc(reinterpret_cast<void**>(&g->out_pin), reinterpret_cast<void**>(&g->out_dev), io)) ||
        (rc = neo_hip::dalloc(&g->prev_bak, io)))
        return rc;
    neo_hip_upols* sh = g->shared;
    int c = 0, wpos = -1;
    for (int i = 0; i < int(g->m.size()); ++i) {
        member& x = g->m[size_t(i)];
        if (!x.live) continue;
        if ((rc = copy_channel(sh, c, x.own, 0, x.own->prev, g->stream))) return rc;
        if (wpos >= 0 && wpos != x.own->wpos) return fail(NEO_HIP_ERUNTIME, "group members out of step");
        wpos = x.own->wpos;
        x.slot = c++;
        x.pending = false;
        g->slot_member.push_back(i);
    }
    NEO_HIP_CHECK(hipStreamSynchronize(g->stream));
    sh->wpos = wpos;
    neo_hip::lvl_filter_changed(sh);  // far segment spectra of the copied filters; the levels re-prime
    sh->batch = false;
    for (auto& x : g->m)
        if (x.live) {
            neo_hip_upols_destroy(x.own);
            x.own = nullptr;
        }
    g->coalesced = true;
    g->npending = 0;
    ++g->stat_switches;
    NEO_GP_ADD(12, tc0);
    return NEO_HIP_OK;
}

// coalesced -> independent: every live member's state into a one-channel handle of its own; a
// member the frame's leader stepped ahead of its call goes back to before that step (previous
// block from the backup, ring row of the step: its own call writes that row again)
int split(group_t* g)
{
    neo_hip_upols* sh = g->shared;
    NEO_GP_T(ts0);
    for (auto& x : g->m) {
        if (!x.live) continue;
        int rc = make_own(g, x);
        if (rc) return rc;
        const bool back = x.pending;
        if (x.slot >= 0) {
            if ((rc = copy_channel(x.own, 0, sh, x.slot, back ? g->prev_bak : sh->prev, g->stream))) return rc;
            x.own->wpos = back ? g->step_w : sh->wpos;
            if (back) --x.steps;
        }
        neo_hip::lvl_filter_changed(x.own);
        x.own->batch = false;
        x.pending = false;
        x.slot = -1;
        x.seen = false;
    }
    NEO_GP_ADD(9, ts0);
    NEO_GP_T(ts1);
    NEO_HIP_CHECK(hipStreamSynchronize(g->stream));
    NEO_GP_ADD(10, ts1);
    NEO_GP_T(ts2);
    free_shared(g);
    NEO_GP_ADD(11, ts2);
    g->coalesced = false;
    g->npending = 0;
    g->nseen = 0;
    g->good_frames = 0;
    ++g->stat_switches;
    return NEO_HIP_OK;
}

// independent mode: one call, then the frame bookkeeping that decides on coalescing
int call_independent(group_t* g, int i, float* io)
{
    member& x = g->m[size_t(i)];
    if (x.seen) {  // called again before the frame completed: not the lock-step pattern
        for (auto& y : g->m) y.seen = false;
        g->nseen = 0;
        g->good_frames = 0;
    }
    // the block through the group's own mapped staging, on the group's stream: no per-call
    // pointer query of the caller's buffer, no per-member stream or staging
    if (!g->stage_pin) {
        if (int rc = neo_hip::halloc(reinterpret_cast<void**>(&g->stage_pin), reinterpret_cast<void**>(&g->stage_dev),
                                     size_t(g->B) * sizeof(float)))
            return rc;
    }
    const size_t bb = size_t(g->B) * sizeof(float);
    std::memcpy(g->stage_pin, io, bb);
    int rc = neo_hip_upols_process_device(x.own, g->stage_dev, g->B, g->stage_dev, g->B, g->stream);
    if (!rc) rc = neo_hip::spin_sync(g->stream);
    if (!rc) std::memcpy(io, g->stage_pin, bb);
    if (rc) return rc;
    ++x.steps;
    x.io_prev = x.io_last;
    x.io_last = io;
    x.seen = true;
    if (++g->nseen < live_count(g)) return NEO_HIP_OK;
    // a complete frame: equal block counts, distinct buffers, each the member's buffer of the
    // frame before (the leader of a coalesced frame reads them)
    bool ok = live_count(g) >= 2 && x.own->ahead;
    std::vector<const float*> ptrs;
    for (auto& y : g->m) {
        if (!y.live) continue;
        ok = ok && y.filtered && y.steps == x.steps && y.io_last && y.io_last == y.io_prev && registered(g, y.io_last);
        ptrs.push_back(y.io_last);
        y.seen = false;
    }
    std::sort(ptrs.begin(), ptrs.end());
    for (size_t k = 1; k < ptrs.size() && ok; ++k) ok = ptrs[k] != ptrs[k - 1];
    g->nseen = 0;
    g->good_frames = ok ? g->good_frames + 1 : 0;
    if (g->good_frames >= 2 && coalesce(g) != NEO_HIP_OK) {  // not fatal: the members keep their own handles
        free_shared(g);
        for (auto& y : g->m) y.slot = -1;
        g->good_frames = 0;
    }
    return NEO_HIP_OK;
}

// the output block of shared-handle channel `slot` into the CPU caches ahead of its member's call
// (the plugin calls the members in order): the GPU wrote it to host memory over PCIe, so the
// member's copy would otherwise stall on DRAM (0.3 us per 2 KB block on MI355X boxes)
inline void prefetch_output(const group_t* g, int slot)
{
    if (slot >= int(g->slot_member.size())) return;
    const char* p = reinterpret_cast<const char*>(g->out_pin + int64_t(slot) * g->B);
    for (size_t k = 0; k < size_t(g->B) * sizeof(float); k += 64) __builtin_prefetch(p + k, 0, 3);
}

// the block a later member's commit writes (its buffer of the last frame): in this core's cache,
// writable, ahead of the copy. A frame read in place by the step without the leader's snapshot
// (FRAME_STABLE) leaves those lines cold: the GPU's reads over PCIe took them out of the caches
// (the probe build's member copy 0.13 -> 0.03 us at 2048 channels, frame p50 355-363 vs 345-468 us
// over three same-box runs; 2 and 8 members ahead no better: profiles/r6_ab_group_prefetch.json)
#ifndef NEO_GROUP_PFW
#define NEO_GROUP_PFW 4
#endif
inline void prefetch_block(const group_t* g, int slot)
{
    if (slot >= int(g->slot_member.size())) return;
    const char* q = reinterpret_cast<const char*>(g->m[size_t(g->slot_member[size_t(slot)])].io_last);
    if (q)
        for (size_t k = 0; k < size_t(g->B) * sizeof(float); k += 64) __builtin_prefetch(q + k, 1, 3);
}

// coalesced mode: the leader's step over every member, or a later member's commit / redo
int call_coalesced(group_t* g, int i, float* io)
{
    member& x = g->m[size_t(i)];
    neo_hip_upols* sh = g->shared;
    const size_t bb = size_t(g->B) * sizeof(float);
    if (x.pending && g->out_inplace && io == x.io_last) {  // the step wrote this member's output in place
        x.pending = false;
        --g->npending;
        return NEO_HIP_OK;
    }
    if (x.pending) {
        float* spec_in = g->in_pin + int64_t(x.slot) * g->B;
        float* out = g->out_pin + int64_t(x.slot) * g->B;
        NEO_GP_T(tc);
        // a stable frame (the owner's promise, neo_hip_upols_group_register_ex): on the buffer the
        // leader's step read in place, the block is the one it read (no snapshot to compare with);
        // on another buffer its block was never read: this channel's step again (FRAME_INPLACE: the
        // output went to the old buffer -- the owner broke the promise; this call is still exact)
        const bool differs =
            g->out_inplace || (g->trust ? io != x.io_last : std::memcmp(io, spec_in, bb) != 0);
        NEO_GP_ADD(5, tc);
        if (differs) {  // the caller's block differs: this channel's step again
            neo_hip::device_guard dg(g->device);  // the commit path alone makes no HIP call
            if (dg.rc) return dg.rc;
            std::memcpy(spec_in, io, bb);
            NEO_HIP_CHECK(hipMemcpyAsync(sh->prev + int64_t(x.slot) * g->B, g->prev_bak + int64_t(x.slot) * g->B, bb,
                                         hipMemcpyDeviceToDevice, g->stream));
            int rc = neo_hip::launch_block_only(sh, g->step_n, g->step_w, x.slot, g->in_dev + int64_t(x.slot) * g->B,
                                                g->out_dev + int64_t(x.slot) * g->B, g->stream);
            if (rc || (rc = neo_hip::spin_sync(g->stream))) return rc;
            ++g->stat_redos;
            NEO_GP_ADD(7, tc);
        }
        NEO_GP_T(tm);
        std::memcpy(io, out, bb);
        NEO_GP_ADD(6, tm);
        prefetch_output(g, x.slot + 2);
        if (g->trust) prefetch_block(g, x.slot + NEO_GROUP_PFW);
        x.pending = false;
        x.io_last = io;
        --g->npending;
        return NEO_HIP_OK;
    }
    if (g->npending > 0) {  // called again before the others took their blocks: back to one handle each
        int rc = split(g);
        if (rc) return rc;
        return call_independent(g, i, io);
    }
    // the frame's leader: every member's block (its own, the others' buffers of the last frame,
    // read only while the owner keeps them registered)
    for (const auto& y : g->m)
        if (y.live && &y != &x && !registered(g, y.io_last)) {
            int rc = split(g);
            if (rc) return rc;
            return call_independent(g, i, io);
        }
    // the frame read in place (registered, page-locked, one stride): the step starts at once and
    // the leader copies the blocks it reads (the members' comparisons) while it runs; else the
    // leader copies them first into the mapped staging the step reads
    const float* in_dev = g->in_dev;
    int64_t ld_in = g->B;
    int rflags = 0;
    const bool inplace = inplace_frame(g, x, io, &in_dev, &ld_in, &rflags);
    const bool stable = inplace && (rflags & (NEO_HIP_GROUP_FRAME_STABLE | NEO_HIP_GROUP_FRAME_INPLACE));
    g->trust = stable;
    g->out_inplace = inplace && (rflags & NEO_HIP_GROUP_FRAME_INPLACE);
    // FRAME_INPLACE: the step writes every member's output into its own block of the frame
    float* out_dev = g->out_inplace ? const_cast<float*>(in_dev) : g->out_dev;
    const int64_t ld_out = g->out_inplace ? ld_in : g->B;
    auto copy_in = [&] {
        for (const auto& y : g->m)
            if (y.live) std::memcpy(g->in_pin + int64_t(y.slot) * g->B, &y == &x ? io : y.io_last, bb);
    };
    NEO_GP_T(t0);
    if (!inplace) copy_in();
    NEO_GP_ADD(0, t0);
    NEO_GP_T(t1);
    NEO_HIP_CHECK(hipMemcpyAsync(g->prev_bak, sh->prev, size_t(sh->C) * bb, hipMemcpyDeviceToDevice, g->stream));
    NEO_GP_ADD(1, t1);
    NEO_GP_T(t2);
    g->step_w = sh->wpos;
    int rc = neo_hip::launch_levels(sh, in_dev, ld_in, out_dev, ld_out, g->stream);
    NEO_GP_ADD(2, t2);
    NEO_GP_T(t3);
    if (inplace && !stable) copy_in();  // beside the step: both read the frame, which nothing writes during this call
    if (rc || (rc = neo_hip::spin_sync(g->stream))) return rc;
    NEO_GP_ADD(3, t3);
    g->step_n = sh->lv_n - 1;
    ++g->stat_steps;
    NEO_GP_T(t4);
    if (!g->out_inplace) std::memcpy(io, g->out_pin + int64_t(x.slot) * g->B, bb);
    NEO_GP_ADD(4, t4);
    prefetch_output(g, x.slot + 1);  // the next members' outputs, written over PCIe: not in any CPU cache
    prefetch_output(g, x.slot + 2);
    if (g->trust && !g->out_inplace)
        for (int k = 1; k <= NEO_GROUP_PFW; ++k) prefetch_block(g, x.slot + k);
    x.io_last = io;
    for (auto& y : g->m) {
        if (!y.live) continue;
        ++y.steps;
        if (&y != &x) {
            y.pending = true;
            ++g->npending;
        }
    }
    return NEO_HIP_OK;
}
}  // namespace

extern "C" {

NEO_HIP_API int neo_hip_upols_group_create(int block, int partitions, int method, int device, neo_hip_upols_group** out)
{
    if (!out) return fail(NEO_HIP_EINVAL, "group pointer is null");
    *out = nullptr;
    if (method != 0 && method != 1) return fail(NEO_HIP_EINVAL, "groups take method 0 (upols) or 1 (upola)");
    if (!neo_hip::valid_block(block)) return fail(NEO_HIP_EINVAL, "block must be a power of two in [16, 4096]");
    if (partitions < 1) return fail(NEO_HIP_EINVAL, "partitions must be >= 1");
    neo_hip::device_guard dg(device);
    if (dg.rc) return dg.rc;
    auto* g = new group_t{};
    (void)hipGetDevice(&g->device);
    g->B = block;
    g->P = partitions;
    g->method = method;
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        return fail(NEO_HIP_ERUNTIME, "hipStreamCreate failed");
    }
    *out = g;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_destroy(neo_hip_upols_group* g)
{
    if (!g) return NEO_HIP_OK;
    neo_hip::device_guard dg(g->device);
    (void)hipStreamSynchronize(g->stream);
    free_shared(g);
    for (auto& x : g->m)
        if (x.own) neo_hip_upols_destroy(x.own);
    neo_hip::hfree(g->stage_pin);
    for (const auto& r : g->reg) unpin_range(r.lo, r.hi);
    (void)hipStreamDestroy(g->stream);
    delete g;
    return NEO_HIP_OK;
}

// every entry point takes the group's lock before it looks at a member (a join on another
// thread may grow the member vector)
static bool live_member(const group_t* g, int id) { return id >= 0 && id < int(g->m.size()) && g->m[size_t(id)].live; }

NEO_HIP_API int neo_hip_upols_group_join(neo_hip_upols_group* g, int* id)
{
    if (!g || !id) return fail(NEO_HIP_EINVAL, "null group or id");
    std::lock_guard<std::mutex> lk(g->mu);
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    if (g->coalesced)
        if (int rc = split(g)) return rc;
    size_t i = 0;
    while (i < g->m.size() && g->m[i].live) ++i;
    if (i == g->m.size()) g->m.emplace_back();
    g->m[i] = member{};
    g->m[i].live = true;
    const int rc = make_own(g, g->m[i]);
    if (rc) {
        if (g->m[i].own) neo_hip_upols_destroy(g->m[i].own);
        g->m[i] = member{};
        return rc;
    }
    for (auto& y : g->m) y.seen = false;
    g->nseen = 0;
    g->good_frames = 0;
    *id = int(i);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_leave(neo_hip_upols_group* g, int id)
{
    if (!g) return fail(NEO_HIP_EINVAL, "null group");
    std::lock_guard<std::mutex> lk(g->mu);
    if (!live_member(g, id)) return fail(NEO_HIP_EINVAL, "no such member");
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    if (g->coalesced)
        if (int rc = split(g)) return rc;
    member& x = g->m[size_t(id)];
    if (x.own) neo_hip_upols_destroy(x.own);
    x = member{};
    for (auto& y : g->m) y.seen = false;
    g->nseen = 0;
    g->good_frames = 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_set_filter(neo_hip_upols_group* g, int id, const void* filter, int is_device)
{
    if (!g || !filter) return fail(NEO_HIP_EINVAL, "null group or filter");
    std::lock_guard<std::mutex> lk(g->mu);
    if (!live_member(g, id)) return fail(NEO_HIP_EINVAL, "no such member");
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    if (g->coalesced)
        if (int rc = split(g)) return rc;
    member& x = g->m[size_t(id)];
    if (int rc = neo_hip_upols_set_filter(x.own, filter, is_device)) return rc;  // resets its state
    x.own->batch = false;
    x.filtered = true;
    x.steps = 0;
    x.seen = false;
    for (auto& y : g->m) y.seen = false;
    g->nseen = 0;
    g->good_frames = 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_process(neo_hip_upols_group* g, int id, float* io)
{
    if (!g || !io) return fail(NEO_HIP_EINVAL, "null group or block");
    std::lock_guard<std::mutex> lk(g->mu);
    if (!live_member(g, id)) return fail(NEO_HIP_EINVAL, "no such member");
    ++g->stat_calls;
    NEO_GP_T(t0);
    if (g->coalesced && g->m[size_t(id)].pending) {  // a member's commit: no device guard (no HIP call)
        const int rc = call_coalesced(g, id, io);
        NEO_GP_ADD(8, t0);
        return rc;
    }
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    const int rc = g->coalesced ? call_coalesced(g, id, io) : call_independent(g, id, io);
    if (g->coalesced) NEO_GP_ADD(8, t0);
    return rc;
}

NEO_HIP_API int neo_hip_upols_group_reset(neo_hip_upols_group* g, int id)
{
    if (!g) return fail(NEO_HIP_EINVAL, "null group");
    std::lock_guard<std::mutex> lk(g->mu);
    if (!live_member(g, id)) return fail(NEO_HIP_EINVAL, "no such member");
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    if (g->coalesced)
        if (int rc = split(g)) return rc;
    member& x = g->m[size_t(id)];
    if (int rc = neo_hip_upols_reset(x.own)) return rc;
    x.steps = 0;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_register_ex(neo_hip_upols_group* g, const void* ptr, int64_t bytes, int flags)
{
    if (!g || !ptr || bytes <= 0) return fail(NEO_HIP_EINVAL, "null group or empty range");
    if (flags & ~(NEO_HIP_GROUP_FRAME_STABLE | NEO_HIP_GROUP_FRAME_INPLACE))
        return fail(NEO_HIP_EINVAL, "unknown group register flags %d", flags);
    std::lock_guard<std::mutex> lk(g->mu);
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr), hi = lo + uint64_t(bytes);
    for (auto& r : g->reg)
        if (r.lo == lo && r.hi == hi) {  // already registered (a per-frame call is cheap): the flags may change
            r.flags = flags;
            return NEO_HIP_OK;
        }
    neo_hip::device_guard dg(g->device);
    if (dg.rc) return dg.rc;
    pin_range(lo, hi);
    g->reg.push_back({lo, hi, flags});
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_register(neo_hip_upols_group* g, const void* ptr, int64_t bytes)
{
    return neo_hip_upols_group_register_ex(g, ptr, bytes, 0);
}

NEO_HIP_API int neo_hip_upols_group_unregister(neo_hip_upols_group* g, const void* ptr)
{
    if (!g) return fail(NEO_HIP_EINVAL, "null group");
    std::lock_guard<std::mutex> lk(g->mu);
    // no kernel reads a range after this returns: every coalesced step and redo completed in its
    // own call, and the next frame splits if a member's buffer is no longer registered
    const uintptr_t lo = reinterpret_cast<uintptr_t>(ptr);
    auto gone = [&](const group_t::range& r) { return !ptr || r.lo == lo; };
    for (const auto& r : g->reg)
        if (gone(r)) unpin_range(r.lo, r.hi);
    g->reg.erase(std::remove_if(g->reg.begin(), g->reg.end(), gone), g->reg.end());
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_group_stats(neo_hip_upols_group* g, int* coalesced, int64_t* frame_steps, int64_t* calls,
                                          int64_t* redos, int64_t* switches)
{
    if (!g) return fail(NEO_HIP_EINVAL, "null group");
    std::lock_guard<std::mutex> lk(g->mu);
    if (coalesced) *coalesced = g->coalesced;
    if (frame_steps) *frame_steps = g->stat_steps;
    if (calls) *calls = g->stat_calls;
    if (redos) *redos = g->stat_redos;
    if (switches) *switches = g->stat_switches;
    return NEO_HIP_OK;
}

}  // extern "C"
