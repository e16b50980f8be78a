// dmem.hip — device memory for convolver handles, sub-allocated from cached chunks.
//
// A plugin brings up and tears down many small convolvers (DenseConvolution::updateImpulseResponse
// rebuilds one per channel, extra/plugin/src/dsp/DenseConvolution.cpp:78-108; a convolver group
// switches between one shared handle and a handle per member). With hipMalloc / hipFree per
// buffer that costs milliseconds per handle: hipFree waits for the whole device (every stream,
// including another handle's resident latency-mode kernel). Here a handle's buffers come from
// chunks per device (first fit, neighbours merged on free) that stay mapped: freeing is a list
// operation, no device synchronization. The caller frees only memory no queued work uses (handles
// join their streams first). A new chunk is 256 MiB, or the request's size above 64 MiB (a
// multichannel handle's filter and delay line). Empty chunks stay cached, up to a quarter of the
// device's memory, and serve any later request that fits: a group switching from its shared
// handle to a handle per member (upols_group.hip split) carves the members' buffers from the
// shared handle's just-freed chunks instead of returning 48 GB to the driver and mapping 45 GB
// anew. Before a new chunk for a request above 64 MiB is mapped, the cached empty chunks are
// returned; neo_hip_memory_trim returns them on demand.
//
// Also the constant tables every handle of a block size shares (twiddles), uploaded once per
// device and never freed.
#include "upols_handle.hpp"

#include <atomic>
#include <map>
#include <memory>
#include <tuple>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace neo_hip {
namespace {

constexpr size_t kAlign = 256;
constexpr size_t kChunk = size_t(256) << 20;
constexpr size_t kDedicated = size_t(64) << 20;

struct chunk {
    char* base = nullptr;
    size_t size = 0, used = 0;
    bool dedicated = false;
    std::map<size_t, size_t> free;  // offset -> bytes, disjoint, merged
};

struct pool {
    std::vector<std::unique_ptr<chunk>> chunks;
    std::vector<std::unique_ptr<chunk>> pinned;  // mapped page-locked host chunks (halloc)
    std::map<int, cf*> tw;                       // shared tables: block size (or -1, the far level) -> table
    hipStream_t streams[4] = {};                 // shared handle streams (shared_stream)
    unsigned next_stream = 0;
};
constexpr size_t kPinnedChunk = size_t(4) << 20;

// one lock for every device's pool (handle bring-up and teardown, not a hot path)
std::mutex g_mu;
std::map<int, pool> g_pools;
std::unordered_map<const void*, std::tuple<int, chunk*, size_t>> g_live;  // pointer -> device, chunk, bytes

size_t empty_bytes(const pool& p)
{
    size_t n = 0;
    for (const auto& c : p.chunks) n += c->used == 0 ? c->size : 0;
    return n;
}

// empty chunks kept cached per device: a quarter of its memory
size_t keep_bytes()
{
    static size_t keep = [] {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
            (void)hipGetLastError();
            return size_t(1) << 30;
        }
        return tot / 4;
    }();
    return keep;
}

void release(pool& p, size_t i)
{
    (void)hipFree(p.chunks[i]->base);
    p.chunks.erase(p.chunks.begin() + std::ptrdiff_t(i));
}

// chunks taken out of a pool under g_mu, returned to the driver after it is released: hipFree
// waits for the device, and no other thread's allocation may wait on the lock meanwhile. Declared
// before the lock_guard, so its destructor runs after the guard's.
struct deferred_free {
    std::vector<std::unique_ptr<chunk>> v;
    void take(pool& p, size_t i)
    {
        v.push_back(std::move(p.chunks[i]));
        p.chunks.erase(p.chunks.begin() + std::ptrdiff_t(i));
    }
    ~deferred_free()
    {
        for (auto& c : v) (void)hipFree(c->base);
    }
};

// persistent (latency-mode) workgroups running per device (resident_admit): while a persistent
// kernel runs, hipFree would wait for it (up to its idle limit, indefinitely while an audio
// thread keeps feeding it), so dfree keeps empty chunks cached instead of returning them
std::atomic<int> g_resident[64];

bool take(chunk& c, size_t bytes, void** out)
{
    for (auto it = c.free.begin(); it != c.free.end(); ++it) {
        if (it->second < bytes) continue;
        const size_t off = it->first, left = it->second - bytes;
        c.free.erase(it);
        if (left) c.free.emplace(off + bytes, left);
        c.used += bytes;
        *out = c.base + off;
        return true;
    }
    return false;
}

}  // namespace

int dalloc(void** out, size_t bytes)
{
    *out = nullptr;
    int dev = 0;
    NEO_HIP_CHECK(hipGetDevice(&dev));
    const size_t n = (std::max<size_t>(bytes, 1) + kAlign - 1) / kAlign * kAlign;
    std::lock_guard<std::mutex> lk(g_mu);
    pool& p = g_pools[dev];
    for (auto& c : p.chunks)
        if (take(*c, n, out)) {
            g_live.emplace(*out, std::make_tuple(dev, c.get(), n));
            return NEO_HIP_OK;
        }
    auto release_empty = [&] {
        for (size_t i = p.chunks.size(); i-- > 0;)
            if (p.chunks[i]->used == 0) release(p, i);
    };
    if (n > kDedicated) release_empty();  // no cached chunk fits: give them back before mapping a big one
    auto c = std::make_unique<chunk>();
    constexpr size_t k2m = size_t(2) << 20;
    c->size = n > kDedicated ? (n + k2m - 1) / k2m * k2m : kChunk;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->base), c->size);
    if (e != hipSuccess) {  // give the cached empty chunks back and try once more
        (void)hipGetLastError();
        release_empty();
        e = hipMalloc(reinterpret_cast<void**>(&c->base), c->size);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(NEO_HIP_ENOMEM, "device allocation of %zu bytes failed", bytes);
        }
    }
    c->free.emplace(0, c->size);
    (void)take(*c, n, out);
    g_live.emplace(*out, std::make_tuple(dev, c.get(), n));
    p.chunks.push_back(std::move(c));
    return NEO_HIP_OK;
}

bool resident_admit(int device, int wgs, int cap)
{
    if (device < 0 || device >= 64) return false;
    int cur = g_resident[device].load();
    do {
        if (cur + wgs > cap) return false;
    } while (!g_resident[device].compare_exchange_weak(cur, cur + wgs));
    return true;
}

void resident_release(int device, int wgs)
{
    if (device >= 0 && device < 64) g_resident[device].fetch_sub(wgs);
}

void dfree(void* ptr)
{
    if (!ptr) return;
    deferred_free doomed;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(ptr);
    if (it == g_live.end()) return;  // not ours: nothing to do (never hipFree a foreign pointer)
    const auto [dev, c, n] = it->second;
    g_live.erase(it);
    pool& p = g_pools[dev];
    size_t off = size_t(static_cast<char*>(ptr) - c->base), len = n;
    auto nx = c->free.lower_bound(off);
    if (nx != c->free.end() && nx->first == off + len) {  // merge with the range after
        len += nx->second;
        nx = c->free.erase(nx);
    }
    if (nx != c->free.begin()) {  // and the range before
        auto pv = std::prev(nx);
        if (pv->first + pv->second == off) {
            off = pv->first;
            len += pv->second;
            c->free.erase(pv);
        }
    }
    c->free.emplace(off, len);
    c->used -= n;
    if (c->used) return;
    if (empty_bytes(p) <= keep_bytes()) return;  // cached for later requests of any size
    if (dev >= 0 && dev < 64 && g_resident[dev].load()) return;  // no hipFree beside a resident kernel
    for (size_t i = 0; i < p.chunks.size(); ++i)
        if (p.chunks[i].get() == c) {
            doomed.take(p, i);  // hipFree after the lock is released
            break;
        }
}

// Page-locked, device-mapped host memory (hipHostMalloc mapped + coherent) from 4 MiB chunks
// that stay allocated (hipHostFree costs ~0.25 ms); larger requests get a chunk of their own,
// freed with them. *dev: the device address of *host.
int halloc(void** host, void** dev, size_t bytes)
{
    *host = *dev = nullptr;
    int d = 0;
    NEO_HIP_CHECK(hipGetDevice(&d));
    const size_t n = (std::max<size_t>(bytes, 1) + kAlign - 1) / kAlign * kAlign;
    std::lock_guard<std::mutex> lk(g_mu);
    pool& p = g_pools[d];
    chunk* c = nullptr;
    if (n <= kPinnedChunk)
        for (auto& x : p.pinned)
            if (!x->dedicated && take(*x, n, host)) {
                c = x.get();
                break;
            }
    if (!c) {
        auto x = std::make_unique<chunk>();
        x->dedicated = n > kPinnedChunk;
        x->size = x->dedicated ? n : kPinnedChunk;
        if (hipHostMalloc(reinterpret_cast<void**>(&x->base), x->size, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
            (void)hipGetLastError();
            return fail(NEO_HIP_ENOMEM, "pinned host allocation of %zu bytes failed", bytes);
        }
        x->free.emplace(0, x->size);
        (void)take(*x, n, host);
        c = x.get();
        p.pinned.push_back(std::move(x));
    }
    void* db = nullptr;
    NEO_HIP_CHECK(hipHostGetDevicePointer(&db, c->base, 0));
    *dev = static_cast<char*>(db) + (static_cast<char*>(*host) - c->base);
    g_live.emplace(*host, std::make_tuple(d, c, n));
    return NEO_HIP_OK;
}

void hfree(void* host)
{
    if (!host) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.find(host);
    if (it == g_live.end()) return;
    const auto [d, c, n] = it->second;
    g_live.erase(it);
    pool& p = g_pools[d];
    if (c->dedicated) {
        (void)hipHostFree(c->base);
        for (size_t i = 0; i < p.pinned.size(); ++i)
            if (p.pinned[i].get() == c) {
                p.pinned.erase(p.pinned.begin() + std::ptrdiff_t(i));
                break;
            }
        return;
    }
    const size_t off = size_t(static_cast<char*>(host) - c->base);
    c->free.emplace(off, n);  // small chunks are kept: no merge needed for correctness, merge anyway
    for (auto a = c->free.begin(); a != c->free.end();) {
        auto b = std::next(a);
        if (b != c->free.end() && a->first + a->second == b->first) {
            a->second += b->second;
            c->free.erase(b);
        } else {
            a = b;
        }
    }
    c->used -= n;
}

// A blocking stream for a handle's own setup and host-I/O work, from a per-device set of four
// (GPU_MAX_HW_QUEUES is 4: more streams only share those hardware queues): creating a stream
// costs ~4 ms and destroying one ~3 ms on MI355X (tests/cpp/bench_hipcost), the whole budget of
// a plugin's convolver bring-up. Never destroyed.
int shared_stream(hipStream_t* out)
{
    int d = 0;
    NEO_HIP_CHECK(hipGetDevice(&d));
    std::lock_guard<std::mutex> lk(g_mu);
    pool& p = g_pools[d];
    // each created when first handed out: creating all four at once took every hardware queue, and
    // the first handle's background stream then shared one with its own stream, its host-buffer
    // blocks queueing behind the background launches (same-box A/B, c5full host round trip p50 /
    // p99: 181-195 / 259-263 us all at once, 132 / 157-166 created one by one, 131-133 / 156-161
    // with a stream of its own per handle as in round 4; tools/gpu_hostio_ab.sh)
    hipStream_t& s = p.streams[p.next_stream++ % 4];
    if (!s) NEO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamDefault));
    *out = s;
    return NEO_HIP_OK;
}

int null_join()
{
    int d = 0;
    NEO_HIP_CHECK(hipGetDevice(&d));
    thread_local std::map<int, hipEvent_t> ev;  // one marker per thread and device, never destroyed
    hipEvent_t& e = ev[d];
    if (!e) NEO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    NEO_HIP_CHECK(hipEventRecord(e, nullptr));
    NEO_HIP_CHECK(hipEventSynchronize(e));
    return NEO_HIP_OK;
}

namespace {
// a constant table shared by every handle on the current device (key: block size, or -1 for the
// far level's), made by upload on first use
template<class F>
int shared_table(cf** out, int key, F upload)
{
    int dev = 0;
    NEO_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_mu);
    pool& p = g_pools[dev];
    if (auto it = p.tw.find(key); it != p.tw.end()) {
        *out = it->second;
        return NEO_HIP_OK;
    }
    cf* d = nullptr;
    if (int rc = upload(&d)) return rc;
    p.tw.emplace(key, d);
    *out = d;
    return NEO_HIP_OK;
}
}  // namespace

// the forward twiddle tables of a B-point packed real transform (upload_tw's contents)
int shared_tw(cf** out, int B)
{
    return shared_table(out, B, [B](cf** d) { return upload_tw(d, B); });
}

int shared_far_tw(cf** out)
{
    return shared_table(out, -1, [](cf** d) -> int {
        const auto t = make_twiddle_table(2 * kFarT);
        NEO_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(d), t.size() * sizeof(cf)));
        NEO_HIP_CHECK(hipMemcpy(*d, t.data(), t.size() * sizeof(cf), hipMemcpyHostToDevice));
        return NEO_HIP_OK;
    });
}

}  // namespace neo_hip

extern "C" {

NEO_HIP_API int neo_hip_memory_trim(int device)
{
    neo_hip::device_guard g(device);
    if (g.rc) return g.rc;
    int dev = 0;
    NEO_HIP_CHECK(hipGetDevice(&dev));
    neo_hip::deferred_free doomed;  // returned after the lock is released
    std::lock_guard<std::mutex> lk(neo_hip::g_mu);
    neo_hip::pool& p = neo_hip::g_pools[dev];
    for (size_t i = p.chunks.size(); i-- > 0;)
        if (p.chunks[i]->used == 0) doomed.take(p, i);
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_memory_info(int device, int64_t* reserved, int64_t* in_use)
{
    neo_hip::device_guard g(device);
    if (g.rc) return g.rc;
    int dev = 0;
    NEO_HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(neo_hip::g_mu);
    neo_hip::pool& p = neo_hip::g_pools[dev];
    int64_t r = 0, u = 0;
    for (const auto& c : p.chunks) {
        r += int64_t(c->size);
        u += int64_t(c->used);
    }
    if (reserved) *reserved = r;
    if (in_use) *in_use = u;
    return NEO_HIP_OK;
}

}  // extern "C"
