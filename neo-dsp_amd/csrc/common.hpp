// common.hpp — host-side plumbing shared by the neo_hip C-ABI translation units:
// the thread-local last-error latch, HIP status checks and twiddle tables.
#pragma once

#include "../../include/neo_hip.h"
#include "fft_device.hpp"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <type_traits>
#include <vector>

namespace neo_hip {

std::string& last_error_slot();

inline int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    last_error_slot() = buf;
    return code;
}

#define NEO_HIP_CHECK(expr)                                                                          \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess)                                                                        \
            return ::neo_hip::fail(NEO_HIP_ERUNTIME, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                   __FILE__, __LINE__);                                              \
    } while (0)

// Kernel launches: check the launch status immediately (catches bad configs).
#define NEO_HIP_LAUNCH_CHECK() NEO_HIP_CHECK(hipGetLastError())

// Scoped hipSetDevice that restores the caller's device.
struct device_guard {
    int prev = -1;
    bool changed = false;  // restore only what this guard changed (every entry point takes one)
    int rc = NEO_HIP_OK;
    explicit device_guard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) {
            if (hipSetDevice(dev) != hipSuccess) {
                (void)hipGetLastError();  // not sticky: a later launch check must not see it
                rc = fail(NEO_HIP_ENODEV, "hipSetDevice(%d) failed", dev);
            } else {
                changed = true;
            }
        }
    }
    ~device_guard()
    {
        if (changed && prev >= 0) (void)hipSetDevice(prev);
    }
};

// Forward twiddle table for an FFT of size n (see twiddle<> in fft_device.hpp): n <=
// kTwFull: W^e for e < max(64, n) (e mod n); larger: [0,64) = W^e, [64, 64+n/64) =
// W^(64h); W = exp(-2*pi*i/n), computed in double (long double for the f64 tables) and
// rounded once.
template<class C = cf>
inline std::vector<C> make_twiddle_table(int64_t n)
{
    using R = real_of<C>;
    using W = std::conditional_t<sizeof(R) == 8, long double, double>;
    const W pi2 = W(2) * W(3.14159265358979323846264338327950288L);
    if (n <= kTwFull) {
        std::vector<C> t(static_cast<size_t>(n < 64 ? 64 : n));
        for (int64_t e = 0; e < int64_t(t.size()); ++e) {
            const W a = -pi2 * W(e % (n > 0 ? n : 1)) / W(n > 0 ? n : 1);
            t[size_t(e)] = {R(std::cos(a)), R(std::sin(a))};
        }
        return t;
    }
    const int64_t lo = 64, hi = n <= 64 ? 0 : n / 64;
    std::vector<C> t(static_cast<size_t>(lo + hi));
    for (int64_t e = 0; e < lo; ++e) {
        const W a = -pi2 * W(e % (n > 0 ? n : 1)) / W(n > 0 ? n : 1);
        t[size_t(e)] = {R(std::cos(a)), R(std::sin(a))};
    }
    for (int64_t h = 0; h < hi; ++h) {
        const W a = -pi2 * W(64 * h) / W(n);
        t[size_t(lo + h)] = {R(std::cos(a)), R(std::sin(a))};
    }
    return t;
}

// Split table for the global-memory passes of large transforms: e = hi*2^lo_bits + lo.
template<class C = cf>
inline std::vector<C> make_split_table(int order, int lo_bits)
{
    using R = real_of<C>;
    using W = std::conditional_t<sizeof(R) == 8, long double, double>;
    const W pi2 = W(2) * W(3.14159265358979323846264338327950288L);
    const int64_t n = int64_t(1) << order, nlo = int64_t(1) << lo_bits, nhi = n >> lo_bits;
    std::vector<C> t(static_cast<size_t>(nlo + nhi));
    for (int64_t e = 0; e < nlo; ++e) {
        const W a = -pi2 * W(e) / W(n);
        t[size_t(e)] = {R(std::cos(a)), R(std::sin(a))};
    }
    for (int64_t h = 0; h < nhi; ++h) {
        const W a = -pi2 * W(h * nlo) / W(n);
        t[size_t(nlo + h)] = {R(std::cos(a)), R(std::sin(a))};
    }
    return t;
}

// dmem.hip: device memory for handle buffers, sub-allocated from cached per-device chunks (freeing
// never synchronizes the device; free only memory no queued work still uses); twiddle tables
// shared by every handle on a device, never freed
int dalloc(void** out, size_t bytes);
void dfree(void* p);
// persistent (latency-mode) workgroups running per device: reserve wgs if the total stays <= cap
// (false: no room, nothing reserved); release them when the kernel is joined
bool resident_admit(int device, int wgs, int cap);
void resident_release(int device, int wgs);
template<class T>
inline int dalloc(T** out, size_t bytes)
{
    void* v = nullptr;
    const int rc = dalloc(&v, bytes);
    *out = static_cast<T*>(v);
    return rc;
}
int halloc(void** host, void** dev, size_t bytes);  // mapped page-locked host memory, pooled
void hfree(void* host);
int shared_stream(hipStream_t* out);  // one of four blocking streams per device, never destroyed
int shared_tw(cf** out, int B);  // upload_tw's table for block B
int shared_far_tw(cf** out);     // the 256-point forward table of the far level

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// A device-resident input's producer, for the synchronous setup calls: the work enqueued on the
// HIP null stream (torch's default stream) before the call. Joined with an event marker on the
// null stream, which waits for the blocking streams' earlier work only; hipDeviceSynchronize (and
// hipStreamSynchronize on the null stream) would also wait for every non-blocking stream, e.g.
// another handle's resident latency-mode kernel, up to its idle limit. A producer on another
// non-blocking stream is the caller's to join (the Python layer synchronizes torch's current
// stream first). dmem.hip.
int null_join();

// The streams a handle's (or plan's) asynchronous calls ran on since its last join: a setup call
// or a destroy waits for these, not for the device. A stream given to such a call stays valid
// until then. On overflow the remembered streams are joined first (their work is then complete).
struct stream_set {
    static constexpr int kMax = 16;
    hipStream_t s[kMax] = {};
    int n = 0;
    int note(hipStream_t x)
    {
        for (int i = 0; i < n; ++i)
            if (s[i] == x) return NEO_HIP_OK;
        if (n == kMax)
            if (int rc = join()) return rc;
        s[n++] = x;
        return NEO_HIP_OK;
    }
    int join()
    {
        const int k = n;
        n = 0;
        for (int i = 0; i < k; ++i) {
            if (!s[i]) {  // the null stream: its own work only (null_join)
                if (int rc = null_join()) return rc;
            } else {
                NEO_HIP_CHECK(hipStreamSynchronize(s[i]));
            }
        }
        return NEO_HIP_OK;
    }
};

// The device address of page-locked host memory (hipHostMalloc, hipHostRegister with the
// mapped flag, neo_hip_host_register), or nullptr for pageable memory (not an error).
inline float* host_mapped(void* p)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: not sticky for later launch checks
        return nullptr;
    }
    return at.type == hipMemoryTypeHost ? static_cast<float*>(at.devicePointer) : nullptr;
}

// Wait for a stream by polling (a real-time caller's block deadline: no yield to the OS
// scheduler, whose wake-up adds tens of microseconds per block).
inline int spin_sync(hipStream_t s)
{
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return NEO_HIP_OK;
        if (e != hipErrorNotReady)
            return fail(NEO_HIP_ERUNTIME, "hipStreamQuery: %s (%s:%d)", hipGetErrorString(e), __FILE__, __LINE__);
    }
}

}  // namespace neo_hip
