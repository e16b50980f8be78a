// bench_hipcost.cpp — diagnostic: what the HIP runtime calls a convolver's bring-up and teardown
// make cost on this box (median and max of N calls each, microseconds): stream create / destroy,
// hipMalloc / hipFree by size, synchronous and stream-ordered memsets, events, pinned host
// memory. Decides what a handle may do per create (handle bring-up).
//   bench_hipcost [N]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

using clk = std::chrono::steady_clock;

static bool first = true;
static void report(const char* name, std::vector<double> t)
{
    std::sort(t.begin(), t.end());
    std::printf("%s\"%s\": [%.1f, %.1f]", first ? "" : ", ", name, t[t.size() / 2], t.back());
    first = false;
}

static void time_pair(const char* a_name, const char* b_name, int n, const std::function<void(int)>& a,
                      const std::function<void(int)>& b)
{
    std::vector<double> ta, tb;
    for (int i = 0; i < n; ++i) {
        auto t0 = clk::now();
        a(i);
        ta.push_back(std::chrono::duration<double>(clk::now() - t0).count() * 1e6);
    }
    for (int i = 0; i < n; ++i) {
        auto t0 = clk::now();
        b(i);
        tb.push_back(std::chrono::duration<double>(clk::now() - t0).count() * 1e6);
    }
    report(a_name, ta);
    report(b_name, tb);
}

int main(int argc, char** argv)
{
    const int N = argc > 1 ? std::atoi(argv[1]) : 64;
    if (hipSetDevice(0) != hipSuccess) {
        std::printf("{\"error\": \"no GPU\"}\n");
        return 0;
    }
    (void)hipFree(nullptr);
    std::printf("{\"n\": %d, \"us\": {", N);
    std::vector<hipStream_t> s(static_cast<size_t>(N));
    time_pair("stream_create", "stream_destroy", N, [&](int i) { (void)hipStreamCreateWithFlags(&s[size_t(i)], hipStreamDefault); },
              [&](int i) { (void)hipStreamDestroy(s[size_t(i)]); });
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    time_pair("stream_create_prio", "stream_destroy_prio", N,
              [&](int i) { (void)hipStreamCreateWithPriority(&s[size_t(i)], hipStreamNonBlocking, lo); },
              [&](int i) { (void)hipStreamDestroy(s[size_t(i)]); });
    std::vector<void*> p(static_cast<size_t>(N));
    for (size_t bytes : {size_t(256), size_t(1) << 20, size_t(8) << 20, size_t(64) << 20, size_t(256) << 20}) {
        const int n = bytes >= (size_t(64) << 20) ? std::min(N, 16) : N;
        std::string a = "malloc_" + std::to_string(bytes >> 10) + "k", b = "free_" + std::to_string(bytes >> 10) + "k";
        time_pair(a.c_str(), b.c_str(), n, [&](int i) { (void)hipMalloc(&p[size_t(i)], bytes); },
                  [&](int i) { (void)hipFree(p[size_t(i)]); });
    }
    void* buf = nullptr;
    (void)hipMalloc(&buf, size_t(8) << 20);
    hipStream_t st = nullptr;
    (void)hipStreamCreate(&st);
    time_pair("memset_8m_sync", "memset_async_8m_enqueue", N, [&](int) { (void)hipMemset(buf, 0, size_t(8) << 20); },
              [&](int) { (void)hipMemsetAsync(buf, 0, size_t(8) << 20, st); });
    time_pair("stream_sync_after_memsets", "stream_sync_idle", 1, [&](int) { (void)hipStreamSynchronize(st); },
              [&](int) { (void)hipStreamSynchronize(st); });
    time_pair("memcpy_h2d_2k_sync", "device_sync_idle", N,
              [&](int) {
                  static float h[512];
                  (void)hipMemcpy(buf, h, sizeof h, hipMemcpyHostToDevice);
              },
              [&](int) { (void)hipDeviceSynchronize(); });
    std::vector<hipEvent_t> e(static_cast<size_t>(N));
    time_pair("event_create", "event_destroy", N,
              [&](int i) { (void)hipEventCreateWithFlags(&e[size_t(i)], hipEventDisableTiming); },
              [&](int i) { (void)hipEventDestroy(e[size_t(i)]); });
    time_pair("host_malloc_4k", "host_free_4k", N,
              [&](int i) { (void)hipHostMalloc(&p[size_t(i)], 4096, hipHostMallocMapped | hipHostMallocCoherent); },
              [&](int i) { (void)hipHostFree(p[size_t(i)]); });
    std::vector<std::vector<float>> hb(static_cast<size_t>(N), std::vector<float>(size_t(1) << 20));
    time_pair("host_register_4m", "host_unregister_4m", N,
              [&](int i) { (void)hipHostRegister(hb[size_t(i)].data(), hb[size_t(i)].size() * 4, hipHostRegisterMapped); },
              [&](int i) { (void)hipHostUnregister(hb[size_t(i)].data()); });
    std::printf("}}\n");
    (void)hipFree(buf);
    (void)hipStreamDestroy(st);
    return 0;
}
