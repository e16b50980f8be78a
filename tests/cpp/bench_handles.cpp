// bench_handles.cpp — diagnostic: the host round trip of one single-channel convolver's
// neo_hip_upols_process call (host block, the handle's staging) while N - 1 other handles of the
// same shape exist and stay idle. bench_handles <N> [block] [partitions]
#include <neo_hip.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv)
{
    const int N = argc > 1 ? std::atoi(argv[1]) : 1, B = argc > 2 ? std::atoi(argv[2]) : 512,
              P = argc > 3 ? std::atoi(argv[3]) : 938;
    std::vector<neo_hip_upols*> h(size_t(N), nullptr);
    std::vector<float> filt(size_t(P) * (B + 1) * 2, 0.0f);
    filt[0] = 1.0f;
    for (int i = 0; i < N; ++i) {
        if (neo_hip_upols_create(1, B, P, 0, &h[size_t(i)]) || neo_hip_upols_set_filter(h[size_t(i)], filt.data(), 0)) {
            std::printf("{\"error\": \"%s\"}\n", neo_hip_last_error());
            return 1;
        }
        if (i == 0) neo_hip_upols_set_batch(h[0], 0);
    }
    std::vector<float> blk(size_t(B), 0.5f);
    std::vector<double> t;
    for (int k = 0; k < 400; ++k) {
        const auto a = std::chrono::steady_clock::now();
        if (neo_hip_upols_process(h[0], blk.data(), 0, nullptr)) {
            std::printf("{\"error\": \"%s\"}\n", neo_hip_last_error());
            return 1;
        }
        if (k >= 100) t.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count() * 1e6);
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"handles\": %d, \"p50_us\": %.2f, \"p99_us\": %.2f, \"max_us\": %.2f}\n", N, t[t.size() / 2],
                t[t.size() * 99 / 100], t.back());
    for (auto* x : h) neo_hip_upols_destroy(x);
    return 0;
}
