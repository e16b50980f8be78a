// bench_create.cpp — diagnostic: what a one-channel convolver costs to bring up, phase by phase
// (the group's switch from one shared handle to a handle per member pays this per member):
// create, set_filter, the first streaming step (level buffers allocated, far segment spectra,
// priming), a later step, destroy; median and max over N handles created one after another,
// after one untimed warm-up handle.
//   bench_create <N> [block] [partitions]
#include <neo_hip.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

using clk = std::chrono::steady_clock;

static double us(clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count() * 1e6; }

int main(int argc, char** argv)
{
    const int N = argc > 1 ? std::atoi(argv[1]) : 64, B = argc > 2 ? std::atoi(argv[2]) : 512,
              P = argc > 3 ? std::atoi(argv[3]) : 938;
    std::vector<float> filt(size_t(P) * (B + 1) * 2, 0.0f), blk(size_t(B), 0.5f);
    filt[0] = 1.0f;
    {  // warm-up, untimed: the HIP runtime's initialization and the first load of every kernel's
       // code object happen once per process, not per handle
        neo_hip_upols* w = nullptr;
        if (neo_hip_upols_create_ex(1, B, P, 0, 0, nullptr, &w) || neo_hip_upols_set_filter(w, filt.data(), 0) ||
            neo_hip_upols_set_batch(w, 0) || neo_hip_upols_process(w, blk.data(), 0, nullptr) ||
            neo_hip_upols_process(w, blk.data(), 0, nullptr)) {
            std::printf("{\"error\": \"%s\"}\n", neo_hip_last_error());
            return 1;
        }
        neo_hip_upols_destroy(w);
    }
    std::vector<neo_hip_upols*> h(size_t(N), nullptr);
    const char* names[5] = {"create", "set_filter", "first_step", "later_step", "destroy"};
    std::vector<std::vector<double>> t(5);
    for (int i = 0; i < N; ++i) {
        auto a = clk::now();
        int rc = neo_hip_upols_create_ex(1, B, P, 0, 0, nullptr, &h[size_t(i)]);
        t[0].push_back(us(a));
        a = clk::now();
        rc = rc ? rc : neo_hip_upols_set_filter(h[size_t(i)], filt.data(), 0);
        t[1].push_back(us(a));
        rc = rc ? rc : neo_hip_upols_set_batch(h[size_t(i)], 0);
        a = clk::now();
        rc = rc ? rc : neo_hip_upols_process(h[size_t(i)], blk.data(), 0, nullptr);
        t[2].push_back(us(a));
        a = clk::now();
        rc = rc ? rc : neo_hip_upols_process(h[size_t(i)], blk.data(), 0, nullptr);
        t[3].push_back(us(a));
        if (rc) {
            std::printf("{\"error\": \"%s\"}\n", neo_hip_last_error());
            return 1;
        }
    }
    for (auto* x : h) {
        auto a = clk::now();
        neo_hip_upols_destroy(x);
        t[4].push_back(us(a));
    }
    std::printf("{\"handles\": %d, \"block\": %d, \"partitions\": %d", N, B, P);
    for (int k = 0; k < 5; ++k) {
        std::sort(t[size_t(k)].begin(), t[size_t(k)].end());
        std::printf(", \"%s_us\": [%.1f, %.1f]", names[k], t[size_t(k)][t[size_t(k)].size() / 2], t[size_t(k)].back());
    }
    std::printf("}\n");
    return 0;
}
