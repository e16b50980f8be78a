// bench_group.cpp — frame times of the plugin's call pattern with the group-backed convolver alias
// (NEO_HIP_CONVOLVER_GROUPS): DenseConvolution holds std::vector<upols_convolver> (
// extra/plugin/src/dsp/DenseConvolution.hpp:35) and processFrame calls them channel by channel on
// its frame buffer (DenseConvolution.cpp:62-74). The owner registers that buffer, so after three
// watched frames a frame is one launch. Also the dense_convolve<Convolver> harness pattern
// (DenseConvolution.hpp:56-67: one scratch block shared by every channel), which never coalesces:
// one launch and one host wait per channel-block, after one frame that switches the group back to
// a handle per member (switch_frame_us). Prints one JSON line (bench.py host_io.group_*).
// mode = 1 registers the frame with NEO_HIP_GROUP_FRAME_STABLE (the owner's promise that only the
// convolvers' calls write it during a frame): members commit without the snapshot comparison;
// mode = 2 with NEO_HIP_GROUP_FRAME_INPLACE too (read only through the calls, each convolver on its
// own channel): the frame's first call writes every output in place.
//   bench_group <channels> <frames> [block] [taps] [mode]
#define NEO_HIP_CONVOLVER_GROUPS 1
#include <neo/convolution.hpp>

#include "../../oracle/neo_oracle.h"

#include <algorithm>
#include <chrono>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using cf = std::complex<float>;
using clk = std::chrono::steady_clock;

static double pct(std::vector<double> v, double p)
{
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, std::size_t(p / 100.0 * double(v.size() - 1) + 0.5))];
}

int main(int argc, char** argv)
{
    int ndev = 0;
    if (neo_hip_device_count(&ndev) != NEO_HIP_OK || ndev < 1) {
        std::printf("{\"error\": \"no GPU\"}\n");
        return 0;
    }
    std::size_t const C = argc > 1 ? std::size_t(std::atol(argv[1])) : 256;
    std::size_t const nf = argc > 2 ? std::size_t(std::atol(argv[2])) : 64;
    std::size_t const B = argc > 3 ? std::size_t(std::atol(argv[3])) : 512;
    std::size_t const L = argc > 4 ? std::size_t(std::atol(argv[4])) : 480000;
    int const mode = argc > 5 ? std::atoi(argv[5]) : 0;
    using promise = neo::convolution::convolver_group::frame;
    // one IR for every channel (the frame time does not depend on the filter's values)
    std::vector<float> ir(L);
    oracle_noise(77, ir.data(), L);
    neo::convolution::normalize_impulse(neo::hip::make_matrix_view(ir.data(), 1, L));
    auto const parts = neo::convolution::uniform_partition(neo::hip::make_matrix_view(ir.data(), 1, L), B);
    std::size_t const P = parts.extent(1), bins = B + 1;
    auto t0 = clk::now();
    neo::convolution::convolver_group owner;
    std::vector<neo::convolution::upols_convolver<cf>> convolvers(C);
    {
        auto scope = owner.scope();
        for (auto& cv : convolvers) cv.filter(neo::hip::make_matrix_view(const_cast<cf*>(parts.data()), P, bins));
    }
    double const setup_s = std::chrono::duration<double>(clk::now() - t0).count();
    std::vector<float> src(C * B * 8), frame(C * B);
    oracle_noise(78, src.data(), src.size());
    owner.register_buffer(frame.data(), frame.size(),
                          mode == 2 ? promise::in_place : (mode == 1 ? promise::stable : promise::plain));
    auto process_frame = [&](std::size_t f) {
        std::memcpy(frame.data(), src.data() + (f % 8) * C * B, C * B * sizeof(float));  // the host fills the frame
        auto const a = clk::now();
        for (std::size_t c = 0; c < C; ++c) convolvers[c](neo::hip::make_view(frame.data() + c * B, B));
        return std::chrono::duration<double>(clk::now() - a).count();
    };
    for (std::size_t f = 0; f < 8; ++f) (void)process_frame(f);  // watched frames, then coalesced
    std::vector<double> ft;
    for (std::size_t f = 0; f < nf; ++f) ft.push_back(process_frame(f) * 1e6);
    int coalesced = 0;
    std::int64_t steps = 0, calls = 0, redos = 0, switches = 0;
    neo::hip::check(neo_hip_upols_group_stats(convolvers[0].group(), &coalesced, &steps, &calls, &redos, &switches));
    // the harness pattern: one shared scratch block for every channel (never coalesces). Its
    // first frame is still coalesced (every member's block redone: untimed), its second splits
    // the group (a handle per member, each member's levels re-primed at its first call: timed
    // as the switch), the frames after it are the steady state
    std::vector<float> scratch(B);
    std::size_t const sf = std::max<std::size_t>(2, 1024 / C);
    std::vector<double> ct;
    double switch_us = 0;
    for (std::size_t f = 0; f <= sf + 1; ++f)
        for (std::size_t c = 0; c < C; ++c) {
            std::memcpy(scratch.data(), src.data() + ((f % 8) * C + c) * B, B * sizeof(float));
            auto const a = clk::now();
            convolvers[c](neo::hip::make_view(scratch.data(), B));
            double const us = std::chrono::duration<double>(clk::now() - a).count() * 1e6;
            if (f == 1) switch_us += us;
            if (f > 1) ct.push_back(us);
        }
    double mean = 0;
    for (double v : ft) mean += v;
    mean /= double(ft.size());
    double cmean = 0;
    for (double v : ct) cmean += v;
    cmean /= double(ct.size());
    std::printf("{\"channels\": %zu, \"block\": %zu, \"partitions\": %zu, \"frames\": %zu, \"frame_mode\": %d, \"coalesced\": %d, "
                "\"one_launch_frames\": %lld, \"redos\": %lld, \"frame_p50_us\": %.2f, \"frame_p99_us\": %.2f, "
                "\"frame_mean_us\": %.2f, \"msamples_s\": %.2f, \"setup_s\": %.2f, "
                "\"shared_scratch\": {\"channel_blocks\": %zu, \"per_channel_block_p50_us\": %.2f, "
                "\"per_channel_block_mean_us\": %.2f, \"frame_us\": %.1f, \"msamples_s\": %.2f, "
                "\"switch_frame_us\": %.1f}}\n",
                C, B, P, nf, mode, coalesced, (long long)steps, (long long)redos, pct(ft, 50), pct(ft, 99), mean,
                double(C * B) / mean, setup_s, ct.size(), pct(ct, 50), cmean, cmean * double(C), double(B) / cmean, switch_us);
    return 0;
}
