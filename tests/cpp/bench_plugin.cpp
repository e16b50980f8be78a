// bench_plugin.cpp — the plugin's own processing class (extra/plugin/src/dsp/Convolution.hpp:60-63,
// 112): std::vector<split_upols_convolver<complex<float>>>, one per channel, each called in place
// on the host's channel buffer once per block. split_* is never aliased to a group, so every
// channel-block is a call of its own: a launch and a host wait (normal mode) or a mailbox record
// for the channel's resident kernel (latency mode). Prints one JSON line (bench.py
// host_io.plugin_*): per-frame (all channels) and per-call microseconds, p50 / p99.
//   bench_plugin <channels> <frames> [block] [taps] [latency 0/1]
#include <neo/convolution.hpp>

#include "../../oracle/neo_oracle.h"

#include <algorithm>
#include <chrono>
#include <complex>
#include <cstdio>
#include <cstdlib>
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
    std::size_t const C = argc > 1 ? std::size_t(std::atol(argv[1])) : 2;
    std::size_t const nf = argc > 2 ? std::size_t(std::atol(argv[2])) : 400;
    std::size_t const B = argc > 3 ? std::size_t(std::atol(argv[3])) : 512;
    std::size_t const L = argc > 4 ? std::size_t(std::atol(argv[4])) : 480000;
    bool const latency = argc > 5 && std::atoi(argv[5]) != 0;
    // a stereo IR (Convolution::update: uniform_partition of every channel, then filter per channel)
    std::vector<float> ir(C * L);
    oracle_noise(91, ir.data(), ir.size());
    neo::convolution::normalize_impulse(neo::hip::make_matrix_view(ir.data(), C, L));
    auto t0 = clk::now();
    std::vector<neo::convolution::split_upols_convolver<cf>> convolvers(C);
    for (std::size_t ch = 0; ch < C; ++ch) {
        auto const parts = neo::convolution::uniform_partition(neo::hip::make_matrix_view(ir.data() + ch * L, 1, L), B);
        std::size_t const P = parts.extent(1), bins = B + 1;
        if (latency) convolvers[ch].latency_mode(true);
        convolvers[ch].filter(neo::hip::make_matrix_view(const_cast<cf*>(parts.data()), P, bins));
    }
    double const setup_s = std::chrono::duration<double>(clk::now() - t0).count();
    std::vector<float> src(C * B * 16), frame(C * B);
    oracle_noise(92, src.data(), src.size());
    std::vector<double> tf, tc;
    tf.reserve(nf);
    tc.reserve(nf * C);
    std::size_t const warm = 16;
    for (std::size_t f = 0; f < nf + warm; ++f) {
        for (std::size_t ch = 0; ch < C; ++ch)
            std::copy_n(src.data() + ((f % 16) * C + ch) * B, B, frame.data() + ch * B);
        auto const a = clk::now();
        for (std::size_t ch = 0; ch < C; ++ch) {  // Convolution::process: one call per channel, in place
            auto const c0 = clk::now();
            convolvers[ch](neo::hip::make_view(frame.data() + ch * B, B));
            if (f >= warm) tc.push_back(std::chrono::duration<double, std::micro>(clk::now() - c0).count());
        }
        if (f >= warm) tf.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    std::printf("{\"channels\": %zu, \"block\": %zu, \"taps\": %zu, \"frames\": %zu, \"latency_mode\": %s, "
                "\"setup_s\": %.4f, \"frame_us_p50\": %.2f, \"frame_us_p99\": %.2f, \"call_us_p50\": %.2f, "
                "\"call_us_p99\": %.2f, \"msamples_per_s_back_to_back\": %.2f}\n",
                C, B, L, nf, latency ? "true" : "false", setup_s, pct(tf, 50), pct(tf, 99), pct(tc, 50), pct(tc, 99),
                double(C * B) / pct(tf, 50));
    return 0;
}
