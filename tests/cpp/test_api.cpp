// test_api.cpp — the reference's own hot-path tests re-expressed against the
// MI355X neo::fft / neo::convolution headers (include/neo/*.hpp -> libneo_hip.so),
// checked against the CPU restatement (oracle/, test infrastructure).
// Mirrors: src/neo/fft/fft_test.cpp:53-130, rfft_test.cpp:40-126,
// src/neo/convolution/uniform_partitioned_convolver_test.cpp:35-75,
// fdl_index_test.cpp:7-68, uniform_partition_test.cpp:8-37.
#include <neo/convolution.hpp>
#include <neo/fft.hpp>

#include "../../oracle/neo_oracle.h"

#include <cmath>
#include <complex>
#include <algorithm>
#include <cstdio>
#include <iterator>
#include <vector>

static int failures = 0;
#define REQUIRE(cond)                                                          \
    do {                                                                       \
        if (!(cond)) {                                                         \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
            ++failures;                                                        \
        }                                                                      \
    } while (0)

using cf = std::complex<float>;

static std::vector<cf> cnoise(std::uint64_t seed, std::size_t n)
{
    std::vector<cf> v(n);
    oracle_noise(seed, reinterpret_cast<float*>(v.data()), 2 * n);
    return v;
}

static std::vector<float> rnoise(std::uint64_t seed, std::size_t n)
{
    std::vector<float> v(n);
    oracle_noise(seed, v.data(), n);
    return v;
}

template<typename A, typename B>
static double max_abs_diff(A const& a, B const& b)
{
    double m = 0;
    for (std::size_t i = 0; i < a.size(); ++i) m = std::max(m, double(std::abs(a[i] - b[i])));
    return m;
}

static void test_fft_plan()
{
    bool threw = false;
    try {
        neo::fft::fft_plan<cf> p{neo::fft::from_order, neo::fft::next_order(neo::fft::fft_plan<cf>::max_size() + 1U)};
    } catch (std::runtime_error const&) {
        threw = true;
    }
    REQUIRE(threw);  // fft_test.cpp:62-67
    for (std::size_t order = 2; order <= 14; ++order) {
        auto plan = neo::fft::fft_plan<cf>{neo::fft::from_order, order};
        REQUIRE(plan.order() == order);
        REQUIRE(plan.size() == neo::fft::size(order));
        REQUIRE(neo::fft::next_order(plan.size()) == plan.order());
        auto const noise = cnoise(order, plan.size());
        // inplace (fft_test.cpp:79-91)
        auto io = noise;
        auto v = neo::hip::make_view(io.data(), io.size());
        neo::fft::fft(plan, v);
        auto ref = noise;
        oracle_fft_c2c(int(order), -1, reinterpret_cast<float*>(ref.data()));
        double peak = 0;
        for (auto const& r : ref) peak = std::max(peak, double(std::abs(r)));
        REQUIRE(max_abs_diff(io, ref) / peak <= 1e-5);
        neo::fft::ifft(plan, v);
        for (auto& x : io) x *= 1.0F / float(plan.size());
        REQUIRE(max_abs_diff(io, noise) <= 1e-5);
        // copy (fft_test.cpp:93-110)
        std::vector<cf> tmp(plan.size()), out(plan.size());
        neo::fft::fft(plan, neo::hip::make_view(noise.data(), noise.size()), neo::hip::make_view(tmp.data(), tmp.size()));
        neo::fft::ifft(plan, neo::hip::make_view(tmp.data(), tmp.size()), neo::hip::make_view(out.data(), out.size()));
        for (auto& x : out) x *= 1.0F / float(plan.size());
        REQUIRE(max_abs_diff(out, noise) <= 1e-5);
        // inplace strided (fft_test.cpp:114-128): column 0 of a [2][N] layout_left buffer
        std::vector<cf> buf(2 * plan.size());
        auto col = neo::hip::make_strided_view(buf.data(), plan.size(), 2);
        for (std::size_t i = 0; i < plan.size(); ++i) col(i) = noise[i];
        neo::fft::fft(plan, col);
        neo::fft::ifft(plan, col);
        double m = 0;
        for (std::size_t i = 0; i < plan.size(); ++i) m = std::max(m, double(std::abs(col(i) / float(plan.size()) - noise[i])));
        REQUIRE(m <= 1e-5);
    }
}

static void test_rfft_plan()
{
    for (std::size_t order = 2; order <= 14; ++order) {
        auto rfft = neo::fft::rfft_plan<float>{neo::fft::from_order, order};
        REQUIRE(rfft.size() == neo::fft::size(order));
        auto signal = rnoise(100 + order, rfft.size());
        auto const original = signal;
        std::vector<cf> spectrum(rfft.size() / 2 + 1);
        neo::fft::rfft(rfft, neo::hip::make_view(signal.data(), signal.size()),
                       neo::hip::make_view(spectrum.data(), spectrum.size()));
        std::vector<cf> ref(rfft.size() / 2 + 1);
        oracle_rfft(int(order), original.data(), reinterpret_cast<float*>(ref.data()));
        double peak = 0;
        for (auto const& r : ref) peak = std::max(peak, double(std::abs(r)));
        REQUIRE(max_abs_diff(spectrum, ref) / peak <= 1e-5);
        neo::fft::irfft(rfft, neo::hip::make_view(spectrum.data(), spectrum.size()),
                        neo::hip::make_view(signal.data(), signal.size()));
        for (auto& x : signal) x *= 1.0F / float(rfft.size());
        REQUIRE(max_abs_diff(signal, original) <= 1e-5);  // rfft_test.cpp:40-71
    }
}

static void test_convolver_identity()
{
    for (std::size_t B : {128, 256, 512, 1024}) {
        std::vector<cf> filt(3 * (B + 1), cf{0, 0});
        for (std::size_t k = 0; k <= B; ++k) filt[k] = cf{1, 0};  // generate_identity_impulse
        auto const signal = rnoise(B, B * 20);
        auto output = signal;
        neo::convolution::upols_convolver<cf> conv;
        conv.filter(neo::hip::make_matrix_view(filt.data(), 3, B + 1));
        for (std::size_t i = 0; i < output.size(); i += B) conv(neo::hip::make_view(output.data() + i, B));
        REQUIRE(max_abs_diff(output, signal) <= 1e-5);
        output = signal;
        neo::convolution::upola_convolver<cf> upola;
        upola.filter(neo::hip::make_matrix_view(filt.data(), 3, B + 1));
        for (std::size_t i = 0; i < output.size(); i += B) upola(neo::hip::make_view(output.data() + i, B));
        REQUIRE(max_abs_diff(output, signal) <= 1e-5);
        neo::convolution::upola_convolver_v2<cf> v2;  // whole blocks, then uneven pieces
        output = signal;
        v2.filter(neo::hip::make_matrix_view(filt.data(), 3, B + 1));
        for (std::size_t i = 0; i < output.size(); i += B) v2(neo::hip::make_view(output.data() + i, B));
        REQUIRE(max_abs_diff(output, signal) <= 1e-5);
        output = signal;
        v2.filter(neo::hip::make_matrix_view(filt.data(), 3, B + 1));
        for (std::size_t i = 0, step = B / 3; i < output.size(); i += step, step = step * 2 % (3 * B) + 1)
            v2(neo::hip::make_view(output.data() + i, std::min(step, output.size() - i)));
        REQUIRE(max_abs_diff(output, signal) <= 1e-5);
        neo::convolution::split_upols_convolver<cf> split;
        output = signal;
        split.filter(neo::hip::make_matrix_view(filt.data(), 3, B + 1));
        for (std::size_t i = 0; i < output.size(); i += B) split(neo::hip::make_view(output.data() + i, B));
        REQUIRE(max_abs_diff(output, signal) <= 1e-5);
    }
}

static void test_dense_convolve_vs_oracle()
{
    std::size_t const C = 3, B = 256, L = 3000, N = B * 12 + 77;
    std::vector<float> ir(C * L), sig(C * N), out(C * N), ref(C * N);
    for (std::size_t c = 0; c < C; ++c) {
        auto a = rnoise(10 + c, L), b = rnoise(20 + c, N);
        std::copy(a.begin(), a.end(), ir.begin() + c * L);
        std::copy(b.begin(), b.end(), sig.begin() + c * N);
    }
    neo::convolution::dense_convolve(sig.data(), C, N, ir.data(), L, B, out.data());
    auto irn = ir;
    oracle_normalize_impulse(irn.data(), C, L);
    auto const P = oracle_num_partitions(L, B);
    REQUIRE(P == neo::convolution::num_partitions(L, B));
    std::vector<float> parts(C * P * (B + 1) * 2);
    oracle_uniform_partition(irn.data(), C, L, B, parts.data());
    oracle_dense_convolve(sig.data(), ref.data(), parts.data(), C, N, P, B, 1);
    double peak = 0;
    for (float r : ref) peak = std::max(peak, double(std::abs(r)));
    REQUIRE(max_abs_diff(out, ref) / peak <= 1e-5);
    // normalize_impulse (rank 2, bit-exact) and uniform_partition through the header API
    auto irh = ir;
    neo::convolution::normalize_impulse(neo::hip::make_matrix_view(irh.data(), C, L));
    REQUIRE(irh == irn);
    auto H = neo::convolution::uniform_partition(neo::hip::make_matrix_view(irn.data(), C, L), B);
    REQUIRE(H.extent(0) == C && H.extent(1) == P && H.extent(2) == B + 1);
    double hp = 0, hd = 0;
    for (std::size_t i = 0; i < H.size(); ++i) {
        cf const r{parts[2 * i], parts[2 * i + 1]};
        hp = std::max(hp, double(std::abs(r)));
        hd = std::max(hd, double(std::abs(H.buf[i] - r)));
    }
    REQUIRE(hd / hp <= 1e-5);
}

// upols_multidevice on the box's device listed twice equals upols_multichannel bit for bit
static void test_multidevice_equals_multichannel()
{
    std::size_t const C = 5, B = 128, L = 128 * 40, N = B * 20;
    std::vector<float> ir(C * L), sig(C * N);
    for (std::size_t c = 0; c < C; ++c) {
        auto a = rnoise(300 + c, L), b = rnoise(400 + c, N);
        std::copy(a.begin(), a.end(), ir.begin() + c * L);
        std::copy(b.begin(), b.end(), sig.begin() + c * N);
    }
    auto const P = neo::convolution::num_partitions(L, B);
    neo::convolution::upols_multidevice md{C, B, P, std::vector<int>{0, 0}};
    neo::convolution::upols_multichannel one{C, B, P};
    REQUIRE(md.shards() == 2);
    md.impulse(ir.data(), L);
    one.impulse(ir.data(), L);
    auto a = sig, b = sig;
    md.process(a.data(), N);
    one.process(b.data(), N);
    REQUIRE(a == b);
}

static void test_upola_v2_pieces_vs_oracle()
{
    // overlap_add_convolver::operator() with sub-block calls, against the restatement
    std::size_t const B = 256, L = 2000, N = B * 10;
    auto ir = rnoise(61, L);
    oracle_normalize_impulse(ir.data(), 1, L);
    auto const P = oracle_num_partitions(L, B);
    std::vector<float> parts(P * (B + 1) * 2);
    oracle_uniform_partition(ir.data(), 1, L, B, parts.data());
    auto const sig = rnoise(62, N);
    auto got = sig, ref = sig;
    neo::convolution::upola_convolver_v2<cf> conv;
    conv.filter(neo::hip::make_matrix_view(reinterpret_cast<cf*>(parts.data()), P, B + 1));
    auto* o = oracle_upola2_create(P, B + 1, parts.data());
    std::size_t const cuts[] = {0, 100, 100 + B, 3 * B + 7, 3 * B + 8, 6 * B, 7 * B + B / 2, N};
    for (std::size_t i = 0; i + 1 < std::size(cuts); ++i) {
        conv(neo::hip::make_view(got.data() + cuts[i], cuts[i + 1] - cuts[i]));
        oracle_upola2_process(o, ref.data() + cuts[i], cuts[i + 1] - cuts[i]);
    }
    oracle_upola2_destroy(o);
    double peak = 0;
    for (float r : ref) peak = std::max(peak, double(std::abs(r)));
    REQUIRE(max_abs_diff(got, ref) / peak <= 1e-5);
}

static void test_double_precision()
{
    // fft_plan<complex<double>> (the reference's complex<double> instantiation) vs the
    // double restatement; rfft_plan<double>; double one-shot convolutions
    using cd = std::complex<double>;
    for (int order : {0, 1, 5, 10, 12, 13, 16}) {
        std::size_t const n = std::size_t(1) << order;
        std::vector<cd> x(n);
        auto const re = rnoise(300 + order, n), im = rnoise(400 + order, n);
        for (std::size_t i = 0; i < n; ++i) x[i] = cd(re[i], im[i]);
        auto ref = x;
        oracle_fft_c2c_f64(order, -1, reinterpret_cast<double*>(ref.data()));
        auto got = x;
        neo::fft::fft_plan<cd> plan{neo::fft::from_order, std::size_t(order)};
        neo::fft::fft(plan, neo::hip::make_view(got.data(), n));
        double peak = 0;
        for (auto v : ref) peak = std::max(peak, std::abs(v));
        REQUIRE(max_abs_diff(got, ref) / peak <= 1e-12);
        neo::fft::ifft(plan, neo::hip::make_view(got.data(), n));
        for (auto& v : got) v /= double(n);
        REQUIRE(max_abs_diff(got, x) <= 1e-12);
    }
    {
        std::size_t const n = 1024;
        std::vector<double> r(n);
        auto const f = rnoise(500, n);
        for (std::size_t i = 0; i < n; ++i) r[i] = f[i];
        std::vector<cd> X(n / 2 + 1), ref(n / 2 + 1);
        oracle_rfft_f64(10, r.data(), reinterpret_cast<double*>(ref.data()));
        neo::fft::rfft_plan<double> rp{neo::fft::from_order, 10};
        neo::fft::rfft(rp, neo::hip::make_view(r.data(), n), neo::hip::make_view(X.data(), n / 2 + 1));
        REQUIRE(max_abs_diff(X, ref) <= 1e-11);
        std::vector<double> back(n);
        neo::fft::irfft(rp, neo::hip::make_view(X.data(), n / 2 + 1), neo::hip::make_view(back.data(), n));
        for (auto& v : back) v /= double(n);
        REQUIRE(max_abs_diff(back, r) <= 1e-13);
    }
    {
        std::vector<double> a(1000), b(333);
        auto const fa = rnoise(601, 1000), fb = rnoise(602, 333);
        std::copy(fa.begin(), fa.end(), a.begin());
        std::copy(fb.begin(), fb.end(), b.begin());
        auto const d = neo::convolution::direct_convolve(a.data(), a.size(), b.data(), b.size());
        auto const f = neo::convolution::fft_convolve(a.data(), a.size(), b.data(), b.size());
        std::vector<double> ref(1332);
        oracle_direct_convolve_f64(a.data(), a.size(), b.data(), b.size(), ref.data());
        REQUIRE(d == ref);  // same loop order, double rounding, no FMA: bit-identical
        REQUIRE(max_abs_diff(f, ref) <= 1e-12);
    }
}

static void test_stft()
{
    // stft_test.cpp:15-37 shapes, and values against the restatement (hann over N)
    for (std::size_t len : {2040, 2048}) {
        std::vector<float> x(len, 0.0F);
        auto const no_overlap = neo::fft::stft(neo::hip::make_matrix_view(x.data(), 1, len),
                                               neo::fft::stft_options<float>{256, 256, 0});
        REQUIRE(no_overlap.extent(0) == 1 && no_overlap.extent(1) == 8 && no_overlap.extent(2) == 129);
        auto const half = neo::fft::stft(neo::hip::make_matrix_view(x.data(), 1, len), 256);
        REQUIRE(half.extent(0) == 1 && half.extent(1) == 16 && half.extent(2) == 129);
    }
    auto const x = rnoise(71, 3000);
    auto const S = neo::fft::stft(neo::hip::make_matrix_view(x.data(), 1, 3000), 256);
    std::vector<float> w(256), ref(S.size() * 2);
    oracle_hann(256, w.data());
    oracle_stft(x.data(), 1, 3000, 256, 256, 128, w.data(), ref.data());
    double peak = 0, err = 0;
    for (std::size_t i = 0; i < S.size(); ++i) {
        cf const r{ref[2 * i], ref[2 * i + 1]};
        peak = std::max(peak, double(std::abs(r)));
        err = std::max(err, double(std::abs(S.buf[i] - r)));
    }
    REQUIRE(err / peak <= 1e-5);
}

static void test_one_shot_convolve()
{
    auto const x = rnoise(55, 1000), p = rnoise(56, 333);
    auto const f = neo::convolution::fft_convolve(x.data(), x.size(), p.data(), p.size());
    auto const d = neo::convolution::direct_convolve(x.data(), x.size(), p.data(), p.size());
    REQUIRE(f.size() == 1332 && d.size() == 1332);
    double peak = 0;
    for (float v : d) peak = std::max(peak, double(std::abs(v)));
    REQUIRE(max_abs_diff(f, d) / peak <= 1e-5);
    REQUIRE(neo::convolution::fft_convolve(x.data(), 0, p.data(), p.size()).empty());
}

static void test_fdl_index()
{
    // fdl_index_test.cpp:7-68
    auto indexer = neo::convolution::fdl_index<int>{3};
    std::vector<std::pair<int, int>> seen;
    indexer([](int i) { REQUIRE(i == 0); }, [&](int f, int g) { seen.emplace_back(f, g); });
    REQUIRE((seen == std::vector<std::pair<int, int>>{{0, 0}, {1, 2}, {2, 1}}));
    seen.clear();
    indexer([](int i) { REQUIRE(i == 1); }, [&](int f, int g) { seen.emplace_back(f, g); });
    REQUIRE((seen == std::vector<std::pair<int, int>>{{0, 1}, {1, 0}, {2, 2}}));
    indexer([](int i) { REQUIRE(i == 2); }, [](int, int) {});
    indexer([](int i) { REQUIRE(i == 0); }, [](int, int) {});
}

static void test_uniform_partition_shapes()
{
    for (auto [C, L] : std::vector<std::pair<std::size_t, std::size_t>>{{1, 4096}, {2, 4096}, {2, 4095}}) {
        std::vector<float> ir(C * L, 0.0F);
        auto H = neo::convolution::uniform_partition(neo::hip::make_matrix_view(ir.data(), C, L), 128);
        REQUIRE(H.extent(0) == C && H.extent(1) == 32 && H.extent(2) == 129);
    }
}

static_assert(neo::convolution::output_size<neo::convolution::mode::full>(1000, 333) == 1332);

static void test_rfftfreq()
{
    // extra/python/test/test.py:65-68 through the C++ header (host arithmetic)
    std::vector<double> f(2);
    neo::rfftfreq(neo::hip::make_view(f.data(), 2), 1.0 / 20.0);
    REQUIRE(f[0] == 0.0 && std::abs(f[1] - 10.0) < 1e-12);
    REQUIRE(std::abs(neo::rfftfreq<double>(2, 1, 1.0 / 44100.0) - 22050.0) < 1e-9);
}

// overlap_test.cpp:21-64 (no-op callback, B x F sizes) and a filter callback against the
// restatement (oracle_overlap_stage), overlap_save and overlap_add
template<typename Stage, int Kind>
static void test_overlap_stage()
{
    for (std::size_t B : {128U, 512U}) {
        for (std::size_t F : {8U, 9U, 10U, 17U, 127U, 128U, 129U, 130U, 512U, 999U, 1024U}) {
            Stage stage{B, F};
            REQUIRE(stage.block_size() == B && stage.filter_size() == F);
            REQUIRE(stage.transform_size() >= B + F - 1);
            auto const sig = rnoise(F, B * 8);
            auto out = sig;
            for (std::size_t i = 0; i < out.size(); i += B) {
                stage(neo::hip::make_view(out.data() + i, B),
                      [&](auto io) { REQUIRE(std::size_t(io.extent(0)) == stage.transform_size() / 2 + 1); });
            }
            REQUIRE(max_abs_diff(out, sig) <= 1e-5);
        }
    }
    std::size_t const B = 128, F = 129;
    Stage stage{B, F};
    auto G = cnoise(91, stage.transform_size() / 2 + 1);
    auto x = rnoise(92, B * 10);
    auto ref = x;
    REQUIRE(oracle_overlap_stage(Kind, B, F, reinterpret_cast<float const*>(G.data()), ref.data(), 10) == 0);
    for (std::size_t i = 0; i < x.size(); i += B) {
        stage(neo::hip::make_view(x.data() + i, B), [&](auto io) {
            for (std::size_t k = 0; k < std::size_t(io.extent(0)); ++k) io(k) *= G[k];
        });
    }
    double peak = 0;
    for (float v : ref) peak = std::max(peak, double(std::abs(v)));
    REQUIRE(max_abs_diff(x, ref) <= 1e-5 * peak);
}

// the latency mode (one resident kernel, synchronous calls) through the single-channel drop-in
// at the reference benchmark's shape (B = 512, 2 s IR: P = 188), against the oracle's dense
// convolution of the same blocks; the multichannel object's paced step groups against the unpaced
static void test_latency_mode_and_paced()
{
    std::size_t const B = 512, L = 96000, nb = 300;
    auto ir = rnoise(31, L);
    oracle_normalize_impulse(ir.data(), 1, L);
    auto const P = std::size_t(oracle_num_partitions(L, B));
    std::vector<float> parts(P * (B + 1) * 2);
    oracle_uniform_partition(ir.data(), 1, L, B, parts.data());
    auto const signal = rnoise(32, B * nb);
    std::vector<float> ref(signal.size());
    oracle_dense_convolve(signal.data(), ref.data(), parts.data(), 1, signal.size(), P, B, 1);
    neo::convolution::upols_convolver<cf> conv;
    conv.latency_mode(true);
    conv.filter(neo::hip::make_matrix_view(reinterpret_cast<cf*>(parts.data()), P, B + 1));
    auto out = signal;
    for (std::size_t i = 0; i < out.size(); i += B) conv(neo::hip::make_view(out.data() + i, B));
    double peak = 0;
    for (float r : ref) peak = std::max(peak, double(std::abs(r)));
    REQUIRE(max_abs_diff(out, ref) <= 1e-5 * peak);
    // step groups (128 channels x B = 512), paced vs not: the same kernels, bit for bit
    std::size_t const C = 128, P2 = 100, n2 = 40;
    std::vector<cf> h2(C * P2 * (B + 1));
    for (std::size_t i = 0; i < h2.size(); ++i)
        h2[i] = cf{float((i * 7919) % 1000) * 1e-4f, float((i * 104729) % 1000) * 1e-4f};
    neo::convolution::upols_multichannel a{C, B, P2}, b{C, B, P2};
    a.filter(h2.data());
    b.filter(h2.data());
    a.paced(true);
    bool same = true;
    for (std::size_t f = 0; f < n2; ++f) {
        auto xa = rnoise(40 + f, C * B), xb = xa;
        a(xa.data());
        b(xb.data());
        same = same && xa == xb;
    }
    REQUIRE(same);
}

int main()
{
    test_fdl_index();
    test_rfftfreq();
    int n = 0;
    if (neo_hip_device_count(&n) != NEO_HIP_OK || n < 1) {
        std::printf("no GPU: only host-side checks ran\n");
        return failures ? 1 : 0;
    }
    test_fft_plan();
    test_rfft_plan();
    test_convolver_identity();
    test_dense_convolve_vs_oracle();
    test_uniform_partition_shapes();
    test_one_shot_convolve();
    test_upola_v2_pieces_vs_oracle();
    test_multidevice_equals_multichannel();
    test_double_precision();
    test_stft();
    test_overlap_stage<neo::convolution::overlap_save<cf>, 0>();
    test_overlap_stage<neo::convolution::overlap_add<cf>, 1>();
    test_latency_mode_and_paced();
    std::printf(failures ? "FAILED (%d)\n" : "all C++ API tests passed\n", failures);
    return failures ? 1 : 0;
}
