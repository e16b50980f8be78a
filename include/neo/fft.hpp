// SPDX-License-Identifier: MIT
// neo/fft.hpp — neo::fft API on MI355X (gfx950).
//
// Same names, argument meaning and error behaviour as the reference's
// src/neo/fft/{fft,rfft,direction,order}.hpp: fft_plan<Complex> (reference alias
// chain fft.hpp:36-52, default c2c_dit2_plan.hpp:21-104) and rfft_plan<Float,
// Complex> (rfft.hpp:15-23, fallback_rfft_plan.hpp:14-61) become HIP plans that
// call libneo_hip.so through the C-ABI in neo_hip.h. Transforms are unnormalized,
// forward = -1. Plans throw std::runtime_error at construction for order >
// max_order() = 27; operator() is noexcept and aborts on a device failure.
// Host views are staged through the plan's device buffers; the batched device
// entry points take device pointers and a hipStream_t (as void*).
#pragma once

#include <neo/hip/detail.hpp>

#include <bit>
#include <cmath>
#include <complex>
#include <concepts>
#include <cstddef>
#include <memory>
#include <stdexcept>
#include <string>
#include <functional>
#include <type_traits>
#include <vector>

namespace neo::fft {

/// src/neo/fft/direction.hpp:8-12
enum struct direction : int
{
    forward = -1,
    backward = 1,
};

/// src/neo/fft/order.hpp:17-24
struct from_order_tag {
    explicit from_order_tag() = default;
};
inline constexpr auto from_order = from_order_tag{};

/// 2^order (order.hpp:26-30)
template<std::integral Int>
[[nodiscard]] constexpr auto size(Int order) noexcept -> Int
{
    return Int(1) << order;
}

/// log2(bit_ceil(size)) (order.hpp:32-37)
template<std::integral Int>
[[nodiscard]] constexpr auto next_order(Int sz) noexcept -> Int
{
    auto const u = static_cast<std::make_unsigned_t<Int>>(sz);
    return static_cast<Int>(std::bit_width(std::bit_ceil(u)) - 1);
}

namespace detail {
struct plan_deleter {
    void operator()(neo_hip_fft_plan* p) const noexcept { neo_hip_fft_plan_destroy(p); }
};
using plan_ptr = std::unique_ptr<neo_hip_fft_plan, plan_deleter>;

inline plan_ptr make_plan(int order, std::int64_t batch, int kind, int device)
{
    neo_hip_fft_plan* p = nullptr;
    neo::hip::check(neo_hip_fft_plan_create(order, batch, kind, device, &p));
    return plan_ptr{p};
}
}  // namespace detail

/// Batched complex-to-complex plan on one GPU (replaces c2c_dit2_plan).
template<typename Complex>
struct hip_fft_plan {
    static_assert(std::same_as<Complex, std::complex<float>> || std::same_as<Complex, std::complex<double>>,
                  "the MI355X path transforms complex<float> or complex<double>");
    using value_type = Complex;
    using size_type = std::size_t;
    static constexpr int kind = NEO_HIP_C2C | (std::same_as<Complex, std::complex<double>> ? NEO_HIP_F64 : 0);

    hip_fft_plan(from_order_tag /*tag*/, size_type order, int device = neo::hip::detail::default_device())
        : _order{check_order(order)}, _device{device}, _plan{detail::make_plan(int(order), 1, kind, device)}
    {}

    [[nodiscard]] static constexpr auto max_order() noexcept -> size_type { return 27; }
    [[nodiscard]] static constexpr auto max_size() noexcept -> size_type { return fft::size(max_order()); }
    [[nodiscard]] auto order() const noexcept -> size_type { return _order; }
    [[nodiscard]] auto size() const noexcept -> size_type { return fft::size(_order); }

    /// in place, unnormalized (c2c_dit2_plan.hpp:81-95); any layout (strided views are staged)
    template<typename Vec>
        requires neo::hip::detail::vector_like<Vec>
    auto operator()(Vec x, direction dir) noexcept -> void
    {
        if (neo::hip::detail::contiguous(x)) {
            auto* p = x.data_handle();
            neo::hip::check_or_abort(neo_hip_fft_execute_host(_plan.get(), p, p, int(dir)));
            return;
        }
        _tmp.resize(size());
        neo::hip::detail::gather(x, _tmp.data());
        neo::hip::check_or_abort(neo_hip_fft_execute_host(_plan.get(), _tmp.data(), _tmp.data(), int(dir)));
        neo::hip::detail::scatter(_tmp.data(), x);
    }

    /// out of place (fft.hpp:62-71 uses it when the plan provides it)
    template<typename InVec, typename OutVec>
        requires neo::hip::detail::vector_like<InVec> && neo::hip::detail::vector_like<OutVec>
    auto operator()(InVec in, OutVec out, direction dir) noexcept -> void
    {
        if (neo::hip::detail::contiguous(in) && neo::hip::detail::contiguous(out)) {
            neo::hip::check_or_abort(neo_hip_fft_execute_host(_plan.get(), in.data_handle(), out.data_handle(), int(dir)));
            return;
        }
        _tmp.resize(size());
        neo::hip::detail::gather(in, _tmp.data());
        neo::hip::check_or_abort(neo_hip_fft_execute_host(_plan.get(), _tmp.data(), _tmp.data(), int(dir)));
        neo::hip::detail::scatter(_tmp.data(), out);
    }

    /// batched device entry: `batch` contiguous transforms, device pointers, hipStream_t as void*
    auto execute_device(Complex const* in, Complex* out, std::size_t batch, direction dir, void* stream = nullptr) -> void
    {
        if (batch != _batch) {
            _batched = detail::make_plan(int(_order), std::int64_t(batch), kind, _device);
            _batch = batch;
        }
        neo::hip::check(neo_hip_fft_execute(_batched.get(), in, out, int(dir), stream));
    }

private:
    static auto check_order(size_type order) -> size_type
    {
        if (order > max_order()) throw std::runtime_error{"neo_hip: unsupported order '" + std::to_string(order) + "'"};
        return order;
    }

    size_type _order;
    int _device;
    detail::plan_ptr _plan;
    detail::plan_ptr _batched;
    std::size_t _batch = 0;
    std::vector<Complex> _tmp;
};

/// The drop-in alias point (reference fft.hpp:36-52 `#if` chain; NEO_HAS_HIP).
template<typename Complex>
using fft_plan = hip_fft_plan<Complex>;

/// fft.hpp:54-90
template<typename Plan, typename Vec>
constexpr auto fft(Plan& plan, Vec inout) -> void
{
    plan(inout, direction::forward);
}

template<typename Plan, typename InVec, typename OutVec>
constexpr auto fft(Plan& plan, InVec input, OutVec output) -> void
{
    plan(input, output, direction::forward);
}

template<typename Plan, typename Vec>
constexpr auto ifft(Plan& plan, Vec inout) -> void
{
    plan(inout, direction::backward);
}

template<typename Plan, typename InVec, typename OutVec>
constexpr auto ifft(Plan& plan, InVec input, OutVec output) -> void
{
    plan(input, output, direction::backward);
}

/// Real <-> complex plan (replaces fallback_rfft_plan): r2c writes N/2+1 bins,
/// c2r reads N/2+1 bins (Im of DC/Nyquist ignored), unnormalized.
template<typename Float, typename Complex = std::complex<Float>>
struct hip_rfft_plan {
    static_assert((std::same_as<Float, float> || std::same_as<Float, double>) &&
                  std::same_as<Complex, std::complex<Float>>);
    using real_type = Float;
    using complex_type = Complex;
    using size_type = std::size_t;
    static constexpr int f64 = std::same_as<Float, double> ? NEO_HIP_F64 : 0;

    hip_rfft_plan(from_order_tag /*tag*/, size_type order, int device = neo::hip::detail::default_device())
        : _order{order},
          _r2c{detail::make_plan(int(order), 1, NEO_HIP_R2C | f64, device)},
          _c2r{detail::make_plan(int(order), 1, NEO_HIP_C2R | f64, device)}
    {}

    [[nodiscard]] auto order() const noexcept -> size_type { return _order; }
    [[nodiscard]] auto size() const noexcept -> size_type { return fft::size(_order); }

    /// r2c: N reals -> N/2+1 bins (fallback_rfft_plan.hpp:27-36)
    template<typename InVec, typename OutVec>
        requires std::floating_point<typename InVec::value_type>
    auto operator()(InVec in, OutVec out) noexcept -> void
    {
        _re.resize(size());
        _cx.resize(size() / 2 + 1);
        neo::hip::detail::gather(in, _re.data());
        neo::hip::check_or_abort(neo_hip_fft_execute_host(_r2c.get(), _re.data(), _cx.data(), -1));
        for (std::size_t i = 0; i < size() / 2 + 1; ++i) neo::hip::detail::at(out, i) = _cx[i];
    }

    /// c2r: >= N/2+1 bins -> N reals (fallback_rfft_plan.hpp:38-55)
    template<typename InVec, typename OutVec>
        requires(!std::floating_point<typename InVec::value_type>)
    auto operator()(InVec in, OutVec out) noexcept -> void
    {
        _re.resize(size());
        _cx.resize(size() / 2 + 1);
        for (std::size_t i = 0; i < size() / 2 + 1; ++i) _cx[i] = Complex(neo::hip::detail::at(in, i));
        neo::hip::check_or_abort(neo_hip_fft_execute_host(_c2r.get(), _cx.data(), _re.data(), +1));
        neo::hip::detail::scatter(_re.data(), out);
    }

private:
    size_type _order;
    detail::plan_ptr _r2c, _c2r;
    std::vector<Float> _re;
    std::vector<Complex> _cx;
};

template<typename Float, typename Complex = std::complex<Float>>
using rfft_plan = hip_rfft_plan<Float, Complex>;

/// rfft.hpp:25-39
template<typename Plan, typename InVec, typename OutVec>
constexpr auto rfft(Plan& plan, InVec input, OutVec output)
{
    return plan(input, output);
}

template<typename Plan, typename InVec, typename OutVec>
constexpr auto irfft(Plan& plan, InVec input, OutVec output)
{
    return plan(input, output);
}

} // namespace neo::fft

namespace neo {
/// rfftfreq.hpp:12-30 (host index arithmetic): bin i of a size-n transform
template<std::floating_point T>
[[nodiscard]] constexpr auto rfftfreq(std::integral auto size, std::integral auto index, double inv_sample_rate) -> T
{
    auto const fs = T(1) / static_cast<T>(inv_sample_rate);
    auto const inv_size = T(1) / static_cast<T>(size);
    return static_cast<T>(index) * fs * inv_size;
}

template<typename Vec>
constexpr auto rfftfreq(Vec vec, double inv_sample_rate) noexcept -> void
{
    auto const size = static_cast<int>(vec.extent(0));
    for (int i = 0; i < size; ++i)
        neo::hip::detail::at(vec, i) =
            rfftfreq<std::remove_cvref_t<decltype(neo::hip::detail::at(vec, i))>>(size, i, inv_sample_rate);
}
}  // namespace neo

namespace neo::fft {

/// norm.hpp (Python scaling modes)
enum struct norm
{
    backward,
    ortho,
    forward,
};

/// stft.hpp:30-37
template<std::floating_point Float>
struct stft_options {
    std::size_t frame_size{};
    std::size_t transform_size{};
    std::size_t overlap_size{};
    std::function<Float(std::size_t, std::size_t)> window{[](std::size_t i, std::size_t n) {
        // hann_window (math/windowing.hpp:29-41)
        auto const two_pi = static_cast<Float>(3.14159265358979323846) * Float(2);
        return Float(0.5) * (Float(1) - std::cos(two_pi * static_cast<Float>(i) / static_cast<Float>(n - 1)));
    }};
};

/// stft_plan (stft.hpp:40-109): x [C][L] -> [C][F][N/2+1] on the GPU (framing + batched r2c)
template<std::floating_point Float, typename Complex = std::complex<Float>>
struct stft_plan {
    static_assert(std::same_as<Float, float> || std::same_as<Float, double>);

    explicit stft_plan(std::size_t transform_size)
        : stft_plan(stft_options<Float>{transform_size, transform_size, transform_size / 2})
    {}

    explicit stft_plan(stft_options<Float> options) : _options{std::move(options)}
    {
        auto const n = fft::size(fft::next_order(_options.transform_size));
        _window.resize(n);
        for (std::size_t i = 0; i < n; ++i) _window[i] = _options.window(i, n);  // fill_window
    }

    template<typename InMat>
        requires neo::hip::detail::matrix_like<InMat>
    [[nodiscard]] auto operator()(InMat x) -> neo::hip::array<Complex, 3>
    {
        auto const C = std::size_t(x.extent(0)), L = std::size_t(x.extent(1));
        std::vector<Float> buf(C * L);
        for (std::size_t c = 0; c < C; ++c)
            for (std::size_t i = 0; i < L; ++i) buf[c * L + i] = Float(neo::hip::detail::at(x, c, i));
        std::int64_t frames = 0;
        neo::hip::check(neo_hip_stft_num_frames(std::int64_t(L), int(_options.frame_size), int(_options.overlap_size),
                                                &frames));
        neo::hip::array<Complex, 3> out;
        out.ext[0] = C;
        out.ext[1] = std::size_t(frames);
        out.ext[2] = _window.size() / 2 + 1;
        out.buf.resize(out.ext[0] * out.ext[1] * out.ext[2]);
        auto const f = [] {
            if constexpr (std::same_as<Float, double>) return neo_hip_stft_f64;
            else return neo_hip_stft;
        }();
        neo::hip::check(f(buf.data(), int(C), std::int64_t(L), int(_options.frame_size),
                          int(_options.transform_size), int(_options.overlap_size), _window.data(), out.data(), 0,
                          neo::hip::detail::default_device()));
        return out;
    }

private:
    stft_options<Float> _options;
    std::vector<Float> _window;
};

/// stft.hpp:111-125
template<typename InMat>
[[nodiscard]] auto stft(InMat x, stft_options<std::remove_cvref_t<decltype(neo::hip::detail::at(x, 0, 0))>> options)
{
    using Float = std::remove_cvref_t<decltype(neo::hip::detail::at(x, 0, 0))>;
    return stft_plan<Float>{std::move(options)}(x);
}

template<typename InMat>
[[nodiscard]] auto stft(InMat x, std::size_t window_size)
{
    using Float = std::remove_cvref_t<decltype(neo::hip::detail::at(x, 0, 0))>;
    return stft_plan<Float>{window_size}(x);
}

/// rfft.hpp:41-62: split the c2c spectrum of a + ib into rfft(a), rfft(b) (host utility)
template<typename InVec, typename OutVecX, typename OutVecY>
auto rfft_deinterleave(InVec dft, OutVecX x, OutVecY y) -> void
{
    using Complex = typename InVec::value_type;
    using Float = typename Complex::value_type;
    auto const n = static_cast<std::size_t>(dft.extent(0));
    auto const i = Complex{Float(0), Float(-1)};
    using neo::hip::detail::at;
    at(x, 0) = Complex(at(dft, 0).real(), Float(0));
    at(y, 0) = Complex(at(dft, 0).imag(), Float(0));
    for (std::size_t k = 1; k < n / 2 + 1; ++k) {
        Complex const zk = at(dft, k);
        Complex const znk = std::conj(Complex(at(dft, n - k)));
        at(x, k) = (zk + znk) * Float(0.5);
        at(y, k) = ((zk - znk) * i) * Float(0.5);
    }
}

}  // namespace neo::fft
