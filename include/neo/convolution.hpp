// SPDX-License-Identifier: MIT
// neo/convolution.hpp — neo::convolution UPOLS API on MI355X (gfx950).
//
// Same names and semantics as the reference's src/neo/convolution/*:
//   fdl_index                 fdl_index.hpp:12-41 (host ring bookkeeping)
//   uniform_partition         uniform_partition.hpp:12-26  -> [C][P][B+1] complex<float>
//   normalize_impulse         normalize_impulse.hpp:11-33  (bit-exact rounding on the GPU)
//   upols_convolver           dense_convolver.hpp:19-20 + uniform_partitioned_convolver.hpp:13-65
//   split_upols_convolver     dense_convolver.hpp:38-42 (same math; one device layout)
//   upola_convolver(_v2)      dense_convolver.hpp:23-28 (overlap_add / overlap_add_convolver)
// plus the GPU-shaped entry the plugin and CLI loops map onto: upols_multichannel,
// C channels stepped by one launch pair per block ([C][B] in, [C][P][B+1] filter),
// and dense_convolve (extra/plugin/src/dsp/DenseConvolution.hpp:39-70).
#pragma once

#include <neo/fft.hpp>
#include <neo/hip/detail.hpp>

#include <algorithm>
#include <complex>
#include <concepts>
#include <cstddef>
#include <memory>
#include <stdexcept>
#include <map>
#include <mutex>
#include <array>
#include <utility>
#include <vector>

namespace neo::convolution {

/// method.hpp:8-17
enum struct method
{
    automatic,
    direct,
    fft,
    ola,
    ols,
    upola,
    upols,
};

/// mode.hpp:12-29 (only `full` has an output size, like the reference)
enum struct mode
{
    full,
    valid,
    same,
};

template<mode Mode, std::integral Int>
[[nodiscard]] constexpr auto output_size(Int signal, Int patch) -> Int
{
    static_assert(Mode == mode::full, "the reference defines output_size for mode::full only");
    return static_cast<Int>(signal + patch - Int(1));
}

/// fdl_index.hpp:12-41 — insert(write_pos), then for segment s: multiply(s, (write_pos + P - s) % P)
template<typename IndexType = std::size_t>
struct fdl_index {
    using value_type = IndexType;

    fdl_index() noexcept = default;
    explicit fdl_index(IndexType num_segments) : _num_segments{num_segments} {}

    auto reset() -> void { _write_pos = 0; }

    template<std::invocable<IndexType> CopyCallback, std::invocable<IndexType, IndexType> MultiplyCallback>
    auto operator()(CopyCallback copy_callback, MultiplyCallback callback) -> void
    {
        copy_callback(_write_pos);
        for (IndexType segment{0}; segment < _num_segments; ++segment) {
            callback(segment, static_cast<IndexType>((_write_pos + _num_segments - segment) % _num_segments));
        }
        if (++_write_pos; _write_pos >= _num_segments) reset();
    }

private:
    IndexType _num_segments{0};
    IndexType _write_pos{0};
};

/// P = ceil(L / B) (stft.hpp:21-25, overlap 0)
[[nodiscard]] inline auto num_partitions(std::size_t length, std::size_t block) -> std::size_t
{
    std::int64_t p = 0;
    neo::hip::check(neo_hip_num_partitions(std::int64_t(length), int(block), &p));
    return std::size_t(p);
}

/// uniform_partition.hpp:12-26: impulse [C][L] -> [C][P][B+1] (computed on the GPU)
template<typename InMat>
    requires neo::hip::detail::matrix_like<InMat>
[[nodiscard]] auto uniform_partition(InMat impulse_response, std::size_t block_size)
    -> neo::hip::array<std::complex<float>, 3>
{
    auto const C = std::size_t(impulse_response.extent(0)), L = std::size_t(impulse_response.extent(1));
    std::vector<float> ir(C * L);
    for (std::size_t c = 0; c < C; ++c)
        for (std::size_t i = 0; i < L; ++i) ir[c * L + i] = float(neo::hip::detail::at(impulse_response, c, i));
    auto const P = num_partitions(L, block_size);
    neo::hip::array<std::complex<float>, 3> out;
    out.buf.resize(C * P * (block_size + 1));
    out.ext[0] = C;
    out.ext[1] = P;
    out.ext[2] = block_size + 1;
    neo::hip::check(neo_hip_uniform_partition(ir.data(), int(C), std::int64_t(L), int(block_size), out.data(), 0,
                                              neo::hip::detail::default_device()));
    return out;
}

/// normalize_impulse.hpp:11-33 (rank 1: unit energy; rank 2: min factor over channels)
template<typename Obj>
auto normalize_impulse(Obj obj) noexcept -> void
{
    std::size_t C = 1, L = 0;
    if constexpr (neo::hip::detail::matrix_like<Obj>) {
        C = std::size_t(obj.extent(0));
        L = std::size_t(obj.extent(1));
    } else {
        L = std::size_t(obj.extent(0));
    }
    if (C == 0 || L == 0) return;
    std::vector<float> buf(C * L);
    for (std::size_t c = 0; c < C; ++c)
        for (std::size_t i = 0; i < L; ++i) {
            if constexpr (neo::hip::detail::matrix_like<Obj>) buf[c * L + i] = neo::hip::detail::at(obj, c, i);
            else buf[i] = neo::hip::detail::at(obj, i);
        }
    neo::hip::check_or_abort(neo_hip_normalize_impulse(buf.data(), int(C), std::int64_t(L), 0,
                                                       neo::hip::detail::default_device()));
    for (std::size_t c = 0; c < C; ++c)
        for (std::size_t i = 0; i < L; ++i) {
            if constexpr (neo::hip::detail::matrix_like<Obj>) neo::hip::detail::at(obj, c, i) = buf[c * L + i];
            else neo::hip::detail::at(obj, i) = buf[i];
        }
}

/// selects upola_convolver_v2 (overlap_add_convolver.hpp:20-136) in upols_multichannel
struct upola_v2_tag {};
inline constexpr upola_v2_tag upola_v2{};

namespace detail {
struct upols_deleter {
    void operator()(neo_hip_upols* h) const noexcept { neo_hip_upols_destroy(h); }
};
using upols_ptr = std::unique_ptr<neo_hip_upols, upols_deleter>;
}  // namespace detail

/// C independent uniformly-partitioned convolvers (UPOLS, or UPOLA with method::upola)
/// on one GPU, stepped together.
struct upols_multichannel {
    upols_multichannel(std::size_t channels, std::size_t block_size, std::size_t partitions,
                       int device = neo::hip::detail::default_device(), method m = method::upols)
        : _C{channels}, _B{block_size}, _P{partitions}
    {
        if (m != method::upols && m != method::upola)
            throw std::invalid_argument{"neo_hip: multichannel convolver supports method::upols and method::upola"};
        neo_hip_upols* h = nullptr;
        auto create = m == method::upols ? neo_hip_upols_create : neo_hip_upola_create;
        neo::hip::check(create(int(channels), int(block_size), int(partitions), device, &h));
        _h.reset(h);
    }

    /// C instances of upola_convolver_v2 (sub-block input through process())
    upols_multichannel(upola_v2_tag, std::size_t channels, std::size_t block_size, std::size_t partitions,
                       int device = neo::hip::detail::default_device())
        : _C{channels}, _B{block_size}, _P{partitions}
    {
        neo_hip_upols* h = nullptr;
        neo::hip::check(neo_hip_upola2_create(int(channels), int(block_size), int(partitions), device, &h));
        _h.reset(h);
    }

    /// filter [C][P][B+1] complex<float>, contiguous host memory; resets state
    auto filter(std::complex<float> const* partitions) -> void
    {
        neo::hip::check(neo_hip_upols_set_filter(_h.get(), partitions, 0));
    }
    /// normalize_impulse (optional) + uniform_partition of ir [C][length] on the GPU
    auto impulse(float const* ir, std::size_t length, bool normalize = true) -> void
    {
        neo::hip::check(neo_hip_upols_set_impulse(_h.get(), ir, std::int64_t(length), normalize ? 1 : 0, 0));
    }
    /// one block for every channel, in place, io [C][B] host memory (synchronous)
    auto operator()(float* io) noexcept -> void { neo::hip::check_or_abort(neo_hip_upols_process(_h.get(), io, 0, nullptr)); }
    /// one block, device pointers, channel c at in + c*ld_in (asynchronous on stream)
    auto process_device(float const* in, std::size_t ld_in, float* out, std::size_t ld_out, void* stream = nullptr) -> void
    {
        neo::hip::check(neo_hip_upols_process_device(_h.get(), in, std::int64_t(ld_in), out, std::int64_t(ld_out), stream));
    }
    /// num_samples per channel, in place, io [C][num_samples] host memory (synchronous);
    /// any count for upola_v2, whole blocks otherwise (overlap_add_convolver.hpp:80-134)
    auto process(float* io, std::size_t num_samples) noexcept -> void
    {
        auto const n = std::int64_t(num_samples);
        neo::hip::check_or_abort(neo_hip_upols_process_samples(_h.get(), io, n, io, n, n, 0, nullptr));
    }
    auto reset() -> void { neo::hip::check(neo_hip_upols_reset(_h.get())); }
    /// latency mode (neo_hip_upols_set_persistent): one resident kernel steps every block; every
    /// call completes on return (shapes up to 16 channels, 256 partitions, B <= 512; throws otherwise)
    auto latency_mode(bool on, double idle_ms = 50.0) -> void
    {
        neo::hip::check(neo_hip_upols_set_persistent(_h.get(), on ? 1 : 0, idle_ms));
    }
    /// paced background work (neo_hip_upols_set_paced): an even cost per call with step groups
    auto paced(bool on) -> void { neo::hip::check(neo_hip_upols_set_paced(_h.get(), on ? 1 : 0)); }
    /// the same with the group's background launch in two pieces (two cross-stream waits per group)
    auto paced_two_pieces() -> void { neo::hip::check(neo_hip_upols_set_paced(_h.get(), 2)); }
    /// offline windows for batched calls of >= 128 blocks (on by default from 128 partitions;
    /// neo_hip_upols_set_offline): 128-block windows through partition-axis transforms
    auto offline(bool on) -> void { neo::hip::check(neo_hip_upols_set_offline(_h.get(), on ? 1 : 0)); }

    [[nodiscard]] auto channels() const noexcept { return _C; }
    [[nodiscard]] auto block_size() const noexcept { return _B; }
    [[nodiscard]] auto partitions() const noexcept { return _P; }

private:
    std::size_t _C, _B, _P;
    detail::upols_ptr _h;
};

namespace detail {
struct upols_multi_deleter {
    void operator()(neo_hip_upols_multi* m) const noexcept { neo_hip_upols_multi_destroy(m); }
};
}  // namespace detail

/// upols_multichannel over several devices of one node (neo_hip_upols_multi_*): channel
/// shard i = [C i / n, C (i + 1) / n) on devices[i] (a device may repeat), no collective
/// (channels are independent, DenseConvolution.hpp:35,50-67); every call runs the shards
/// concurrently. Results equal one upols_multichannel over all channels bit for bit.
struct upols_multidevice {
    upols_multidevice(std::size_t channels, std::size_t block_size, std::size_t partitions,
                      std::vector<int> const& devices, method m = method::upols)
        : _C{channels}, _B{block_size}, _P{partitions}
    {
        int const mi = m == method::upols ? 0 : m == method::upola ? 1 : -1;
        if (mi < 0) throw std::invalid_argument{"neo_hip: multidevice convolver supports method::upols and method::upola"};
        neo_hip_upols_multi* h = nullptr;
        neo::hip::check(neo_hip_upols_multi_create(int(channels), int(block_size), int(partitions), devices.data(),
                                                   int(devices.size()), mi, nullptr, &h));
        _h.reset(h);
    }

    /// filter [C][P][B+1] complex<float>, contiguous host memory; resets state
    auto filter(std::complex<float> const* partitions) -> void
    {
        neo::hip::check(neo_hip_upols_multi_set_filter(_h.get(), partitions));
    }
    /// normalize_impulse over all channels (optional) + uniform_partition of ir [C][length]
    auto impulse(float const* ir, std::size_t length, bool normalize = true) -> void
    {
        neo::hip::check(neo_hip_upols_multi_set_impulse(_h.get(), ir, std::int64_t(length), normalize ? 1 : 0));
    }
    /// num_samples (whole blocks) per channel, in place, io [C][num_samples] host memory
    auto process(float* io, std::size_t num_samples) -> void
    {
        auto const n = std::int64_t(num_samples);
        neo::hip::check(neo_hip_upols_multi_process_samples(_h.get(), io, n, io, n, n));
    }
    auto reset() -> void { neo::hip::check(neo_hip_upols_multi_reset(_h.get())); }
    [[nodiscard]] auto shards() const -> int
    {
        int n = 0;
        neo::hip::check(neo_hip_upols_multi_shards(_h.get(), &n));
        return n;
    }

    [[nodiscard]] auto channels() const noexcept { return _C; }
    [[nodiscard]] auto block_size() const noexcept { return _B; }
    [[nodiscard]] auto partitions() const noexcept { return _P; }

private:
    std::size_t _C, _B, _P;
    std::unique_ptr<neo_hip_upols_multi, detail::upols_multi_deleter> _h;
};

/// Single-channel drop-in for upols_convolver<complex<float>> (uniform_partitioned_convolver.hpp:13-65)
/// and, with M = method::upola, upola_convolver: default-constructible; filter([P][B+1])
/// (re)initializes everything; operator()(block[B]) in place.
template<typename Complex, method M = method::upols>
struct hip_upols_convolver {
    static_assert(std::same_as<Complex, std::complex<float>>);
    using value_type = Complex;
    using accumulator_type = neo::hip::array<Complex, 1>;

    hip_upols_convolver() = default;

    template<typename InMat>
        requires neo::hip::detail::matrix_like<InMat>
    auto filter(InMat filter) -> void
    {
        auto const P = std::size_t(filter.extent(0)), bins = std::size_t(filter.extent(1));
        std::vector<Complex> h(P * bins);
        for (std::size_t p = 0; p < P; ++p)
            for (std::size_t k = 0; k < bins; ++k) h[p * bins + k] = Complex(neo::hip::detail::at(filter, p, k));
        if (!_impl || _impl->partitions() != P || _impl->block_size() != bins - 1) {
            _impl = std::make_unique<upols_multichannel>(1, bins - 1, P, neo::hip::detail::default_device(), M);
            if (_latency) _impl->latency_mode(true, _idle_ms);
        }
        _impl->filter(h.data());
        _block.resize(bins - 1);
    }

    /// latency mode for this instance (upols_multichannel::latency_mode), kept across filter()
    /// calls; applied at the next filter() when no filter was set yet
    auto latency_mode(bool on, double idle_ms = 50.0) -> void
    {
        _latency = on;
        _idle_ms = idle_ms;
        if (_impl) _impl->latency_mode(on, idle_ms);
    }

    template<typename Vec>
        requires neo::hip::detail::vector_like<Vec>
    auto operator()(Vec block) -> void
    {
        if (neo::hip::detail::contiguous(block)) {
            (*_impl)(block.data_handle());
            return;
        }
        neo::hip::detail::gather(block, _block.data());
        (*_impl)(_block.data());
        neo::hip::detail::scatter(_block.data(), block);
    }

private:
    std::unique_ptr<upols_multichannel> _impl;
    std::vector<float> _block;
    bool _latency = false;
    double _idle_ms = 50.0;
};

/// Single-channel drop-in for upola_convolver_v2<complex<float>> (dense_convolver.hpp:28,
/// overlap_add_convolver.hpp:20-136): operator()(samples) takes any number of samples.
template<typename Complex>
struct hip_upola2_convolver {
    static_assert(std::same_as<Complex, std::complex<float>>);
    using value_type = Complex;
    using accumulator_type = neo::hip::array<Complex, 1>;

    hip_upola2_convolver() = default;

    template<typename InMat>
        requires neo::hip::detail::matrix_like<InMat>
    auto filter(InMat filter) -> void
    {
        auto const P = std::size_t(filter.extent(0)), bins = std::size_t(filter.extent(1));
        std::vector<Complex> h(P * bins);
        for (std::size_t p = 0; p < P; ++p)
            for (std::size_t k = 0; k < bins; ++k) h[p * bins + k] = Complex(neo::hip::detail::at(filter, p, k));
        if (!_impl || _impl->partitions() != P || _impl->block_size() != bins - 1)
            _impl = std::make_unique<upols_multichannel>(upola_v2, 1, bins - 1, P);
        _impl->filter(h.data());
    }

    template<typename Vec>
        requires neo::hip::detail::vector_like<Vec>
    auto operator()(Vec inout) -> void
    {
        auto const n = std::size_t(inout.extent(0));
        if (neo::hip::detail::contiguous(inout)) {
            _impl->process(inout.data_handle(), n);
            return;
        }
        _buf.resize(n);
        neo::hip::detail::gather(inout, _buf.data());
        _impl->process(_buf.data(), n);
        neo::hip::detail::scatter(_buf.data(), inout);
    }

private:
    std::unique_ptr<upols_multichannel> _impl;
    std::vector<float> _buf;
};

namespace detail {
struct group_deleter {
    void operator()(neo_hip_upols_group* g) const noexcept { neo_hip_upols_group_destroy(g); }
};
}  // namespace detail

/// The convolvers of ONE owner (one plugin instance: DenseConvolution's
/// std::vector<upols_convolver>, DenseConvolution.hpp:35), grouped per shape
/// (neo_hip_upols_group_*): grouped_upols_convolver instances whose filter() runs inside a
/// scope() of this object join its group of their shape; instances outside any scope run alone.
/// register_buffer() names host memory the owner keeps allocated (its frame buffer) until
/// unregister_all(): only convolvers called on such buffers are stepped together.
class convolver_group {
public:
    convolver_group() = default;
    convolver_group(convolver_group const&) = delete;
    auto operator=(convolver_group const&) -> convolver_group& = delete;

    /// RAII: convolvers whose filter() runs on this thread while the scope lives join `g`
    class scope_guard {
    public:
        explicit scope_guard(convolver_group& g) noexcept : _prev{current()} { current() = &g; }
        ~scope_guard() { current() = _prev; }
        scope_guard(scope_guard const&) = delete;
        auto operator=(scope_guard const&) -> scope_guard& = delete;

    private:
        convolver_group* _prev;
    };
    [[nodiscard]] auto scope() -> scope_guard { return scope_guard{*this}; }

    /// what the owner promises about a registered frame buffer (neo_hip_upols_group_register_ex)
    enum class frame : int {
        plain = 0,                           ///< allocated until unregister_all(): exact comparison per member
        stable = NEO_HIP_GROUP_FRAME_STABLE,  ///< + written by nothing but the convolvers' calls during a frame
        in_place = NEO_HIP_GROUP_FRAME_STABLE | NEO_HIP_GROUP_FRAME_INPLACE,  ///< + read only through them, each
                                                                              ///< on the same block: outputs in place
    };
    /// [ptr, ptr + samples) stays allocated until unregister_all() (cheap to repeat per frame), with
    /// the owner's promise about it during a frame (the plugin's loop over a filled frame keeps
    /// frame::in_place; frame::stable skips the members' snapshot comparison)
    auto register_buffer(float const* ptr, std::size_t samples, frame promise = frame::plain) -> void
    {
        std::lock_guard<std::mutex> lk{_mu};
        auto const flags = int(promise);
        bool found = false;
        for (auto& r : _ranges)
            if (r.ptr == ptr && r.samples == samples) {
                r.flags = flags;
                found = true;
            }
        if (!found) _ranges.push_back({ptr, samples, flags});
        for (auto& [key, g] : _groups)
            neo::hip::check(neo_hip_upols_group_register_ex(g.get(), ptr, std::int64_t(samples * sizeof(float)), flags));
    }
    /// before the registered memory is freed or reallocated (e.g. at prepare())
    auto unregister_all() -> void
    {
        std::lock_guard<std::mutex> lk{_mu};
        _ranges.clear();
        for (auto& [key, g] : _groups) neo::hip::check(neo_hip_upols_group_unregister(g.get(), nullptr));
    }

    /// the group of one shape (created on first use, with the ranges registered so far)
    auto acquire(std::size_t block, std::size_t partitions, method m, int device) -> std::shared_ptr<neo_hip_upols_group>
    {
        std::lock_guard<std::mutex> lk{_mu};
        auto const key = std::array<std::size_t, 4>{block, partitions, std::size_t(m == method::upola), std::size_t(device)};
        if (auto it = _groups.find(key); it != _groups.end()) return it->second;
        auto g = make_group(block, partitions, m, device);
        for (auto const& r : _ranges)
            neo::hip::check(
                neo_hip_upols_group_register_ex(g.get(), r.ptr, std::int64_t(r.samples * sizeof(float)), r.flags));
        _groups.emplace(key, g);
        return g;
    }

    static auto make_group(std::size_t block, std::size_t partitions, method m, int device)
        -> std::shared_ptr<neo_hip_upols_group>
    {
        neo_hip_upols_group* raw = nullptr;
        neo::hip::check(
            neo_hip_upols_group_create(int(block), int(partitions), m == method::upola ? 1 : 0, device, &raw));
        return std::shared_ptr<neo_hip_upols_group>(raw, detail::group_deleter{});
    }

    /// the group scope active on this thread, or null
    static auto current() noexcept -> convolver_group*&
    {
        thread_local convolver_group* cur = nullptr;
        return cur;
    }

private:
    std::mutex _mu;
    std::map<std::array<std::size_t, 4>, std::shared_ptr<neo_hip_upols_group>> _groups;
    struct range {
        float const* ptr;
        std::size_t samples;
        int flags;
    };
    std::vector<range> _ranges;
};

/// Single-channel drop-in for upols_convolver<complex<float>> (uniform_partitioned_convolver.hpp:13-65)
/// that joins the convolver_group whose scope() is active when its filter() runs (else it runs
/// alone): in the plugin's frame pattern (DenseConvolution.cpp:62-74: every instance called once
/// per frame on a buffer of its own, inside the owner's registered frame buffer) a frame of all
/// instances is ONE launch instead of one launch and one wait per instance; each instance's
/// outputs are its own sequential convolver's in any pattern. upols_convolver / upola_convolver
/// are this type when NEO_HIP_CONVOLVER_GROUPS is defined (the split_* forms are not: the
/// plugin's Convolution.hpp:61 runs them on the host's own output buffer).
template<typename Complex, method M = method::upols>
struct grouped_upols_convolver {
    static_assert(std::same_as<Complex, std::complex<float>>);
    using value_type = Complex;
    using accumulator_type = neo::hip::array<Complex, 1>;

    grouped_upols_convolver() = default;
    grouped_upols_convolver(grouped_upols_convolver&& o) noexcept
        : _g{std::move(o._g)}, _owner{o._owner}, _id{std::exchange(o._id, -1)}, _B{o._B}, _P{o._P},
          _block{std::move(o._block)}
    {}
    auto operator=(grouped_upols_convolver&& o) noexcept -> grouped_upols_convolver&
    {
        if (this != &o) {
            leave();
            _g = std::move(o._g);
            _owner = o._owner;
            _id = std::exchange(o._id, -1);
            _B = o._B;
            _P = o._P;
            _block = std::move(o._block);
        }
        return *this;
    }
    ~grouped_upols_convolver() { leave(); }

    template<typename InMat>
        requires neo::hip::detail::matrix_like<InMat>
    auto filter(InMat filter) -> void
    {
        auto const P = std::size_t(filter.extent(0)), bins = std::size_t(filter.extent(1));
        std::vector<Complex> h(P * bins);
        for (std::size_t p = 0; p < P; ++p)
            for (std::size_t k = 0; k < bins; ++k) h[p * bins + k] = Complex(neo::hip::detail::at(filter, p, k));
        auto* owner = convolver_group::current();
        if (!_g || _P != P || _B != bins - 1 || owner != _owner) {
            leave();
            auto const dev = neo::hip::detail::default_device();
            _g = owner ? owner->acquire(bins - 1, P, M, dev) : convolver_group::make_group(bins - 1, P, M, dev);
            _owner = owner;
            neo::hip::check(neo_hip_upols_group_join(_g.get(), &_id));
            _B = bins - 1;
            _P = P;
            _block.resize(_B);
        }
        neo::hip::check(neo_hip_upols_group_set_filter(_g.get(), _id, h.data(), 0));
    }

    template<typename Vec>
        requires neo::hip::detail::vector_like<Vec>
    auto operator()(Vec block) -> void
    {
        if (neo::hip::detail::contiguous(block)) {
            neo::hip::check_or_abort(neo_hip_upols_group_process(_g.get(), _id, block.data_handle()));
            return;
        }
        neo::hip::detail::gather(block, _block.data());
        neo::hip::check_or_abort(neo_hip_upols_group_process(_g.get(), _id, _block.data()));
        neo::hip::detail::scatter(_block.data(), block);
    }

    /// the group this instance belongs to (diagnostics: neo_hip_upols_group_stats)
    [[nodiscard]] auto group() const noexcept -> neo_hip_upols_group* { return _g.get(); }

private:
    void leave() noexcept
    {
        if (_g && _id >= 0) (void)neo_hip_upols_group_leave(_g.get(), _id);
        _g.reset();
        _owner = nullptr;
        _id = -1;
    }

    std::shared_ptr<neo_hip_upols_group> _g;
    convolver_group* _owner = nullptr;
    int _id = -1;
    std::size_t _B = 0, _P = 0;
    std::vector<float> _block;
};

namespace detail {
struct overlap_deleter {
    void operator()(neo_hip_overlap* h) const noexcept { neo_hip_overlap_destroy(h); }
};

/// overlap_save / overlap_add (overlap_save.hpp:19-112, overlap_add.hpp:23-107) on the GPU:
/// ctor(block_size, filter_size), transform size 2^next_order(B + F - 1); operator()(block,
/// callback) runs the window update and rfft on the device, hands the callback the
/// transform_size() / 2 + 1 bins (a host view it may modify in place), then the irfft, 1/n and
/// the output block, in place.
template<typename Complex, int Kind>
struct hip_overlap {
    static_assert(std::same_as<Complex, std::complex<float>>);
    using value_type = Complex;
    using complex_type = Complex;
    using real_type = typename Complex::value_type;
    using size_type = std::size_t;

    hip_overlap(size_type block_size, size_type filter_size)
    {
        neo_hip_overlap* h = nullptr;
        neo::hip::check(neo_hip_overlap_create(Kind, 1, std::int64_t(block_size), std::int64_t(filter_size),
                                               neo::hip::detail::default_device(), &h));
        _h.reset(h);
        std::int64_t b = 0, f = 0, n = 0;
        neo::hip::check(neo_hip_overlap_info(h, &b, &f, &n));
        _block = size_type(b);
        _filter = size_type(f);
        _n = size_type(n);
        _bins.resize(_n / 2 + 1);
        _buf.resize(_block);
    }

    [[nodiscard]] auto block_size() const noexcept -> size_type { return _block; }
    [[nodiscard]] auto filter_size() const noexcept -> size_type { return _filter; }
    [[nodiscard]] auto transform_size() const noexcept -> size_type { return _n; }

    template<typename Vec, typename Callback>
        requires neo::hip::detail::vector_like<Vec>
    auto operator()(Vec block, Callback callback) -> void
    {
        float* io = _buf.data();
        bool const direct = neo::hip::detail::contiguous(block) && std::size_t(block.extent(0)) == _block;
        if (direct) io = block.data_handle();
        else neo::hip::detail::gather(block, _buf.data());
        neo::hip::check_or_abort(neo_hip_overlap_forward(_h.get(), io, std::int64_t(_block), _bins.data(), 0, nullptr));
        callback(neo::hip::make_view(_bins.data(), _bins.size()));
        neo::hip::check_or_abort(neo_hip_overlap_inverse(_h.get(), _bins.data(), io, std::int64_t(_block), 0, nullptr));
        if (!direct) neo::hip::detail::scatter(_buf.data(), block);
    }

private:
    std::unique_ptr<neo_hip_overlap, overlap_deleter> _h;
    size_type _block{}, _filter{}, _n{};
    std::vector<Complex> _bins;
    std::vector<float> _buf;
};
}  // namespace detail

template<typename Complex>
using overlap_save = detail::hip_overlap<Complex, 0>;

template<typename Complex>
using overlap_add = detail::hip_overlap<Complex, 1>;

#ifdef NEO_HIP_CONVOLVER_GROUPS
template<typename Complex>
using upols_convolver = grouped_upols_convolver<Complex>;

template<typename Complex>
using split_upols_convolver = hip_upols_convolver<Complex>;

/// dense_convolver.hpp:23-24, 32-35 (overlap-add stage, same FDL MAC)
template<typename Complex>
using upola_convolver = grouped_upols_convolver<Complex, method::upola>;

template<typename Complex>
using split_upola_convolver = hip_upols_convolver<Complex, method::upola>;
#else
template<typename Complex>
using upols_convolver = hip_upols_convolver<Complex>;

template<typename Complex>
using split_upols_convolver = hip_upols_convolver<Complex>;

/// dense_convolver.hpp:23-24, 32-35 (overlap-add stage, same FDL MAC)
template<typename Complex>
using upola_convolver = hip_upols_convolver<Complex, method::upola>;

template<typename Complex>
using split_upola_convolver = hip_upols_convolver<Complex, method::upola>;
#endif

/// dense_convolver.hpp:28
template<typename Complex>
using upola_convolver_v2 = hip_upola2_convolver<Complex>;

/// dense_convolve<upols_convolver> (DenseConvolution.hpp:39-70) over plain arrays:
/// signal [C][N], ir [C][L] -> out [C][N]; normalizes + partitions the IR, tail block zero-padded.
inline auto dense_convolve(float const* signal, std::size_t channels, std::size_t num_samples, float const* ir,
                           std::size_t ir_length, std::size_t block_size, float* out, method m = method::upols) -> void
{
    upols_multichannel conv{channels, block_size, num_partitions(ir_length, block_size),
                            neo::hip::detail::default_device(), m};
    conv.impulse(ir, ir_length, true);
    // whole signal in chunks of <= 2^26 samples: one upload, batched passes over the
    // filter and FDL, one download per chunk; the tail block is zero-padded
    std::size_t const nb = (num_samples + block_size - 1) / block_size;
    std::size_t chunk = std::max<std::size_t>(1, (std::size_t(1) << 26) / (channels * block_size));
    chunk = std::max<std::size_t>(256, chunk / 256 * 256);  // whole offline passes (two windows of 128 blocks)
    std::vector<float> buf;
    for (std::size_t t0 = 0; t0 < nb; t0 += chunk) {
        std::size_t const t1 = std::min(nb, t0 + chunk), lo = t0 * block_size,
                          hi = std::min(num_samples, t1 * block_size), n = (t1 - t0) * block_size;
        buf.assign(channels * n, 0.0F);
        for (std::size_t c = 0; c < channels; ++c)
            std::copy(signal + c * num_samples + lo, signal + c * num_samples + hi, buf.data() + c * n);
        conv.process(buf.data(), n);
        for (std::size_t c = 0; c < channels; ++c)
            std::copy(buf.data() + c * n, buf.data() + c * n + (hi - lo), out + c * num_samples + lo);
    }
}

/// fft_convolve (fft_convolver.hpp:72-93): full linear convolution on the GPU, host arrays
/// (float or double, like the reference's Python overloads, main.cpp:255-258)
template<typename Float>
    requires(std::same_as<Float, float> || std::same_as<Float, double>)
inline auto fft_convolve(Float const* signal, std::size_t n, Float const* patch, std::size_t m) -> std::vector<Float>
{
    if (n == 0 || m == 0) return {};
    std::vector<Float> out(n + m - 1);
    auto const f = [] {
        if constexpr (std::same_as<Float, double>) return neo_hip_fft_convolve_f64;
        else return neo_hip_fft_convolve;
    }();
    neo::hip::check(f(signal, std::int64_t(n), patch, std::int64_t(m), out.data(), 0, neo::hip::detail::default_device()));
    return out;
}

/// direct_convolve (direct_convolve.hpp:58-68): same loop order and rounding as the reference
template<typename Float>
    requires(std::same_as<Float, float> || std::same_as<Float, double>)
inline auto direct_convolve(Float const* signal, std::size_t n, Float const* patch, std::size_t m)
    -> std::vector<Float>
{
    if (n == 0 || m == 0) return {};
    std::vector<Float> out(n + m - 1);
    auto const f = [] {
        if constexpr (std::same_as<Float, double>) return neo_hip_direct_convolve_f64;
        else return neo_hip_direct_convolve;
    }();
    neo::hip::check(f(signal, std::int64_t(n), patch, std::int64_t(m), out.data(), 0, neo::hip::detail::default_device()));
    return out;
}

}  // namespace neo::convolution
