// SPDX-License-Identifier: MIT
// neo/hip/detail.hpp — plumbing shared by the neo::fft / neo::convolution headers:
// RAII over the C-ABI handles, status -> exception/abort mapping, and access to
// mdspan-like views (Kokkos stdex::mdspan in the reference, or neo::hip::view).
#pragma once

#include <neo_hip.h>

#include <array>
#include <complex>
#include <concepts>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace neo::hip {

// Throwing check (construction / setup paths: the reference throws std::runtime_error,
// src/neo/fft/reference/c2c_dit2_plan.hpp:97-104).
inline void check(int rc)
{
    if (rc != NEO_HIP_OK) throw std::runtime_error(std::string{"neo_hip: "} + neo_hip_last_error());
}

// Execution paths are noexcept in the reference (c2c_dit2_plan.hpp:81-95,
// uniform_partitioned_convolver.hpp:47-65): a device failure there is fatal.
inline void check_or_abort(int rc) noexcept
{
    if (rc != NEO_HIP_OK) {
        std::fprintf(stderr, "neo_hip fatal: %s\n", neo_hip_last_error());
        std::abort();
    }
}

// Minimal owning/non-owning views with the mdspan surface the API needs
// (extent, stride, data_handle, operator()). Kokkos mdspan satisfies the same
// concepts, so the headers accept either.
template<typename T>
struct view1d {
    using value_type = std::remove_cv_t<T>;
    using element_type = T;
    using index_type = std::size_t;
    T* ptr = nullptr;
    std::size_t n = 0, s = 1;
    static constexpr std::size_t rank() { return 1; }
    std::size_t extent(std::size_t) const { return n; }
    std::size_t stride(std::size_t) const { return s; }
    std::size_t size() const { return n; }
    T* data_handle() const { return ptr; }
    T& operator()(std::size_t i) const { return ptr[i * s]; }
    T& operator[](std::size_t i) const { return ptr[i * s]; }
};

template<typename T>
struct view2d {
    using value_type = std::remove_cv_t<T>;
    using element_type = T;
    using index_type = std::size_t;
    T* ptr = nullptr;
    std::size_t n0 = 0, n1 = 0, s0 = 0, s1 = 1;
    static constexpr std::size_t rank() { return 2; }
    std::size_t extent(std::size_t r) const { return r == 0 ? n0 : n1; }
    std::size_t stride(std::size_t r) const { return r == 0 ? s0 : s1; }
    T* data_handle() const { return ptr; }
    T& operator()(std::size_t i, std::size_t j) const { return ptr[i * s0 + j * s1]; }
};

template<typename T>
view1d<T> make_view(T* p, std::size_t n)
{
    return {p, n, 1};
}

template<typename T>
view1d<T> make_strided_view(T* p, std::size_t n, std::size_t stride)
{
    return {p, n, stride};
}

template<typename T>
view2d<T> make_matrix_view(T* p, std::size_t rows, std::size_t cols)
{
    return {p, rows, cols, cols, 1};
}

// Owning row-major array (stands in for stdex::mdarray in the return types).
template<typename T, std::size_t Rank>
struct array {
    std::vector<T> buf;
    std::size_t ext[Rank]{};
    std::size_t extent(std::size_t r) const { return ext[r]; }
    std::size_t size() const { return buf.size(); }
    T* data() { return buf.data(); }
    const T* data() const { return buf.data(); }
    template<typename... I>
    T& operator()(I... idx)
    {
        std::size_t ids[] = {std::size_t(idx)...}, off = 0;
        for (std::size_t r = 0; r < Rank; ++r) off = off * ext[r] + ids[r];
        return buf[off];
    }
    auto to_mdspan()
    {
        if constexpr (Rank == 1) return view1d<T>{buf.data(), ext[0], 1};
        else if constexpr (Rank == 2) return view2d<T>{buf.data(), ext[0], ext[1], ext[1], 1};
        else return buf.data();
    }
};

namespace detail {

template<typename V>
concept vector_like = requires(V v) {
    v.extent(0);
    v.stride(0);
    v.data_handle();
};

template<typename V>
concept matrix_like = vector_like<V> && requires(V v) {
    v.extent(1);
    v.stride(1);
};

template<typename V>
decltype(auto) at(V const& v, std::size_t i)
{
    if constexpr (requires { v(i); }) return v(i);
    else return v[i];
}

template<typename V>
decltype(auto) at(V const& v, std::size_t i, std::size_t j)
{
    if constexpr (requires { v(i, j); }) return v(i, j);
    else return v[std::array<std::size_t, 2>{i, j}];  // C++20 mdspan array indexing
}

template<typename V>
bool contiguous(V const& v)
{
    return v.extent(0) <= 1 || v.stride(0) == 1;
}

// copy a vector view into contiguous storage (any layout) and back
template<typename T, typename V>
void gather(V const& v, T* dst)
{
    for (std::size_t i = 0; i < std::size_t(v.extent(0)); ++i) dst[i] = T(at(v, i));
}

template<typename T, typename V>
void scatter(T const* src, V const& v)
{
    for (std::size_t i = 0; i < std::size_t(v.extent(0)); ++i) at(v, i) = src[i];
}

inline int default_device()
{
    if (char const* e = std::getenv("NEO_HIP_DEVICE")) return std::atoi(e);
    return 0;
}

}  // namespace detail
}  // namespace neo::hip
