// fft_device_real.hpp — packed real<->complex FFT steps (gfx950).
//
// A 2M-point real transform runs as an M-point complex FFT of
// z[n] = x[2n] + i x[2n+1] plus one O(M) "split" step, instead of the
// reference's full 2M-point complex FFT of zero-imaginary data
// (src/neo/fft/fallback/fallback_rfft_plan.hpp:27-55; the reference states the
// same packing trick in src/neo/fft/experimental/rfft.hpp:138-207). Results are
// the same bins up to rounding.
//
// "Packed" spectra (the UPOLS device layout) hold M complex values per row with
// the two purely-real bins folded into bin 0: X[0] = {DC, Nyquist}.
#pragma once

#include "fft_device.hpp"

namespace neo_hip {

// Forward split: Z = FFT_M(z) in `zl` (natural order, lpad'ed). Returns X[k]
// for k in [0, M); X[0] is packed {DC, Nyquist}. tw2 = twiddle table of size 2M.
// w = the forward twiddle e^{-i pi k / M} (twiddle<2M, -1>(tw2, k)), given by the caller
template<int M, class C>
__device__ __forceinline__ C r2c_split_w(const C* zl, C w, int k)
{
    using R = real_of<C>;
    const C zk = zl[lpad(k)];
    if (k == 0) return {zk.x + zk.y, zk.x - zk.y};
    const C zc = cconj(zl[lpad(M - k)]);
    const C fe = cscale(cadd(zk, zc), R(0.5));
    const C d = csub(zk, zc);
    const C fo = {R(0.5) * d.y, R(-0.5) * d.x};  // -i/2 * (zk - zc)
    return cadd(fe, cmul(w, fo));
}

template<int M, class C>
__device__ __forceinline__ C r2c_split(const C* zl, const C* tw2, int k)
{
    return r2c_split_w<M>(zl, k == 0 ? C{1, 0} : twiddle<2 * M, -1>(tw2, k), k);
}

// Inverse split: from X[k] and X[M-k] (k in [0, M)) build Z[k] such that
// IFFT_M(Z) (unnormalized) = z with x[2n] = Re z[n], x[2n+1] = Im z[n] equal to
// the unnormalized 2M-point inverse (fallback_rfft_plan.hpp:38-55: Hermitian
// fill, backward c2c, real part; imaginary parts of DC/Nyquist ignored).
// xk = X[k], xmk = X[M-k] for k > 0; for k == 0 pass dc/nyq in xk.x / xmk.x.
// w = the inverse twiddle e^{+i pi k / M} (twiddle<2M, +1>(tw2, k)), given by the caller
template<int M, class C>
__device__ __forceinline__ C c2r_join_w(C xk, C xmk, C w, int k)
{
    C a, b;  // a = X[k], b = conj(X[M-k])
    if (k == 0) {
        a = {xk.x, 0};
        b = {xmk.x, 0};
    } else {
        a = xk;
        b = cconj(xmk);
    }
    const C fe = cadd(a, b);
    const C fo = cmul(csub(a, b), w);
    return {fe.x - fo.y, fe.y + fo.x};  // fe + i*fo
}

template<int M, class C>
__device__ __forceinline__ C c2r_join(C xk, C xmk, const C* tw2, int k)
{
    return c2r_join_w<M>(xk, xmk, twiddle<2 * M, +1>(tw2, k), k);
}

}  // namespace neo_hip
