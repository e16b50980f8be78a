/*
 * neo_oracle_f64.c — CPU restatement of the double-precision side of the path:
 * fft_plan<complex<double>> (c2c_dit2_plan), rfft_plan<double> (fallback_rfft_plan),
 * fft_convolve<double> and direct_convolve<double>, as bound by the reference's
 * Python module for complex128 / float64 arrays (extra/python/src/main.cpp:248-258).
 *
 * TEST INFRASTRUCTURE ONLY (see neo_oracle.c). Same algorithm as the float restatement
 * with Float = double: twiddle angles computed in double (twiddle.hpp:17-29), table
 * bit-reverse, radix-2 DIT v3, full-complex r2c / Hermitian-fill c2r, unnormalized.
 * Pinned by float64 numpy (pocketfft) and np.convolve truth in tests/test_oracle.py.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_MAX_ORDER 27

/* twiddle.hpp:17-29 with Float = double: angle = sign * (pi*2) * index / size */
static void twiddle_d(size_t size, size_t index, int dir, double* re, double* im)
{
    const double sign = dir < 0 ? -1.0 : 1.0;
    const double two_pi = 3.14159265358979323846 * 2.0;
    const double angle = sign * two_pi * (double)index / (double)size;
    *re = cos(angle);
    *im = sin(angle);
}

static uint32_t bitrev_u32(uint32_t i, int order)
{
    uint32_t r = 0;
    for (int j = 0; j < order; ++j) r |= ((i >> j) & 1u) << (order - 1 - j);
    return r;
}

/* bitrevorder.hpp:19-32 then c2c_dit2.hpp:122-168 (v3), in place */
int oracle_fft_c2c_f64(int order, int dir, double* x)
{
    if (order < 0 || order > ORACLE_MAX_ORDER) return -1;
    if (order == 0) return 0;
    const size_t n = (size_t)1 << order;
    double* tw = (double*)malloc(sizeof(double) * n); /* n/2 complex */
    if (!tw) return -2;
    for (size_t i = 0; i < n / 2; ++i) twiddle_d(n, i, dir, &tw[2 * i], &tw[2 * i + 1]);
    for (uint32_t i = 0; i < (uint32_t)n; ++i) {
        const uint32_t j = bitrev_u32(i, order);
        if (i < j) {
            double t0 = x[2 * i], t1 = x[2 * i + 1];
            x[2 * i] = x[2 * j]; x[2 * i + 1] = x[2 * j + 1];
            x[2 * j] = t0;       x[2 * j + 1] = t1;
        }
    }
    for (size_t k = 0; k < n; k += 2) {
        const double ar = x[2 * k], ai = x[2 * k + 1], br = x[2 * k + 2], bi = x[2 * k + 3];
        x[2 * k] = ar + br;     x[2 * k + 1] = ai + bi;
        x[2 * k + 2] = ar - br; x[2 * k + 3] = ai - bi;
    }
    for (int stage = 1; stage < order; ++stage) {
        const size_t len = (size_t)1 << stage, stride = len * 2, tws = (size_t)1 << (order - stage - 1);
        for (size_t k = 0; k < n; k += stride) {
            for (size_t p = 0; p < len; ++p) {
                const double wr = tw[2 * (p * tws)], wi = tw[2 * (p * tws) + 1];
                const size_t i1 = k + p, i2 = k + p + len;
                const double xr = x[2 * i2], xi = x[2 * i2 + 1];
                const double tr = wr * xr - wi * xi, ti = wr * xi + wi * xr;
                const double ar = x[2 * i1], ai = x[2 * i1 + 1];
                x[2 * i1] = ar + tr; x[2 * i1 + 1] = ai + ti;
                x[2 * i2] = ar - tr; x[2 * i2 + 1] = ai - ti;
            }
        }
    }
    free(tw);
    return 0;
}

/* fallback_rfft_plan.hpp:27-36 */
int oracle_rfft_f64(int order, const double* in, double* out /* n/2+1 complex */)
{
    const size_t n = (size_t)1 << order;
    double* buf = (double*)calloc(2 * n, sizeof(double));
    if (!buf) return -2;
    for (size_t i = 0; i < n; ++i) buf[2 * i] = in[i];
    int rc = oracle_fft_c2c_f64(order, -1, buf);
    if (rc == 0) memcpy(out, buf, sizeof(double) * 2 * (n / 2 + 1));
    free(buf);
    return rc;
}

/* fallback_rfft_plan.hpp:38-55: Hermitian fill, backward c2c, real part, no 1/n */
int oracle_irfft_f64(int order, const double* in, double* out)
{
    const size_t n = (size_t)1 << order, coeffs = n / 2 + 1;
    double* buf = (double*)calloc(2 * n, sizeof(double));
    if (!buf) return -2;
    memcpy(buf, in, sizeof(double) * 2 * coeffs);
    for (size_t i = coeffs; i < n; ++i) {
        buf[2 * i] = buf[2 * (n - i)];
        buf[2 * i + 1] = -buf[2 * (n - i) + 1];
    }
    int rc = oracle_fft_c2c_f64(order, +1, buf);
    if (rc == 0) for (size_t i = 0; i < n; ++i) out[i] = buf[2 * i];
    free(buf);
    return rc;
}

/* fft_convolver.hpp:19-93 with Float = double */
int oracle_fft_convolve_f64(const double* signal, size_t n, const double* patch, size_t m, double* out)
{
    if (n == 0 || m == 0) return 0;
    const size_t len = n + m - 1;
    int order = 0;
    while (((size_t)1 << order) < len) ++order;
    const size_t N = (size_t)1 << order, bins = N / 2 + 1;
    double* tmp = (double*)calloc(N, sizeof(double));
    double* a = (double*)malloc(sizeof(double) * 2 * bins);
    double* b = (double*)malloc(sizeof(double) * 2 * bins);
    memcpy(tmp, signal, sizeof(double) * n);
    int rc = oracle_rfft_f64(order, tmp, a);
    memset(tmp, 0, sizeof(double) * N);
    memcpy(tmp, patch, sizeof(double) * m);
    if (!rc) rc = oracle_rfft_f64(order, tmp, b);
    if (!rc) {
        for (size_t k = 0; k < bins; ++k) {
            const double xr = a[2 * k], xi = a[2 * k + 1], yr = b[2 * k], yi = b[2 * k + 1];
            a[2 * k] = xr * yr - xi * yi;
            a[2 * k + 1] = xr * yi + xi * yr;
        }
        rc = oracle_irfft_f64(order, a, tmp);
    }
    if (!rc) {
        const double scale = 1.0 / (double)N;
        for (size_t i = 0; i < len; ++i) out[i] = tmp[i] * scale;
    }
    free(tmp); free(a); free(b);
    return rc;
}

/* direct_convolve.hpp:14-56 with Float = double: same loop order, double accumulation */
void oracle_direct_convolve_f64(const double* signal, size_t n, const double* patch, size_t l, double* out)
{
    const size_t mm = n + l - 1;
    const double* a = signal;
    const double* b = patch;
    size_t na = n, nb = l;
    if (n < l) { a = patch; b = signal; na = l; nb = n; }
    size_t i = 0;
    for (size_t k = 0; k < nb; ++k) {
        out[k] = 0.0;
        for (size_t m = 0; m <= k; ++m) out[k] += a[m] * b[k - m];
    }
    for (size_t k = nb; k < mm; ++k) {
        out[k] = 0.0;
        ++i;
        const size_t t1 = nb + i, tmin = t1 < na ? t1 : na;
        for (size_t m = i; m < tmin; ++m) out[k] += a[m] * b[k - m];
    }
}
