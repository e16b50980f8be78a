/* neo_baseline.c — the reference's SIMD CPU path for dense_convolve<upols_convolver>, restated
 * for bench.py's cpu_baseline (TEST / MEASUREMENT INFRASTRUCTURE ONLY: never linked by the
 * product; the parity oracle stays the exact scalar restatement in neo_oracle.c).
 *
 * The reference's Linux CI builds with -march=native and NEO_ENABLE_XSIMD=ON
 * (/root/reference/.github/workflows/build.yml:34, CMakeLists.txt:11). On an AVX-512 host
 * the split AVX path is compiled out (multiply_add.hpp:149: "not defined AVX512F") and the
 * interleaved FDL MAC of dense_filter is the xsimd loop (multiply_add.hpp:196-223):
 *   out[i:i+n] = x[i:i+n] * y[i:i+n] + z[i:i+n] as xsimd::batch<std::complex<float>>
 * i.e. unaligned loads that deinterleave each operand into a real and an imaginary vector,
 * elementwise complex multiply-add, reinterleaving stores; a scalar tail. xsimd
 * (a third-party dependency, not in /root/reference) is restated here with intrinsics:
 * AVX-512F (16 complex per batch) or AVX2 + FMA (8), picked at run time
 * (__builtin_cpu_supports), scalar otherwise. The per-block flow is that of
 * uniform_partitioned_convolver.hpp:47-65 with overlap_save.hpp:84-112: slide the window,
 * rfft, insert the FDL row, zero the accumulator, one MAC per partition (fdl_index.hpp:23-36),
 * irfft, scale, emit; the transforms are the oracle's (c2c_dit2 + real split, a few
 * per-mille of the work at P >= 64). Channels split over pthreads (the harness's choice). */
#include "neo_oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef void (*mac_fn)(const float* x, const float* y, float* acc, size_t n);

static void mac_scalar(const float* x, const float* y, float* acc, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        const float xr = x[2 * i], xi = x[2 * i + 1], yr = y[2 * i], yi = y[2 * i + 1];
        acc[2 * i] += xr * yr - xi * yi;
        acc[2 * i + 1] += xr * yi + xi * yr;
    }
}

__attribute__((target("avx512f"))) static void mac_avx512(const float* x, const float* y, float* acc, size_t n)
{
    /* deinterleave / reinterleave permutations of two 16-float vectors */
    const __m512i ire = _mm512_setr_epi32(0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30);
    const __m512i iim = _mm512_setr_epi32(1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25, 27, 29, 31);
    const __m512i ilo = _mm512_setr_epi32(0, 16, 1, 17, 2, 18, 3, 19, 4, 20, 5, 21, 6, 22, 7, 23);
    const __m512i ihi = _mm512_setr_epi32(8, 24, 9, 25, 10, 26, 11, 27, 12, 28, 13, 29, 14, 30, 15, 31);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        const __m512 x0 = _mm512_loadu_ps(x + 2 * i), x1 = _mm512_loadu_ps(x + 2 * i + 16);
        const __m512 y0 = _mm512_loadu_ps(y + 2 * i), y1 = _mm512_loadu_ps(y + 2 * i + 16);
        const __m512 z0 = _mm512_loadu_ps(acc + 2 * i), z1 = _mm512_loadu_ps(acc + 2 * i + 16);
        const __m512 xr = _mm512_permutex2var_ps(x0, ire, x1), xi = _mm512_permutex2var_ps(x0, iim, x1);
        const __m512 yr = _mm512_permutex2var_ps(y0, ire, y1), yi = _mm512_permutex2var_ps(y0, iim, y1);
        const __m512 zr = _mm512_permutex2var_ps(z0, ire, z1), zi = _mm512_permutex2var_ps(z0, iim, z1);
        const __m512 re = _mm512_add_ps(_mm512_fmsub_ps(xr, yr, _mm512_mul_ps(xi, yi)), zr);
        const __m512 im = _mm512_add_ps(_mm512_fmadd_ps(xr, yi, _mm512_mul_ps(xi, yr)), zi);
        _mm512_storeu_ps(acc + 2 * i, _mm512_permutex2var_ps(re, ilo, im));
        _mm512_storeu_ps(acc + 2 * i + 16, _mm512_permutex2var_ps(re, ihi, im));
    }
    mac_scalar(x + 2 * i, y + 2 * i, acc + 2 * i, n - i);
}

__attribute__((target("avx2,fma"))) static void mac_avx2(const float* x, const float* y, float* acc, size_t n)
{
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        /* deinterleave 8 complex: shuffle within 128-bit lanes, then fix the lane order */
        const __m256 x0 = _mm256_loadu_ps(x + 2 * i), x1 = _mm256_loadu_ps(x + 2 * i + 8);
        const __m256 y0 = _mm256_loadu_ps(y + 2 * i), y1 = _mm256_loadu_ps(y + 2 * i + 8);
        const __m256 z0 = _mm256_loadu_ps(acc + 2 * i), z1 = _mm256_loadu_ps(acc + 2 * i + 8);
#define DEINT(a, b, r, m)                                                                                    \
    const __m256 r = (__m256)_mm256_permute4x64_pd((__m256d)_mm256_shuffle_ps(a, b, 0x88), 0xd8);           \
    const __m256 m = (__m256)_mm256_permute4x64_pd((__m256d)_mm256_shuffle_ps(a, b, 0xdd), 0xd8);
        DEINT(x0, x1, xr, xi)
        DEINT(y0, y1, yr, yi)
        DEINT(z0, z1, zr, zi)
#undef DEINT
        const __m256 re = _mm256_add_ps(_mm256_fmsub_ps(xr, yr, _mm256_mul_ps(xi, yi)), zr);
        const __m256 im = _mm256_add_ps(_mm256_fmadd_ps(xr, yi, _mm256_mul_ps(xi, yr)), zi);
        const __m256 rp = (__m256)_mm256_permute4x64_pd((__m256d)re, 0xd8);
        const __m256 ip = (__m256)_mm256_permute4x64_pd((__m256d)im, 0xd8);
        _mm256_storeu_ps(acc + 2 * i, _mm256_unpacklo_ps(rp, ip));
        _mm256_storeu_ps(acc + 2 * i + 8, _mm256_unpackhi_ps(rp, ip));
    }
    mac_scalar(x + 2 * i, y + 2 * i, acc + 2 * i, n - i);
}

/* 2: AVX-512F, 1: AVX2 + FMA, 0: scalar */
int baseline_simd_level(void)
{
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f")) return 2;
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return 1;
    return 0;
}

static mac_fn pick(int level)
{
    const int have = baseline_simd_level();
    if (level < 0 || level > have) level = have;
    return level == 2 ? mac_avx512 : level == 1 ? mac_avx2 : mac_scalar;
}

typedef struct {
    const float* signal;
    float* out;
    const float* parts;
    size_t C, N, P, B, c0, c1;
    mac_fn mac;
    int rc;
} bl_job;

static void* bl_worker(void* arg)
{
    bl_job* j = (bl_job*)arg;
    const size_t B = j->B, P = j->P, bins = B + 1;
    int order = 0;
    while (((size_t)1 << order) < 2 * B - 1) ++order; /* overlap_save.hpp:53 */
    const size_t n = (size_t)1 << order;
    float* fdl = (float*)malloc(sizeof(float) * 2 * P * bins);
    float* acc = (float*)malloc(sizeof(float) * 2 * bins);
    float* window = (float*)malloc(sizeof(float) * n);
    float* cbuf = (float*)malloc(sizeof(float) * 2 * n);
    float* rbuf = (float*)malloc(sizeof(float) * n);
    if (!fdl || !acc || !window || !cbuf || !rbuf) j->rc = -2;
    for (size_t c = j->c0; c < j->c1 && j->rc == 0; ++c) {
        const float* H = j->parts + 2 * bins * P * c;
        memset(fdl, 0, sizeof(float) * 2 * P * bins);
        memset(window, 0, sizeof(float) * n);
        size_t w = 0;
        for (size_t i = 0; i < j->N && j->rc == 0; i += B) {
            const size_t cnt = (j->N - i) < B ? (j->N - i) : B;
            memmove(window, window + B, sizeof(float) * (n - B));
            memset(window + (n - B), 0, sizeof(float) * B);
            memcpy(window + (n - B), j->signal + c * j->N + i, sizeof(float) * cnt);
            j->rc = oracle_rfft(order, window, cbuf);
            memcpy(fdl + 2 * bins * w, cbuf, sizeof(float) * 2 * bins);
            memset(acc, 0, sizeof(float) * 2 * bins);
            for (size_t s = 0; s < P; ++s) j->mac(fdl + 2 * bins * s, H + 2 * bins * ((w + P - s) % P), acc, bins);
            memcpy(cbuf, acc, sizeof(float) * 2 * bins); /* the callback works in place on the stage's buffer */
            if (!j->rc) j->rc = oracle_irfft(order, cbuf, rbuf);
            const float scale = 1.0f / (float)n;
            for (size_t k = 0; k < cnt; ++k) j->out[c * j->N + i + k] = rbuf[n - B + k] * scale;
            if (++w >= P) w = 0;
        }
    }
    free(fdl);
    free(acc);
    free(window);
    free(cbuf);
    free(rbuf);
    return NULL;
}

/* dense_convolve on [C][N] signals with [C][P][B+1] partitions; simd_level -1 = best */
int baseline_dense_convolve(const float* signal, float* out, const float* parts, size_t C, size_t N, size_t P,
                            size_t B, int threads, int simd_level)
{
    if (threads < 1) threads = 1;
    if ((size_t)threads > C) threads = (int)C;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    bl_job jobs[256];
    const mac_fn mac = pick(simd_level);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (bl_job){signal, out, parts, C, N, P, B, C * t / threads, C * (t + 1) / threads, mac, 0};
        if (threads == 1) bl_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, bl_worker, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; ++t) {
        if (threads > 1) pthread_join(tid[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    return rc;
}
