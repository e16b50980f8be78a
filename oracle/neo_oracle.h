/* neo_oracle.h — declarations of the CPU restatement (TEST INFRASTRUCTURE ONLY). */
#ifndef NEO_ORACLE_H
#define NEO_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
int oracle_fft_c2c(int order, int dir, float* x);
int oracle_rfft(int order, const float* in, float* out);
int oracle_irfft(int order, const float* in, float* out);
int oracle_overlap_stage(int kind, size_t block, size_t filter, const float* G, float* signal, size_t num_blocks);
void oracle_normalize_impulse(float* ir, size_t channels, size_t length);
size_t oracle_num_partitions(size_t length, size_t block);
int oracle_uniform_partition(const float* ir, size_t channels, size_t length, size_t block, float* out);
int oracle_dense_convolve(const float* signal, float* out, const float* parts, size_t C, size_t N, size_t P, size_t B,
                          int threads);
void oracle_noise(uint64_t seed, float* out, size_t n);
typedef struct oracle_upola2 oracle_upola2;
oracle_upola2* oracle_upola2_create(size_t P, size_t bins, const float* H);
void oracle_upola2_destroy(oracle_upola2* u);
int oracle_upola2_process(oracle_upola2* u, float* inout, size_t num_samples);
void oracle_hann(size_t size, float* w);
size_t oracle_stft_frames(size_t L, size_t frame, size_t overlap);
int oracle_stft(const float* x, size_t C, size_t L, size_t frame, size_t transform, size_t overlap,
                const float* window, float* out);
int oracle_fft_c2c_f64(int order, int dir, double* x);
int oracle_rfft_f64(int order, const double* in, double* out);
int oracle_irfft_f64(int order, const double* in, double* out);
int oracle_fft_convolve_f64(const double* signal, size_t n, const double* patch, size_t m, double* out);
void oracle_direct_convolve_f64(const double* signal, size_t n, const double* patch, size_t l, double* out);
#ifdef __cplusplus
}
#endif
#endif
