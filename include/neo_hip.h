/*
 * neo_hip.h — C-ABI drop-in boundary of the MI355X (gfx950) FFT + UPOLS hot path.
 *
 * libneo_hip.so exports exactly these symbols. Plain pointers, sizes and int
 * status codes only (no HIP / torch / C++ types in the signatures), so the
 * reference's C++ headers (include/neo/fft.hpp, include/neo/convolution.hpp in
 * this repo), its pybind11 module or any FFI can bind them.
 *
 * Conventions shared with the reference (paths relative to neo-dsp's tree):
 *   - complex data is interleaved float {re, im} = std::complex<float>
 *     (src/neo/complex/scalar_complex.hpp:14-114);
 *   - direction: -1 = forward e^{-2 pi i nk/N}, +1 = backward
 *     (src/neo/fft/direction.hpp:8-12); transforms are UNNORMALIZED
 *     (src/neo/fft/reference/c2c_dit2_plan.hpp:81-95);
 *   - r2c writes N/2+1 bins; c2r reads N/2+1 bins, ignores the imaginary parts of
 *     the DC and Nyquist bins and does not scale
 *     (src/neo/fft/fallback/fallback_rfft_plan.hpp:27-55);
 *   - UPOLS filters are uniform_partition's [C][P][B+1] layout
 *     (src/neo/convolution/uniform_partition.hpp:12-26).
 * Every function returns NEO_HIP_OK (0) or a nonzero status; neo_hip_last_error()
 * then holds a message (thread-local). Construction errors map to the
 * reference's std::runtime_error (c2c_dit2_plan.hpp:97-104).
 */
#ifndef NEO_HIP_H
#define NEO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define NEO_HIP_API __attribute__((visibility("default")))
#else
#define NEO_HIP_API
#endif

enum neo_hip_status {
    NEO_HIP_OK = 0,
    NEO_HIP_EINVAL = 1,   /* bad argument (order > max_order, null pointer, shape) */
    NEO_HIP_ERUNTIME = 2, /* HIP runtime / kernel failure */
    NEO_HIP_ENOMEM = 3,   /* device allocation failed */
    NEO_HIP_ENODEV = 4    /* no such GPU */
};

/* fft kinds; OR NEO_HIP_F64 for std::complex<double> / double plans (the reference's
 * fft_plan<complex<double>>, rfft_plan<double>; Python _neo.fft complex128 overloads,
 * extra/python/src/main.cpp:248-252). */
enum neo_hip_fft_kind { NEO_HIP_C2C = 0, NEO_HIP_R2C = 1, NEO_HIP_C2R = 2, NEO_HIP_F64 = 16 };

typedef struct neo_hip_fft_plan neo_hip_fft_plan;
typedef struct neo_hip_upols neo_hip_upols;

/* -- library ------------------------------------------------------------ */
/* ABI version of this header. neo_hip_upols_opts grows with it (0.1.0: 6 ints; 0.2.0: the 10
 * below), so a caller checks neo_hip_version() == NEO_HIP_VERSION before passing one. */
#define NEO_HIP_VERSION 200 /* 0.2.0 */
NEO_HIP_API const char* neo_hip_last_error(void);
NEO_HIP_API int neo_hip_version(void);
NEO_HIP_API int neo_hip_device_count(int* count);
/* Page-lock a caller-owned host range [p, p + bytes) and map it for every device, so that
 * host-memory entry points (neo_hip_upols_process) read and write it in place over PCIe
 * instead of staging it. The caller keeps the range alive until neo_hip_host_unregister(p). */
NEO_HIP_API int neo_hip_host_register(void* p, int64_t bytes);
NEO_HIP_API int neo_hip_host_unregister(void* p);
/* Handle buffers come from per-device chunks the library keeps mapped (256 MiB, or a request's own
 * size above 64 MiB), so creating and destroying convolvers never synchronizes the device. Empty
 * chunks stay cached (up to a quarter of the device's memory) for later handles; trim returns
 * every chunk no handle uses; info reports the bytes held and the bytes in use on a device. */
NEO_HIP_API int neo_hip_memory_trim(int device);
NEO_HIP_API int neo_hip_memory_info(int device, int64_t* reserved, int64_t* in_use);

/* -- FFT plans ------------------------------------------------------------
 * Replaces fft_plan<complex<float>> = c2c_dit2_plan (src/neo/fft/fft.hpp:36-52,
 * c2c_dit2_plan.hpp:21-104) and rfft_plan<float> = fallback_rfft_plan
 * (src/neo/fft/rfft.hpp:15-23, fallback_rfft_plan.hpp:14-61), batched.
 * max order 27 (c2c_dit2_plan.hpp:58-61); order > 27 -> NEO_HIP_EINVAL. */
NEO_HIP_API int neo_hip_fft_max_order(void);
NEO_HIP_API int neo_hip_fft_plan_create(int order, int64_t batch, int kind, int device, neo_hip_fft_plan** plan);
NEO_HIP_API int neo_hip_fft_plan_destroy(neo_hip_fft_plan* plan);
/* Device pointers, asynchronous on `stream` (a hipStream_t; NULL = the HIP
 * null stream, which is also torch's default stream). c2c: in/out [batch][N] complex (in == out allowed).
 * r2c: in [batch][N] float, out [batch][N/2+1] complex.
 * c2r: in [batch][N/2+1] complex, out [batch][N] float. `direction` is used by
 * c2c only (r2c is forward, c2r backward, as in fallback_rfft_plan). */
NEO_HIP_API int neo_hip_fft_execute(neo_hip_fft_plan* plan, const void* in, void* out, int direction, void* stream);
/* Host pointers, synchronous (staging through the plan's device buffers). */
NEO_HIP_API int neo_hip_fft_execute_host(neo_hip_fft_plan* plan, const void* in, void* out, int direction);

/* -- UPOLS convolver --------------------------------------------------------
 * Replaces C instances of upols_convolver<complex<float>> (one per channel,
 * src/neo/convolution/dense_convolver.hpp:19-20;
 * uniform_partitioned_convolver.hpp:13-65; overlap_save.hpp:84-112;
 * fdl_index.hpp:23-36) as driven by dense_convolve / DenseConvolution
 * (extra/plugin/src/dsp/DenseConvolution.hpp:35,39-70). `block` = B must be a
 * power of two in [16, 4096]; output block t corresponds to input block t
 * (zero latency). Channels are independent. */
NEO_HIP_API int neo_hip_upols_create(int channels, int block, int partitions, int device, neo_hip_upols** h);
/* Same engine with the overlap-add stage: C instances of upola_convolver<complex<float>>
 * (dense_convolver.hpp:23-24; overlap_add.hpp:76-106). All other neo_hip_upols_*
 * entry points apply to it unchanged. */
NEO_HIP_API int neo_hip_upola_create(int channels, int block, int partitions, int device, neo_hip_upols** h);
/* C instances of upola_convolver_v2<complex<float>> = overlap_add_convolver
 * (dense_convolver.hpp:28; overlap_add_convolver.hpp:20-136): overlap-add that also
 * takes sub-block input through neo_hip_upols_process_samples, with the reference's
 * window state (the irfft result is written back into the real window, :114). Whole
 * blocks through the other process calls behave like neo_hip_upola_create. */
NEO_HIP_API int neo_hip_upola2_create(int channels, int block, int partitions, int device, neo_hip_upols** h);
/* Any of the three with explicit choices instead of the shape-based defaults
 * (method 0 = upols, 1 = upola, 2 = upola v2; opts NULL = all defaults). Results are the
 * same for every choice up to float summation order; they exist so that every code path
 * can be exercised and timed on any shape. */
typedef struct neo_hip_upols_opts {
    int fused;            /* plain step: -1 auto (one launch below 64 MiB of filter + FDL), 0 MAC + finish, 1 one launch */
    int split_workgroups; /* plain step: 0 auto (1024 workgroups, >= 8 or 16 partitions per split), else the
                             workgroup target for its partition splits, taken as given (up to 64 per channel) */
    int batch_blocks;     /* batched passes: 0 auto (32), else blocks per pass (power of two, 2..32) */
    int batch_bins;       /* batched passes: 0 auto (1), else bins per lane vector (1 or 2) */
    int levels;           /* single-block steps: -1 auto (streaming levels from 64 partitions), 0 plain step, 1 levels */
    int far_level;        /* streaming levels, partitions >= 256: -1 auto (= 1), 0 a 128-block Toeplitz level (more
                             VALU / LDS work), 1 the 128-block partition-axis transform level with stored segment
                             and row-pair spectra, 2 the same transform recomputed every window from the filter and
                             FDL rows (fewest bytes; 2 nseg + 1 transforms per unit and window: more VALU, a longer
                             chain) */
    int far_group;        /* far transform level: 0 auto, else 1..4 windows per phase-1 pass over the stored
                             segment spectra (auto: 2, or round(sqrt(2 (nseg - 1))) from 32768 16-column units) */
    int toep_split;       /* 32-block Toeplitz level: 0 auto (2 below 256 16-column units), 1 whole windows per
                             workgroup, 2 two window halves */
    int step_group;       /* streaming levels: 0 auto, 1 one launch per block (the block and 1/T of every level's
                             next window), 2, 4 or 8 step groups: the block of every call as a launch of its own on the
                             caller's stream, the level slices of G calls as ONE launch on the handle's background
                             stream, issued at the group's first call (ordered by events; the output of a call is
                             complete when the caller's stream reaches it, as with G = 1) */
    int far_phase2;       /* far transform level, G = 1: 0 auto, 1 one workgroup per unit (the fresh row pair's
                             transform kept in registers for the window's products), 2 two steps (the fresh
                             transform stored to its slot, read back with the products one step later: half the
                             chain per step); step groups always run 1 */
} neo_hip_upols_opts;
NEO_HIP_API int neo_hip_upols_create_ex(int channels, int block, int partitions, int device, int method,
                                        const neo_hip_upols_opts* opts, neo_hip_upols** h);
NEO_HIP_API int neo_hip_upols_destroy(neo_hip_upols* h);
/* filter [C][P][B+1] complex (uniform_partition layout), host or device memory;
 * like uniform_partitioned_convolver::filter() it also resets all state. */
NEO_HIP_API int neo_hip_upols_set_filter(neo_hip_upols* h, const void* filter, int is_device);
/* normalize_impulse + uniform_partition of ir [C][L] float straight into the
 * convolver (setup path, DenseConvolution.cpp:78-108); host or device memory. */
NEO_HIP_API int neo_hip_upols_set_impulse(neo_hip_upols* h, const float* ir, int64_t length, int normalize, int is_device);
/* one block for all channels, in place: io [C][B] float. Host memory, synchronous (own
 * stream if `stream` is NULL): the step kernel reads and writes the block over PCIe
 * itself -- in place if io is page-locked (neo_hip_host_register / hipHostMalloc), else
 * through the handle's mapped pinned staging (one memcpy each way) -- and the call waits by
 * polling the stream. Device memory: same as process_device on `stream`. */
NEO_HIP_API int neo_hip_upols_process(neo_hip_upols* h, float* io, int io_is_device, void* stream);
/* one block, device pointers, channel c at in + c*ld_in / out + c*ld_out
 * (in == out allowed); asynchronous on `stream` (NULL = HIP null stream). */
NEO_HIP_API int neo_hip_upols_process_device(neo_hip_upols* h, const float* in, int64_t ld_in, float* out,
                                             int64_t ld_out, void* stream);
/* nblocks consecutive blocks: channel c samples at in + c*ld + t*B (16-byte aligned, ld
 * a multiple of 4; in == out allowed). With batching on (the default) whole groups of T
 * blocks (32 for B <= 512, fewer for larger blocks; neo_hip_upols_batch_info) share one
 * pass over the filter and the FDL, so HBM traffic per block drops ~T-fold; results equal the one-block-per-pass path within
 * float rounding (another summation order). The rest run one block per pass. */
NEO_HIP_API int neo_hip_upols_process_blocks(neo_hip_upols* h, const float* in, float* out, int64_t ld,
                                             int64_t nblocks, void* stream);
/* process_blocks batching on (default) or off (one block per pass, as a real-time
 * caller stepping process_device block by block). */
NEO_HIP_API int neo_hip_upols_set_batch(neo_hip_upols* h, int enable);
/* blocks one process_blocks pass consumes (1 with batching off) and its splits per channel */
NEO_HIP_API int neo_hip_upols_batch_info(neo_hip_upols* h, int* blocks_per_pass, int* splits);
/* Offline windows (whole-block handles of >= 128 partitions; on by default): with batching on,
 * every 256 (or 128) whole blocks of a process_blocks / process_samples call take ONE pass that
 * computes each 128-block window of every bin as the far level does its band -- DFT256 along the
 * block axis of each 128-partition segment's FDL rows, times the filter segment's spectrum (made
 * at the first pass after a filter change), one inverse transform per window -- instead of T-block
 * MAC passes over all P partitions: ~(nseg + 2) 128 FDL rows and nseg 256 spectrum rows per column
 * and pass, not 2 P per 32 blocks. Same outputs within float rounding (the blocks are known up
 * front, as in the reference's offline harness, extra/plugin/src/dsp/DenseConvolution.hpp:39-70,
 * extra/plugin/src/ui/BenchmarkTab.hpp:47-66). The rest of a call runs the T-block passes. */
NEO_HIP_API int neo_hip_upols_set_offline(neo_hip_upols* h, int enable);
/* offline windows on, and the 128-partition segments they transform */
NEO_HIP_API int neo_hip_upols_get_offline(neo_hip_upols* h, int* enabled, int* segments);
/* num_samples samples for every channel: channel c at in + c*ld_in / out + c*ld_out
 * (in == out allowed), host (synchronous) or device (asynchronous on `stream`) memory.
 * upola_convolver_v2 handles accept any count, split at block boundaries like
 * overlap_add_convolver::operator() (:80-134); upols / upola handles need a multiple
 * of the block (the reference's operator() takes exactly one block). */
NEO_HIP_API int neo_hip_upols_process_samples(neo_hip_upols* h, const float* in, int64_t ld_in, float* out,
                                              int64_t ld_out, int64_t num_samples, int is_device, void* stream);
NEO_HIP_API int neo_hip_upols_reset(neo_hip_upols* h);
/* Streaming levels for single-block steps (upols / upola; upols_levels.hip): the
 * partitions are cut into bands -- p in [0, 8) MAC'd by the block itself; Toeplitz windows
 * of 4 / 8 / 16 / 32 blocks for [8, 16) / [16, 32) / [32, 64) / [64, 256); for [256, P) a
 * 128-block partition-axis transform (or, by neo_hip_upols_opts.far_level, a Toeplitz window
 * of 128 blocks) -- and every band's contribution to the
 * blocks of its next window is computed during the current window, a slice of the columns
 * per block step, so every call does the same work (ONE launch per block, k_lvl_step: the
 * block and the slices side by side). Output is the same block by
 * block (summation order differs), latency stays one block. Default on from 64 partitions
 * (B <= 1024); v2 handles refuse it. Switching is allowed at any block boundary (the next
 * step computes the current windows whole). */
NEO_HIP_API int neo_hip_upols_set_ahead(neo_hip_upols* h, int enable);
/* enabled, block position in the current far window, longest window, number of levels */
NEO_HIP_API int neo_hip_upols_get_ahead(neo_hip_upols* h, int* enabled, int* phase, int* window, int* levels);
/* The level plan for `partitions` (no device needed): the block step takes [0, a0);
 * Toeplitz level l < nlevels has a window of T[l] blocks and the band [a[l], b[l]);
 * nseg far segments of 128 partitions from 256 (arrays of >= 5 entries); the automatic
 * choice of far_level. */
NEO_HIP_API int neo_hip_upols_level_plan(int partitions, int* a0, int* nlevels, int* T, int* a, int* b, int* nseg);
/* The step groups' background plan for (channels, block, partitions, step_group; 0 = automatic)
 * with default options (no device needed; for tests): phi[l], the window offset of Toeplitz level
 * l (its windows start at t0 + W T - phi: a level of 4 G <= T <= 32 blocks starts half a window
 * later, so the groups where the levels skip fall apart); the cycle length in step groups; the unit
 * cuts of every background level in level order, cycle / (T / G) windows of T / G cuts each, into
 * cuts[cuts_cap] (*ncuts = how many there are); the predicted background bytes per step group of
 * the cycle into loads[loads_cap]. uniform != 0: equal parts and no offsets (for comparison). */
NEO_HIP_API int neo_hip_upols_part_plan(int channels, int block, int partitions, int step_group, int uniform, int* phi,
                                        int* cycle, int* cuts, int cuts_cap, int* ncuts, double* loads, int loads_cap);
/* Paced background work (step groups only; a no-op with one launch per block): enable = 1 issues
 * the step group's background launch in G pieces, one per call, and every block waits for the
 * piece of the call before it; enable = 2 issues it in two pieces, at the group's calls 0 and
 * G / 2, and those calls' blocks wait for the piece before. Either way no call waits for more
 * than one piece of background work, so the host round trip per block is even (p99 near p50)
 * instead of one call in 2 G paying for two groups' launches. Same outputs; costs one
 * cross-stream wait per piece. 0 = off. The levels re-prime when it changes. */
NEO_HIP_API int neo_hip_upols_set_paced(neo_hip_upols* h, int enable);
/* Latency mode for latency-bound shapes (up to 16 channels; C3, and the reference benchmark's
 * one channel at B = 4096): ONE persistent kernel per handle steps every block. With the
 * streaming levels (64 partitions and up, blocks up to 512, the far level included) it runs their
 * block and slice roles, the Toeplitz levels' slices beside the caller's next block instead of
 * before it; without them (fewer than 64 partitions, any block up to 4096) the plain fused step.
 * A call writes the block's record to a mailbox in mapped host memory and spins until the kernel
 * reports the block done: no launch and no stream wait per block. Every process call is then
 * SYNCHRONOUS (complete on return; the stream argument is not used) and device inputs must be
 * ready when it is made. The kernel leaves after idle_ms without a block (the next call
 * relaunches it) and whenever a setup call (set_filter, set_impulse, reset, set_ahead,
 * set_persistent(0), destroy) runs. Outputs equal the normal step's bit for bit (the same sums in
 * the same order; the levels re-prime on entry and exit). Not available: EINVAL names the
 * reason. */
NEO_HIP_API int neo_hip_upols_set_persistent(neo_hip_upols* h, int enable, double idle_ms);
/* requested, kernel resident now, persistent launches so far */
NEO_HIP_API int neo_hip_upols_get_persistent(neo_hip_upols* h, int* enabled, int* running, int64_t* launches);
/* GPU time of the last min(63, cap) latency-mode steps, oldest first, in us: from the kernel
 * reading the block's record to its completion signal (both on the GPU clock) */
NEO_HIP_API int neo_hip_upols_persist_step_times(neo_hip_upols* h, double* us, int64_t cap, int64_t* count);
/* windows per far phase-1 pass the handle runs (neo_hip_upols_opts.far_group or the automatic
 * choice); 0 without a far transform level */
NEO_HIP_API int neo_hip_upols_get_far_group(neo_hip_upols* h, int* windows);
/* the form of the handle's p >= 256 band: 0 none, 1 partition-axis transform with stored segment
 * and row-pair spectra (far phase 1 + 2), 2 the same transform recomputed every window from the
 * filter and FDL rows (neo_hip_upols_opts.far_level 2), 3 the
 * 128-block Toeplitz level (far_level 0) */
NEO_HIP_API int neo_hip_upols_get_far_form(neo_hip_upols* h, int* form);
/* steps per background launch of the streaming levels' slices (neo_hip_upols_opts.step_group or
 * the automatic choice): 1 = one launch per step */
NEO_HIP_API int neo_hip_upols_get_step_group(neo_hip_upols* h, int* steps);
/* make `stream` wait (device-side, no host wait) for every background slice launch of the
 * handle's step groups issued so far; a no-op with one launch per step. Outputs never need
 * it (a block's launch already waits for the slices it reads); a caller bracketing steps with
 * events on `stream`, or reusing the device's bandwidth right after, does. No reference
 * counterpart: the reference's operator() is synchronous (uniform_partitioned_convolver.hpp:47-65). */
NEO_HIP_API int neo_hip_upols_join_background(neo_hip_upols* h, void* stream);
/* -- Multichannel convolver over several devices ------------------------------
 * C channels cut into n contiguous shards, shard i = channels [C i / n, C (i + 1) / n) on
 * devices[i] (a device may repeat), each a neo_hip_upols handle of its own (own stream).
 * The reference steps all channels of a plugin instance in one loop
 * (extra/plugin/src/dsp/DenseConvolution.hpp:35,50-67); channels never interact, so there is
 * no collective: every call below fans out to the shards concurrently (one host thread per
 * shard) and returns when all are done. Shard results equal those of one handle over all
 * channels within float summation order: the shape-based code-path choices (far window
 * group, Toeplitz window parts, fused step, splits) follow each shard's own channel count;
 * they are bit for bit equal where those choices coincide (the same opts force them).
 * method / opts as neo_hip_upols_create_ex. */
typedef struct neo_hip_upols_multi neo_hip_upols_multi;
NEO_HIP_API int neo_hip_upols_multi_create(int channels, int block, int partitions, const int* devices, int ndevices,
                                           int method, const neo_hip_upols_opts* opts, neo_hip_upols_multi** m);
NEO_HIP_API int neo_hip_upols_multi_destroy(neo_hip_upols_multi* m);
NEO_HIP_API int neo_hip_upols_multi_shards(neo_hip_upols_multi* m, int* nshards);
/* shard i: its handle (for device-resident I/O with neo_hip_upols_process_device /
 * process_blocks on that device), device, first channel and channel count */
NEO_HIP_API int neo_hip_upols_multi_shard(neo_hip_upols_multi* m, int i, neo_hip_upols** h, int* device,
                                          int* first_channel, int* channels);
/* filter [C][P][B+1] complex, host memory; resets all state */
NEO_HIP_API int neo_hip_upols_multi_set_filter(neo_hip_upols_multi* m, const void* filter);
/* ir [C][length] float, host memory; normalize: one factor over all C channels
 * (normalize_impulse.hpp:21-30), as a single handle would */
NEO_HIP_API int neo_hip_upols_multi_set_impulse(neo_hip_upols_multi* m, const float* ir, int64_t length, int normalize);
/* num_samples per channel (channel c at in + c*ld_in / out + c*ld_out, in == out allowed),
 * host memory, synchronous; block rules as neo_hip_upols_process_samples */
NEO_HIP_API int neo_hip_upols_multi_process_samples(neo_hip_upols_multi* m, const float* in, int64_t ld_in, float* out,
                                                    int64_t ld_out, int64_t num_samples);
NEO_HIP_API int neo_hip_upols_multi_reset(neo_hip_upols_multi* m);
/* -- Groups of single-channel convolvers (upols_group.hip) ---------------------------------
 * Members are C independent one-channel upols / upola convolvers of one shape, each with its
 * own filter and state, as the plugin's std::vector<upols_convolver> (DenseConvolution.hpp:35)
 * holds them; process(member, io) is that member's operator()(block): one block of B samples,
 * host memory, in place, complete on return. A group belongs to ONE owner (one plugin
 * instance's convolvers; C++: neo::convolution::convolver_group). While the callers follow the
 * plugin's frame pattern (every member called once per frame on a buffer of its own that it
 * reuses) AND every member's buffer lies in a range the owner registered, the group steps every
 * member in ONE launch at a frame's first call, from the blocks in the other members'
 * registered buffers, and later calls only verify their block (a different block re-runs that
 * member's block step alone); any other pattern runs each member on a handle of its own. Either
 * way each member's outputs are those of its own sequential convolver (up to float summation
 * order after a mode switch, which re-primes the streaming levels). The group never reads a
 * buffer outside the registered ranges. method 0 upols, 1 upola. */
typedef struct neo_hip_upols_group neo_hip_upols_group;
NEO_HIP_API int neo_hip_upols_group_create(int block, int partitions, int method, int device, neo_hip_upols_group** g);
NEO_HIP_API int neo_hip_upols_group_destroy(neo_hip_upols_group* g);
NEO_HIP_API int neo_hip_upols_group_join(neo_hip_upols_group* g, int* member);
NEO_HIP_API int neo_hip_upols_group_leave(neo_hip_upols_group* g, int member);
/* filter [P][B+1] complex (uniform_partition layout of one channel); resets the member's state */
NEO_HIP_API int neo_hip_upols_group_set_filter(neo_hip_upols_group* g, int member, const void* filter, int is_device);
NEO_HIP_API int neo_hip_upols_group_process(neo_hip_upols_group* g, int member, float* io);
NEO_HIP_API int neo_hip_upols_group_reset(neo_hip_upols_group* g, int member);
/* register [ptr, ptr + bytes) of host memory the owner keeps allocated until it unregisters it
 * (e.g. the plugin's frame buffer, ConstantOverlapAdd.hpp:34, between two prepare() calls):
 * only members whose buffers lie in a registered range are stepped ahead of their call.
 * Registering a range again is a no-op (cheap enough per frame). unregister(ptr) removes the
 * range starting at ptr, unregister(NULL) every range; the group then stops reading them
 * before the call returns (a coalesced group splits at its next frame). */
NEO_HIP_API int neo_hip_upols_group_register(neo_hip_upols_group* g, const void* ptr, int64_t bytes);
/* register_ex with flags: NEO_HIP_GROUP_FRAME_STABLE = the owner also promises that during a frame
 * (from its first member call until every member has made its call) nothing but those calls writes
 * the range, as in the plugin's loop over the channels of a filled frame (DenseConvolution.cpp:62-74).
 * A frame read in place from such a range then skips the leader's snapshot of every member's block
 * and the members' comparisons with it: a member's call on the buffer the step read is the copy of
 * its output (a call on another buffer re-runs that member's block step, exact). Without the flag
 * (register) each member's block is compared exactly and re-stepped on a difference. Registering the
 * same range again updates its flags. */
#define NEO_HIP_GROUP_FRAME_STABLE 1
/* NEO_HIP_GROUP_FRAME_INPLACE (implies STABLE): the owner also reads or writes a member's block only
 * through that member's call, every member on the same block of the range every frame -- exactly
 * processFrame's loop. The frame's first call then writes EVERY member's output into its block in
 * place, and a later member's call has nothing left to do. A member called on another buffer is
 * still stepped exactly (its own block step again), but its speculative output was written to its
 * old block: that is the promise the flag makes. */
#define NEO_HIP_GROUP_FRAME_INPLACE 2
NEO_HIP_API int neo_hip_upols_group_register_ex(neo_hip_upols_group* g, const void* ptr, int64_t bytes, int flags);
NEO_HIP_API int neo_hip_upols_group_unregister(neo_hip_upols_group* g, const void* ptr);
/* coalesced now; one-launch frame steps, member calls, block re-runs, mode switches so far */
NEO_HIP_API int neo_hip_upols_group_stats(neo_hip_upols_group* g, int* coalesced, int64_t* frame_steps, int64_t* calls,
                                          int64_t* redos, int64_t* switches);
/* Kernel timing with HIP events recorded on the launch stream (for the roofline in
 * bench.py): enable = n > 0 brackets every n-th launch group with events (0 = off).
 * timing() returns the summed ms of the bracketed part and the count of timed groups:
 * the MAC kernel of a plain or batched step, the whole step of a streaming-level step.
 * timing_detail() returns per part (ms[4], launches[4]): streaming-level steps 0 = the
 * step kernel (step groups: the block launch and the wait for the previous group's slices,
 * 1 = the slice launches on the background stream, one per G steps); plain / batched steps
 * 0 = MAC kernel. Both drain the events. */
NEO_HIP_API int neo_hip_upols_set_timing(neo_hip_upols* h, int enable);
NEO_HIP_API int neo_hip_upols_timing(neo_hip_upols* h, double* mac_ms, int64_t* launches);
NEO_HIP_API int neo_hip_upols_timing_detail(neo_hip_upols* h, double* ms, int64_t* launches);
/* the duration of every timed launch group in order (first to last event; a streaming
 * step: the whole step), up to cap into ms; count = groups recorded. Drains the events. */
NEO_HIP_API int neo_hip_upols_step_times(neo_hip_upols* h, double* ms, int64_t cap, int64_t* count);
NEO_HIP_API int neo_hip_upols_info(neo_hip_upols* h, int* channels, int* block, int* partitions, int* splits);

/* -- standalone overlap stages (overlap_save.hpp:19-112, overlap_add.hpp:23-107) -----------
 * C independent stages of block B (a power of two) for filters of F taps, transform size
 * n = 2^next_order(B + F - 1) (<= 2^27). The reference's operator()(block, callback) split
 * at the callback: forward = window update + rfft -> spectrum [C][n/2 + 1] complex (what the
 * callback sees), inverse = irfft of the (processed) spectrum, 1/n, output block. kind 0 =
 * overlap_save (window slid left by B, block at its end; output = the last B samples), 1 =
 * overlap_add (block at the window's start, [B, 2B) zeroed; output = first B + overlap, the
 * irfft written back into the window as the reference does). Blocks: channel c at in + c*ld.
 * Host memory: synchronous (own stream if NULL); device memory: asynchronous on `stream`. */
typedef struct neo_hip_overlap neo_hip_overlap;
NEO_HIP_API int neo_hip_overlap_create(int kind, int channels, int64_t block, int64_t filter, int device,
                                       neo_hip_overlap** h);
NEO_HIP_API int neo_hip_overlap_destroy(neo_hip_overlap* h);
NEO_HIP_API int neo_hip_overlap_info(neo_hip_overlap* h, int64_t* block, int64_t* filter, int64_t* transform_size);
NEO_HIP_API int neo_hip_overlap_reset(neo_hip_overlap* h);
NEO_HIP_API int neo_hip_overlap_forward(neo_hip_overlap* h, const float* in, int64_t ld_in, void* spectrum,
                                        int is_device, void* stream);
NEO_HIP_API int neo_hip_overlap_inverse(neo_hip_overlap* h, const void* spectrum, float* out, int64_t ld_out,
                                        int is_device, void* stream);

/* -- setup path (uniform_partition.hpp:12-26, normalize_impulse.hpp:11-33) -- */
NEO_HIP_API int neo_hip_num_partitions(int64_t length, int block, int64_t* partitions);
/* ir [C][L] float -> out [C][P][B+1] complex; host or device pointers. */
NEO_HIP_API int neo_hip_uniform_partition(const float* ir, int channels, int64_t length, int block, void* out,
                                          int is_device, int device);
/* in place on ir [C][L]: scale all channels by min_c 1/sqrt(sum ir[c]^2). */
NEO_HIP_API int neo_hip_normalize_impulse(float* ir, int channels, int64_t length, int is_device, int device);

/* -- one-shot full convolution (extra/python/src/neo/__init__.py:43-48) ----
 * out has n + m - 1 samples; n == 0 or m == 0 is a no-op (empty result).
 * fft_convolve: fft_convolver.hpp:19-93 (one r2c/c2r pair of size
 * 2^next_order(n+m-1) <= 2^27). direct_convolve: direct_convolve.hpp:14-56,
 * bit-identical to the reference's float loop. Host or device pointers. */
NEO_HIP_API int neo_hip_fft_convolve(const float* signal, int64_t n, const float* patch, int64_t m, float* out,
                                     int is_device, int device);
NEO_HIP_API int neo_hip_direct_convolve(const float* signal, int64_t n, const float* patch, int64_t m, float* out,
                                        int is_device, int device);
/* double overloads (main.cpp:257-258 bind both float and double) */
NEO_HIP_API int neo_hip_fft_convolve_f64(const double* signal, int64_t n, const double* patch, int64_t m, double* out,
                                         int is_device, int device);
NEO_HIP_API int neo_hip_direct_convolve_f64(const double* signal, int64_t n, const double* patch, int64_t m,
                                            double* out, int is_device, int device);

/* -- STFT (stft_plan, src/neo/fft/stft.hpp:40-109) ------------------------------
 * x [C][L] -> out [C][F][N/2+1] complex (float or double), N = 2^next_order(transform_size),
 * hop = frame_size - overlap, F = neo_hip_stft_num_frames(L, frame_size, overlap)
 * (detail::num_sftf_frames, :21-25). Frame f = x[f*hop, +min(L - f*hop, frame_size))
 * zero-padded to N, times window[0, N) (NULL = hann_window over N, windowing.hpp:29-41),
 * then rfft. Host or device pointers (window in the same memory as x). */
NEO_HIP_API int neo_hip_stft_num_frames(int64_t length, int frame_size, int overlap, int64_t* frames);
NEO_HIP_API int neo_hip_stft(const float* x, int channels, int64_t length, int frame_size, int transform_size,
                             int overlap, const float* window, void* out, int is_device, int device);
NEO_HIP_API int neo_hip_stft_f64(const double* x, int channels, int64_t length, int frame_size, int transform_size,
                                 int overlap, const double* window, void* out, int is_device, int device);

#ifdef __cplusplus
}
#endif

#endif /* NEO_HIP_H */
