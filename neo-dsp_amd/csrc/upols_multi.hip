// upols_multi.hip — the multichannel convolver over several devices of one node: C channels
// cut into contiguous shards, one neo_hip_upols handle (own device, own stream) per shard.
//
// The reference runs all channels of a plugin instance in one loop
// (extra/plugin/src/dsp/DenseConvolution.hpp:35 one convolver per channel, :50-67
// dense_convolve stepping them block by block); channels never interact, so sharding them
// needs no collective on the data path (BASELINE north_star: channels shard across the 8 GPUs
// of a node). Every call fans out to the shards from one host thread per shard, so the
// devices work concurrently; a shard's results are bit for bit those of an unsharded handle
// on the same channels (same kernels, same per-channel arithmetic; normalize_impulse's
// min-over-channels factor is taken over ALL channels first).
#include "upols_handle.hpp"

#include <thread>
#include <vector>

struct neo_hip_upols_multi {
    int C = 0, B = 0, P = 0;
    std::vector<neo_hip_upols*> shard;
    std::vector<int> dev, c0, nc;  // per shard: device, first channel, channels
};

namespace {

// run f(i) for every shard, one thread each; the first failure's code and message win
template<class F>
int fan_out(neo_hip_upols_multi* m, F f)
{
    const size_t n = m->shard.size();
    std::vector<int> rc(n, NEO_HIP_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            rc[i] = f(int(i));
            if (rc[i]) msg[i] = neo_hip_last_error();
        });
    for (auto& t : th) t.join();
    for (size_t i = 0; i < n; ++i)
        if (rc[i]) return neo_hip::fail(rc[i], "shard %zu (device %d): %s", i, m->dev[i], msg[i].c_str());
    return NEO_HIP_OK;
}

}  // namespace

using neo_hip::fail;

extern "C" {

NEO_HIP_API int neo_hip_upols_multi_create(int channels, int block, int partitions, const int* devices, int ndevices,
                                           int method, const neo_hip_upols_opts* opts, neo_hip_upols_multi** out)
{
    if (!out || !devices) return fail(NEO_HIP_EINVAL, "null argument");
    *out = nullptr;
    if (ndevices < 1 || ndevices > channels)
        return fail(NEO_HIP_EINVAL, "need 1 <= devices (%d) <= channels (%d)", ndevices, channels);
    auto* m = new (std::nothrow) neo_hip_upols_multi;
    if (!m) return fail(NEO_HIP_ENOMEM, "out of host memory");
    m->C = channels;
    m->B = block;
    m->P = partitions;
    for (int i = 0; i < ndevices; ++i) {
        const int a = int(int64_t(channels) * i / ndevices), b = int(int64_t(channels) * (i + 1) / ndevices);
        m->dev.push_back(devices[i]);
        m->c0.push_back(a);
        m->nc.push_back(b - a);
    }
    m->shard.assign(size_t(ndevices), nullptr);
    // created one after another: handle creation touches per-device state (streams, tables)
    for (int i = 0; i < ndevices; ++i) {
        if (int rc = neo_hip_upols_create_ex(m->nc[size_t(i)], block, partitions, m->dev[size_t(i)], method, opts,
                                             &m->shard[size_t(i)])) {
            const std::string e = neo_hip_last_error();
            neo_hip_upols_multi_destroy(m);
            return fail(rc, "shard %d (device %d): %s", i, devices[i], e.c_str());
        }
    }
    *out = m;
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_multi_destroy(neo_hip_upols_multi* m)
{
    if (!m) return NEO_HIP_OK;
    int rc = NEO_HIP_OK;
    for (auto* h : m->shard)
        if (h) {
            const int r = neo_hip_upols_destroy(h);
            if (!rc) rc = r;
        }
    delete m;
    return rc;
}

NEO_HIP_API int neo_hip_upols_multi_shards(neo_hip_upols_multi* m, int* nshards)
{
    if (!m || !nshards) return fail(NEO_HIP_EINVAL, "null argument");
    *nshards = int(m->shard.size());
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_multi_shard(neo_hip_upols_multi* m, int i, neo_hip_upols** h, int* device,
                                          int* first_channel, int* channels)
{
    if (!m) return fail(NEO_HIP_EINVAL, "null handle");
    if (i < 0 || i >= int(m->shard.size())) return fail(NEO_HIP_EINVAL, "shard %d out of range", i);
    if (h) *h = m->shard[size_t(i)];
    if (device) *device = m->dev[size_t(i)];
    if (first_channel) *first_channel = m->c0[size_t(i)];
    if (channels) *channels = m->nc[size_t(i)];
    return NEO_HIP_OK;
}

NEO_HIP_API int neo_hip_upols_multi_set_filter(neo_hip_upols_multi* m, const void* filter)
{
    if (!m || !filter) return fail(NEO_HIP_EINVAL, "null argument");
    const size_t per_channel = size_t(m->P) * size_t(m->B + 1) * 2 * sizeof(float);
    const char* base = static_cast<const char*>(filter);
    return fan_out(m, [&](int i) {
        return neo_hip_upols_set_filter(m->shard[size_t(i)], base + size_t(m->c0[size_t(i)]) * per_channel, 0);
    });
}

NEO_HIP_API int neo_hip_upols_multi_set_impulse(neo_hip_upols_multi* m, const float* ir, int64_t length, int normalize)
{
    if (!m || !ir) return fail(NEO_HIP_EINVAL, "null argument");
    if (length < 1) return fail(NEO_HIP_EINVAL, "length must be >= 1");
    const float* src = ir;
    std::vector<float> tmp;
    if (normalize) {  // one factor over all channels (normalize_impulse.hpp:21-30), then per shard as is
        tmp.assign(ir, ir + size_t(m->C) * size_t(length));
        if (int rc = neo_hip_normalize_impulse(tmp.data(), m->C, length, 0, m->dev[0])) return rc;
        src = tmp.data();
    }
    return fan_out(m, [&](int i) {
        return neo_hip_upols_set_impulse(m->shard[size_t(i)], src + size_t(m->c0[size_t(i)]) * size_t(length), length,
                                         0, 0);
    });
}

NEO_HIP_API int neo_hip_upols_multi_process_samples(neo_hip_upols_multi* m, const float* in, int64_t ld_in, float* out,
                                                    int64_t ld_out, int64_t num_samples)
{
    if (!m || !in || !out) return fail(NEO_HIP_EINVAL, "null argument");
    return fan_out(m, [&](int i) {
        const int64_t c = m->c0[size_t(i)];
        return neo_hip_upols_process_samples(m->shard[size_t(i)], in + c * ld_in, ld_in, out + c * ld_out, ld_out,
                                             num_samples, 0, nullptr);
    });
}

NEO_HIP_API int neo_hip_upols_multi_reset(neo_hip_upols_multi* m)
{
    if (!m) return fail(NEO_HIP_EINVAL, "null handle");
    return fan_out(m, [&](int i) { return neo_hip_upols_reset(m->shard[size_t(i)]); });
}

}  // extern "C"
