// test_group.cpp — the plugin's call pattern with the convolver alias built for groups
// (NEO_HIP_CONVOLVER_GROUPS): extra/plugin/src/dsp/DenseConvolution.hpp:35 holds
// std::vector<upols_convolver<complex<float>>>, DenseConvolution.cpp:62-74 calls them channel by
// channel on the frame's AudioBlock. The owner (DenseConvolution) holds a convolver_group: the
// convolvers take their filters inside its scope() and the frame buffer is registered with it.
// 256 instances must equal one upols_multichannel over the same channels bit for bit, and
// (after the three frames the group watches: every buffer reused twice) run one launch per
// frame. The frame buffer is then freed and reallocated (a new prepare()): the owner
// unregisters it first, the group splits, re-coalesces on the new buffer, outputs stay exact.
// Convolvers outside any scope never coalesce.
#define NEO_HIP_CONVOLVER_GROUPS 1
#include <neo/convolution.hpp>

#include "../../oracle/neo_oracle.h"

#include <complex>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

using cf = std::complex<float>;

int main()
{
    int ndev = 0;
    if (neo_hip_device_count(&ndev) != NEO_HIP_OK || ndev < 1) {
        std::printf("no GPU: nothing to run\n");
        return 0;
    }
    std::size_t const C = 256, B = 512, L = 3 * 48000, nf = 24;
    std::vector<float> ir(C * L);
    for (std::size_t c = 0; c < C; ++c) oracle_noise(9000 + c, ir.data() + c * L, L);
    neo::convolution::normalize_impulse(neo::hip::make_matrix_view(ir.data(), C, L));
    auto const parts = neo::convolution::uniform_partition(neo::hip::make_matrix_view(ir.data(), C, L), B);
    std::size_t const P = parts.extent(1), bins = B + 1;
    // the plugin: one convolver per channel, each given its channel's partitions
    neo::convolution::convolver_group owner;  // DenseConvolution's member
    std::vector<neo::convolution::upols_convolver<cf>> convolvers(C);
    {
        auto scope = owner.scope();  // updateImpulseResponse()
        for (std::size_t c = 0; c < C; ++c)
            convolvers[c].filter(neo::hip::make_matrix_view(const_cast<cf*>(parts.data()) + c * P * bins, P, bins));
    }
    neo::convolution::upols_multichannel ref{C, B, P};
    ref.filter(parts.data());
    auto frame = std::make_unique<std::vector<float>>(C * B);
    std::vector<float> expect(C * B);
    owner.register_buffer(frame->data(), frame->size());  // the owner's frame buffer (ConstantOverlapAdd::_frame)
    int bad = 0;
    std::size_t const realloc_at = 12;
    for (std::size_t f = 0; f < nf; ++f) {
        if (f == realloc_at) {  // prepare(): the frame buffer is freed and allocated anew
            owner.unregister_all();
            frame.reset();
            std::vector<float> hole(C * B, 1.0F);  // keep the old address from coming straight back
            frame = std::make_unique<std::vector<float>>(C * B);
            owner.register_buffer(frame->data(), frame->size());
        }
        for (std::size_t c = 0; c < C; ++c) oracle_noise(20000 + f * C + c, frame->data() + c * B, B);
        expect = *frame;
        ref(expect.data());
        for (std::size_t c = 0; c < C; ++c)  // DenseConvolution::processFrame
            convolvers[c](neo::hip::make_view(frame->data() + c * B, B));
        if (std::memcmp(frame->data(), expect.data(), frame->size() * sizeof(float)) != 0) {
            std::printf("FAIL frame %zu differs from upols_multichannel\n", f);
            ++bad;
        }
    }
    int coalesced = 0;
    std::int64_t steps = 0, calls = 0, redos = 0, switches = 0;
    neo::hip::check(neo_hip_upols_group_stats(convolvers[0].group(), &coalesced, &steps, &calls, &redos, &switches));
    std::printf("group: coalesced %d, one-launch frames %lld of %zu, calls %lld, redos %lld, switches %lld\n", coalesced,
                (long long)steps, nf, (long long)calls, (long long)redos, (long long)switches);
    // frames 0-2 watched, 3-11 coalesced; at 12 the leader finds its neighbours' buffers
    // unregistered: split, 12-14 watched again, 15.. coalesced (3 switches)
    if (!coalesced || steps != std::int64_t(nf - 6) || calls != std::int64_t(nf * C) || redos != 0 || switches != 3) ++bad;
    // convolvers outside any scope: each alone, never one launch for several
    std::vector<neo::convolution::upols_convolver<cf>> alone(4);
    for (std::size_t c = 0; c < alone.size(); ++c)
        alone[c].filter(neo::hip::make_matrix_view(const_cast<cf*>(parts.data()) + c * P * bins, P, bins));
    if (alone[0].group() == alone[1].group()) {
        std::printf("FAIL unscoped convolvers share a group\n");
        ++bad;
    }
    std::printf(bad ? "FAILED\n" : "group test passed\n");
    return bad ? 1 : 0;
}
