// Connection batches: the classifier's slot mode over both tuples of every
// connection in one launch (kernels.hpp launch_classify4_pair).
//
// testConnection (aclengine_mock.go:394-471) evaluates a connection with two
// tuples: SYN (src, dst, dport) through the source's inbound and the
// destination's outbound ACL, SYN-ACK (dst, src, sport) through the
// destination's inbound and the source's outbound ACL.  A large ACL is
// evaluated here for both tuples of every connection; the connection kernel
// then reads the two result words instead of scanning the ACL.  One launch
// stages the image once per workgroup and reads each connection's fields
// once (13 B), writing 8 B.  The OTHER image (protocols > 2: networks alone
// decide, evalACL's switch has no case) is staged beside the main image
// when both fit LDS (no slot counters in this mode), so those connections
// are classified from LDS in place instead of by a chain of global loads.
#include "kernels_dev.hpp"

namespace cls {

namespace {

template <int kMode, int kList, int kD>
__global__ __launch_bounds__(kClsBlock) void classify4_pair(Cls4Dev t, Cls4Dev o, uint32_t o_at, Pkts4 p,
                                                            const uint16_t* sport, uint32_t* out, uint64_t stride) {
    extern __shared__ uint4 smem[];
    {
        const uint4* a = reinterpret_cast<const uint4*>(t.img);
        for (uint32_t i = threadIdx.x; i < t.img_bytes / 16u; i += blockDim.x) smem[i] = a[i];
        if (o_at) {
            const uint4* b = reinterpret_cast<const uint4*>(o.img);
            uint4* ob = smem + o_at / 16u;
            for (uint32_t i = threadIdx.x; i < o.img_bytes / 16u; i += blockDim.x) ob[i] = b[i];
        }
        __syncthreads();
    }
    const Img<true> im{nullptr};
    const Img<false> og{reinterpret_cast<const uint8_t*>(o.img)};
    // protocols > 2, one packet of the SYN (k = 0) or SYN-ACK (k = 1) tuple:
    // result | OTHER slot (after the main image's) << 2
    auto other1 = [&](uint32_t s, uint32_t d, uint32_t port) -> uint32_t {
        const uint32_t s1[1] = {s}, d1[1] = {d}, p1[1] = {port}, z1[1] = {0u};
        uint32_t r1[1], k1[1];
        if (o_at) classify_n<1, true, 0, 0, -1>(im, o, s1, d1, p1, z1, r1, k1);
        else classify_n<1, false, 0, 0, -1>(og, o, s1, d1, p1, z1, r1, k1);
        return r1[0] | ((t.n_ctr + k1[0]) << 2);
    };
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nsteps = uint32_t(p.n / 4u);
    const uint4* S = reinterpret_cast<const uint4*>(p.src);
    const uint4* D = reinterpret_cast<const uint4*>(p.dst);
    const uint2* DP = reinterpret_cast<const uint2*>(p.dport);
    const uint2* SP = reinterpret_cast<const uint2*>(sport);
    const uint32_t* PR = reinterpret_cast<const uint32_t*>(p.proto);
    uint4* OS = reinterpret_cast<uint4*>(out);
    uint4* OA = reinterpret_cast<uint4*>(out + stride);
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        const uint4 s4 = ldnt(at(S, g)), d4 = ldnt(at(D, g));
        const uint2 dp2 = ldnt(at(DP, g)), sp2 = ldnt(at(SP, g));
        const uint32_t pr = ldnt(at(PR, g));
        const uint32_t sa[4] = {s4.x, s4.y, s4.z, s4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
        const uint32_t dpa[4] = {dp2.x & 0xFFFFu, dp2.x >> 16, dp2.y & 0xFFFFu, dp2.y >> 16};
        const uint32_t spa[4] = {sp2.x & 0xFFFFu, sp2.x >> 16, sp2.y & 0xFFFFu, sp2.y >> 16};
        const uint32_t ra[4] = {pr & 0xFFu, (pr >> 8) & 0xFFu, (pr >> 16) & 0xFFu, pr >> 24};
        uint32_t r0[4], k0[4], r1[4], k1[4];
        classify_n<4, true, kMode, kList, kD>(im, t, sa, da, dpa, ra, r0, k0);
        classify_n<4, true, kMode, kList, kD>(im, t, da, sa, spa, ra, r1, k1);
        uint32_t w0[4], w1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w0[q] = r0[q] | (k0[q] << 2);
            w1[q] = r1[q] | (k1[q] << 2);
        }
        // some protocol byte > 2 (SWAR, as classify4_cls)
        if (__any(((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (ra[q] > 2u) {
                    w0[q] = other1(sa[q], da[q], dpa[q]);
                    w1[q] = other1(da[q], sa[q], spa[q]);
                }
            }
        }
        OS[g] = make_uint4(w0[0], w0[1], w0[2], w0[3]);
        OA[g] = make_uint4(w1[0], w1[1], w1[2], w1[3]);
    }
    for (uint32_t i = nsteps * 4u + tid; i < uint32_t(p.n); i += nthreads) {
        const uint32_t s = p.src[i], d = p.dst[i], dp = p.dport[i], sp = sport[i], pr = p.proto[i];
        uint32_t w0, w1;
        if (pr > 2u) {
            w0 = other1(s, d, dp);
            w1 = other1(d, s, sp);
        } else {
            const uint32_t sa[1] = {s}, da[1] = {d}, dpa[1] = {dp}, spa[1] = {sp}, ra[1] = {pr};
            uint32_t r[1], k[1];
            classify_n<1, true, kMode, kList, -1>(im, t, sa, da, dpa, ra, r, k);
            w0 = r[0] | (k[0] << 2);
            classify_n<1, true, kMode, kList, -1>(im, t, da, sa, spa, ra, r, k);
            w1 = r[0] | (k[0] << 2);
        }
        out[i] = w0;
        out[stride + i] = w1;
    }
}

template <int kMode, int kList, int kD>
void launch_pair_d(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                   uint32_t* out, uint64_t stride, const LaunchCfg& cfg) {
    const size_t lds = o_at ? o_at + o.img_bytes : t.img_bytes;
    lds_attr(reinterpret_cast<const void*>(classify4_pair<kMode, kList, kD>), lds);
    hipLaunchKernelGGL((classify4_pair<kMode, kList, kD>), dim3(cfg.grid), dim3(kClsBlock), lds, cfg.stream, t, o,
                       o_at, p, sport, out, stride);
}

// sublist modes: the search depth as a template argument (the rendered
// global tables' one-length hash, as the hot classify kernel)
template <int kMode, int kList>
void launch_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                 uint32_t* out, uint64_t stride, const LaunchCfg& cfg) {
    if constexpr (kMode == 2 && (kList == 3 || kList == 4)) {
        switch (t.bv_steps) {
        case 0: launch_pair_d<kMode, kList, 0>(t, o, o_at, p, sport, out, stride, cfg); return;
        case 1: launch_pair_d<kMode, kList, 1>(t, o, o_at, p, sport, out, stride, cfg); return;
        case 2: launch_pair_d<kMode, kList, 2>(t, o, o_at, p, sport, out, stride, cfg); return;
        case 3: launch_pair_d<kMode, kList, 3>(t, o, o_at, p, sport, out, stride, cfg); return;
        case 4: launch_pair_d<kMode, kList, 4>(t, o, o_at, p, sport, out, stride, cfg); return;
        case 5: launch_pair_d<kMode, kList, 5>(t, o, o_at, p, sport, out, stride, cfg); return;
        default: break;
        }
    }
    launch_pair_d<kMode, kList, -1>(t, o, o_at, p, sport, out, stride, cfg);
}

}  // namespace

hipError_t launch_classify4_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p,
                                 const uint16_t* sport, uint32_t* out, uint64_t stride, const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, true, false) || o.mode != 0 || o.list_mode != 0) return hipErrorInvalidValue;
    const int src = src_variant(t);
#define PAIR_CASE(S, M, L) \
    case 8 * S + L: launch_pair<M, L>(t, o, o_at, p, sport, out, stride, cfg); break;
    switch (8 * src + int(t.list_mode)) {
        PAIR_CASE(0, 0, 0) PAIR_CASE(0, 0, 1) PAIR_CASE(0, 0, 2) PAIR_CASE(0, 0, 3) PAIR_CASE(0, 0, 4)
        PAIR_CASE(0, 0, 5) PAIR_CASE(0, 0, 6)
        PAIR_CASE(1, 1, 0) PAIR_CASE(1, 1, 1) PAIR_CASE(1, 1, 2) PAIR_CASE(1, 1, 3) PAIR_CASE(1, 1, 4)
        PAIR_CASE(1, 1, 5) PAIR_CASE(1, 1, 6)
        PAIR_CASE(2, 2, 0) PAIR_CASE(2, 2, 1) PAIR_CASE(2, 2, 2) PAIR_CASE(2, 2, 3) PAIR_CASE(2, 2, 4)
        PAIR_CASE(2, 2, 5) PAIR_CASE(2, 2, 6)
        PAIR_CASE(3, 4, 3) PAIR_CASE(3, 4, 4) PAIR_CASE(3, 4, 5) PAIR_CASE(3, 4, 6)
    default: return hipErrorInvalidValue;
    }
#undef PAIR_CASE
    return hipGetLastError();
}

}  // namespace cls
