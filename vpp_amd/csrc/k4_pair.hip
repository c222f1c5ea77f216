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
// when both fit LDS (no slot counters in this mode).  Those connections are
// queued with their fields (16-B entries in the workgroup's segment of oq,
// its fill counted in LDS) and
// classified on the OTHER image after the workgroup's main loop, one per
// lane: the OTHER chain (interval search, candidate scan) then runs once per
// 1024 of them instead of once per wave step that holds any.
#include "kernels_dev.hpp"

namespace cls {

namespace {

static_assert(kClsBlock == kPairBlock, "pair_queue_words sizes the queue for this block");

template <int kMode, int kList, int kD>
__global__ __launch_bounds__(kClsBlock) void classify4_pair(Cls4Dev t, Cls4Dev o, uint32_t o_at, Pkts4 p,
                                                            const uint16_t* sport, uint32_t* out, uint64_t stride,
                                                            uint32_t* oq, uint32_t oq_seg, uint32_t q_lds) {
    extern __shared__ uint4 smem[];
    typedef __attribute__((address_space(3))) uint32_t* lctr_t;
    if (threadIdx.x == 0) *lctr_t(q_lds) = 0u;          // the queue fill (made visible by the barrier below)
    lds_copy(smem, reinterpret_cast<const uint4*>(t.img), t.img_bytes / 16u);
    if (o_at) lds_copy(smem + o_at / 16u, reinterpret_cast<const uint4*>(o.img), o.img_bytes / 16u);
    __syncthreads();
    const Img<true> im{nullptr};
    const Img<false> og{reinterpret_cast<const uint8_t*>(o.img)};
    // protocols > 2, both tuples of one connection -- SYN (s, d, dp) and
    // SYN-ACK (d, s, sp) -- on the OTHER image, their two chains interleaved:
    // result | OTHER slot (after the main image's) << 2
    auto other2 = [&](uint32_t s, uint32_t d, uint32_t dp, uint32_t sp, uint32_t& w0, uint32_t& w1) {
        const uint32_t s2[2] = {s, d}, d2[2] = {d, s}, p2[2] = {dp, sp}, z2[2] = {0u, 0u};
        uint32_t r2[2], k2[2];
        if (o_at) classify_n<2, true, 0, 0, -1>(im, o, s2, d2, p2, z2, r2, k2);
        else classify_n<2, false, 0, 0, -1>(og, o, s2, d2, p2, z2, r2, k2);
        w0 = r2[0] | ((t.n_ctr + k2[0]) << 2);
        w1 = r2[1] | ((t.n_ctr + k2[1]) << 2);
    };
    const uint32_t lane = __lane_id();
    const uint64_t lt = (1ull << lane) - 1ull;
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
    uint4* OQ = reinterpret_cast<uint4*>(oq);       // queued: {index, src, dst, dport | sport << 16}
    // G groups of four connections per lane per iteration: two (16 chains,
    // 108 VGPRs) measured slower than one, 41.9 against 40.8 us
    // (profiles/r04h2_pair_ab.txt)
    constexpr int G = 1;
    for (uint32_t g0 = tid; g0 < nsteps; g0 += G * nthreads) {
        uint32_t s8[8 * G], d8[8 * G], p8[8 * G], r8[8 * G], prs[G];
        bool live[G];
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const uint32_t g = g0 + uint32_t(h) * nthreads;
            live[h] = h == 0 || g < nsteps;
            const uint32_t gc = live[h] ? g : g0;
            const uint4 s4 = ldnt(at(S, gc)), d4 = ldnt(at(D, gc));
            const uint2 dp2 = ldnt(at(DP, gc)), sp2 = ldnt(at(SP, gc));
            const uint32_t pr = ldnt(at(PR, gc));
            prs[h] = pr;
            const uint32_t sa[4] = {s4.x, s4.y, s4.z, s4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
            const uint32_t dpa[4] = {dp2.x & 0xFFFFu, dp2.x >> 16, dp2.y & 0xFFFFu, dp2.y >> 16};
            const uint32_t spa[4] = {sp2.x & 0xFFFFu, sp2.x >> 16, sp2.y & 0xFFFFu, sp2.y >> 16};
            // both tuples of the four connections as one group of eight: their
            // eight chains of dependent LDS reads run interleaved
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t r = (pr >> (8 * q)) & 0xFFu;
                s8[8 * h + q] = sa[q]; s8[8 * h + 4 + q] = da[q];
                d8[8 * h + q] = da[q]; d8[8 * h + 4 + q] = sa[q];
                p8[8 * h + q] = dpa[q]; p8[8 * h + 4 + q] = spa[q];
                r8[8 * h + q] = r; r8[8 * h + 4 + q] = r;
            }
        }
        uint32_t res8[8 * G], k8[8 * G];
        classify_n<8 * G, true, kMode, kList, kD>(im, t, s8, d8, p8, r8, res8, k8);
#pragma unroll
        for (int h = 0; h < G; ++h) {
            const uint32_t g = g0 + uint32_t(h) * nthreads, pr = prs[h];
            uint32_t w0[4], w1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                w0[q] = res8[8 * h + q] | (k8[8 * h + q] << 2);
                w1[q] = res8[8 * h + 4 + q] | (k8[8 * h + 4 + q] << 2);
            }
            // Some protocol byte > 2 (SWAR, as classify4_cls): those connections
            // go to the workgroup's queue (one reservation per wave step); their
            // words above are overwritten after the main loop
            const bool oth = live[h] && ((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u;
            if (__any(oth)) {
                uint64_t m[4];
                uint32_t c[5];
                c[0] = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    m[q] = __ballot(oth && ((pr >> (8 * q)) & 0xFFu) > 2u);
                    c[q + 1] = c[q] + uint32_t(__popcll(m[q]));
                }
                uint32_t base = 0u;
                if (lane == 0u)
                    base = __hip_atomic_fetch_add(lctr_t(q_lds), c[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                base = __shfl(base, 0);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if ((m[q] >> lane) & 1u) {
                        const uint32_t k = base + c[q] + uint32_t(__popcll(m[q] & lt));
                        if (k < oq_seg)
                            OQ[uint64_t(blockIdx.x) * oq_seg + k] =
                                make_uint4(4u * g + uint32_t(q), s8[8 * h + q], d8[8 * h + q],
                                           p8[8 * h + q] | (p8[8 * h + 4 + q] << 16));
                        else    // the segment is full (a fixed size per workgroup): classify in place
                            other2(s8[8 * h + q], d8[8 * h + q], p8[8 * h + q], p8[8 * h + 4 + q], w0[q], w1[q]);
                    }
            }
            if (live[h]) {
                OS[g] = make_uint4(w0[0], w0[1], w0[2], w0[3]);
                OA[g] = make_uint4(w1[0], w1[1], w1[2], w1[3]);
            }
        }
    }
    for (uint32_t i = nsteps * 4u + tid; i < uint32_t(p.n); i += nthreads) {
        const uint32_t s = p.src[i], d = p.dst[i], dp = p.dport[i], sp = sport[i], pr = p.proto[i];
        uint32_t w0, w1;
        if (pr > 2u) {
            other2(s, d, dp, sp, w0, w1);
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
    // the queued connections of protocol > 2, one per lane, their fields
    // from the queue entry (no gather from the connection arrays; the barrier
    // orders their words after the main loop's stores of the same words)
    __syncthreads();
    const uint32_t nq = min(*lctr_t(q_lds), oq_seg);
    for (uint32_t j = threadIdx.x; j < nq; j += blockDim.x) {
        const uint4 e = OQ[uint64_t(blockIdx.x) * oq_seg + j];
        uint32_t w0, w1;
        other2(e.y, e.z, e.w & 0xFFFFu, e.w >> 16, w0, w1);
        out[e.x] = w0;
        out[stride + e.x] = w1;
    }
}

template <int kMode, int kList, int kD>
void launch_pair_d(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                   uint32_t* out, uint64_t stride, uint32_t* oq, uint32_t oq_cap, const LaunchCfg& cfg) {
    const uint32_t q_lds = ((o_at ? o_at + o.img_bytes : t.img_bytes) + 15u) & ~15u;   // the queue fill word
    const size_t lds = q_lds + 16u;
    lds_attr(reinterpret_cast<const void*>(classify4_pair<kMode, kList, kD>), lds);
    hipLaunchKernelGGL((classify4_pair<kMode, kList, kD>), dim3(cfg.grid), dim3(kClsBlock), lds, cfg.stream, t, o,
                       o_at, p, sport, out, stride, oq, oq_cap, q_lds);
}

// sublist modes: the search depth as a template argument (the rendered
// global tables' one-length hash, as the hot classify kernel)
template <int kMode, int kList>
void launch_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                 uint32_t* out, uint64_t stride, uint32_t* oq, uint32_t oq_cap, const LaunchCfg& cfg) {
    if constexpr (kMode == 2 && (kList == 3 || kList == 4)) {
        switch (t.bv_steps) {
        case 0: launch_pair_d<kMode, kList, 0>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        case 1: launch_pair_d<kMode, kList, 1>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        case 2: launch_pair_d<kMode, kList, 2>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        case 3: launch_pair_d<kMode, kList, 3>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        case 4: launch_pair_d<kMode, kList, 4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        case 5: launch_pair_d<kMode, kList, 5>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); return;
        default: break;
        }
    }
    launch_pair_d<kMode, kList, -1>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg);
}

}  // namespace

hipError_t launch_classify4_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p,
                                 const uint16_t* sport, uint32_t* out, uint64_t stride, uint32_t* oq,
                                 uint32_t oq_cap, const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, true, false) || o.mode != 0 || o.list_mode != 0) return hipErrorInvalidValue;
    const int src = src_variant(t);
#define PAIR_CASE(S, M, L) \
    case 8 * S + L: launch_pair<M, L>(t, o, o_at, p, sport, out, stride, oq, oq_cap, cfg); break;
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
