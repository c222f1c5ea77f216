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
// once (13 B), writing 1 B (the two results) or two counter-index words.
//
// The default image (kO4) is the table's pair image: a fourth cell per
// source class for protocols > 2 (networks alone decide, evalACL's switch
// has no case for them), so every connection takes the main loop's eight
// interleaved chains.  That replaced the path below, whose OTHER queue
// upkeep and end-of-launch drain were 3.1 and 6.7 of its 27.4 us at 4 Mi
// connections (profiles/r06pab_pair_breakdown.txt; 17.6-18.4 us on the pair
// image, profiles/r06o4_pair_image_ab.txt).
//
// The OTHER-queue path (the main image plus the OTHER image; tables whose
// pair image does not fit LDS, batches counting by slot): the OTHER image is
// staged beside the main image when both fit LDS, else over the main image
// once every wave has left its main loop (o_late; global memory before:
// 30.4 against 28.5 us when forced on config 3).  Connections of protocol
// > 2 are queued with their fields (16-B entries in the wave's segment:
// first in the LDS left after the images, then in global memory, its fill a
// wave-uniform register) and classified on the OTHER image after the wave's
// main loop, one per lane.  When the OTHER image's source classes are the
// main image's (cdiv != 0: same interval bounds and class numbering, checked
// by the host), an entry carries the two tuples' classes, found by the main
// loop's lookups, and the drain starts at the class row (27.3 -> 26.3 us).
// The OTHER image's candidates check no ports, so the entry does not carry
// them.
#include "kernels_dev.hpp"

namespace cls {

namespace {

static_assert(kClsBlock == kPairBlock, "pair_queue_words sizes the queue for this block");

// kO4: t is the pair image (four cells per class, compile.hpp
// Cls4Opts::with_other): every connection is classified in the main loop,
// no OTHER queue and no drain (o, o_at, the queue and cdiv unused)
template <int kMode, int kList, int kD, bool kO4>
__global__ __launch_bounds__(kClsBlock) void classify4_pair(Cls4Dev t, Cls4Dev o, uint32_t o_at, Pkts4 p,
                                                            const uint16_t* sport, uint32_t* out, uint64_t stride,
                                                            uint32_t* oq, uint32_t gqw, uint32_t q_lds,
                                                            const uint32_t* slot_rule, uint32_t ctr_base,
                                                            uint32_t wbytes, uint32_t lqw, uint32_t o_late,
                                                            uint32_t cdiv, const uint16_t* slot16, uint32_t srl,
                                                            uint32_t srl_n) {
    extern __shared__ uint4 smem[];
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
    // the wave's queue segment: {index, src, dst, dport | sport << 16} or
    // (cdiv) {index, src, dst, SYN class | SYN-ACK class << 16}
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t lq = q_lds + 16u * lqw * (threadIdx.x >> 6);
    uint4* const GQ = reinterpret_cast<uint4*>(oq) + uint64_t(wave) * gqw;
    uint32_t wq = 0;                                    // the segment's fill (wave-uniform)
    // Four connections' fields per lane, fetched one step ahead: a batch of a
    // few Mi connections gives each lane only a few steps, each of which
    // would otherwise start with a full memory latency (the kernel waited on
    // 61 % of its wave-cycles, profiles/r04s_sq_counters_conn_locals12.txt).
    // The first step's loads go out before the image staging.
    struct Fields {
        uint4 s4, d4;
        uint2 dp2, sp2;
        uint32_t pr;
    };
    auto fetch = [&](uint32_t g, Fields& f) {
        f.s4 = ldnt(at(S, g));
        f.d4 = ldnt(at(D, g));
        f.dp2 = ldnt(at(DP, g));
        f.sp2 = ldnt(at(SP, g));
        f.pr = ldnt(at(PR, g));
    };
    Fields nx{};
    if (tid < nsteps) fetch(tid, nx);
    // both images in one round of loads (a second round is a second memory
    // latency before the first step)
    // (srl: the slot -> rule map as u16 at LDS byte srl, srl_n 16-B units;
    // it takes the OTHER image's place -- the pair image has none)
    lds_copy2(smem, reinterpret_cast<const uint4*>(t.img), t.img_bytes / 16u, srl ? srl / 16u : o_at / 16u,
              srl ? reinterpret_cast<const uint4*>(slot16) : reinterpret_cast<const uint4*>(o.img),
              srl ? srl_n : o_at ? o.img_bytes / 16u : 0u);
    __syncthreads();
    const Img<true> im{nullptr};
    const Img<false> og{reinterpret_cast<const uint8_t*>(o.img)};
    // a word's payload: the slot, or (counting) its counter index
    // (from the LDS copy of the map when there is one)
    auto key = [&](uint32_t slot) {
        return srl ? ctr_base + *lds16_t(srl + 2u * slot) : slot_rule ? ctr_base + slot_rule[slot] : slot;
    };
    // one connection's two words: u32, u16 (wbytes 2: the host keeps the
    // counter indices below 2^14; both in one u32), or (wbytes 1) its two
    // results in one byte
    auto put = [&](uint32_t i, uint32_t w0, uint32_t w1) {
        if (wbytes == 1u) {
            reinterpret_cast<uint8_t*>(out)[i] = uint8_t((w0 & 3u) | (w1 & 3u) << 2);
        } else if (wbytes == 2u) {
            out[i] = (w0 & 0xFFFFu) | w1 << 16;
        } else {
            out[i] = w0;
            out[stride + i] = w1;
        }
    };
    // protocols > 2, both tuples of one connection -- SYN (s, d, dp) and
    // SYN-ACK (d, s, sp) -- on the OTHER image, their two chains interleaved:
    // result | OTHER slot (after the main image's) << 2.  lds: the OTHER
    // image is in LDS (beside the main one, or staged late for the drain)
    auto other2 = [&](uint32_t s, uint32_t d, uint32_t dp, uint32_t sp, uint32_t& w0, uint32_t& w1, bool lds) {
        const uint32_t s2[2] = {s, d}, d2[2] = {d, s}, p2[2] = {dp, sp}, z2[2] = {0u, 0u};
        uint32_t r2[2], k2[2];
        if (lds) classify_n<2, true, 0, 0, -1>(im, o, s2, d2, p2, z2, r2, k2);
        else classify_n<2, false, 0, 0, -1>(og, o, s2, d2, p2, z2, r2, k2);
        w0 = r2[0] | (key(t.n_ctr + k2[0]) << 2);
        w1 = r2[1] | (key(t.n_ctr + k2[1]) << 2);
    };
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        const Fields f = nx;
        if (g + nthreads < nsteps) fetch(g + nthreads, nx);
        const uint32_t pr = f.pr;
        const uint32_t sa[4] = {f.s4.x, f.s4.y, f.s4.z, f.s4.w}, da[4] = {f.d4.x, f.d4.y, f.d4.z, f.d4.w};
        const uint32_t dpa[4] = {f.dp2.x & 0xFFFFu, f.dp2.x >> 16, f.dp2.y & 0xFFFFu, f.dp2.y >> 16};
        const uint32_t spa[4] = {f.sp2.x & 0xFFFFu, f.sp2.x >> 16, f.sp2.y & 0xFFFFu, f.sp2.y >> 16};
        // both tuples of the four connections as one group of eight: their
        // eight chains of dependent LDS reads run interleaved
        uint32_t s8[8], d8[8], p8[8], r8[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t r = (pr >> (8 * q)) & 0xFFu;
            s8[q] = sa[q]; s8[4 + q] = da[q];
            d8[q] = da[q]; d8[4 + q] = sa[q];
            p8[q] = dpa[q]; p8[4 + q] = spa[q];
            r8[q] = r; r8[4 + q] = r;
        }
        uint32_t rv[8], k8[8], row8[8];
        classify_n<8, true, kMode, kList, kD, kO4 ? 4 : 3>(im, t, s8, d8, p8, r8, rv, k8, kO4 ? nullptr : &row8);
        uint32_t w0[4], w1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            w0[q] = rv[q] | (key(k8[q]) << 2);
            w1[q] = rv[4 + q] | (key(k8[4 + q]) << 2);
        }
        // Some protocol byte > 2 (SWAR, as classify4_cls): those connections
        // go to the wave's queue segment; their words above are overwritten
        // after the main loop
        const bool oth = !kO4 && ((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u;
        if (__any(oth)) {
            wq = __builtin_amdgcn_readfirstlane(wq);     // (lanes done with the loop keep stale copies)
            uint64_t m[4];
            uint32_t c[5];
            c[0] = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                m[q] = __ballot(oth && ((pr >> (8 * q)) & 0xFFu) > 2u);
                c[q + 1] = c[q] + uint32_t(__popcll(m[q]));
            }
            const uint32_t base = wq;
            wq += c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((m[q] >> lane) & 1u) {
                    const uint32_t k = base + c[q] + uint32_t(__popcll(m[q] & lt));
                    // (the class: the row's offset / row_bytes, by ceil(2^32 / row_bytes))
                    const uint32_t w3 = cdiv ? __umulhi(row8[q] - t.off_cells, cdiv) |
                                                   __umulhi(row8[4 + q] - t.off_cells, cdiv) << 16
                                             : p8[q] | (p8[4 + q] << 16);
                    const uint4 ent = make_uint4(4u * g + uint32_t(q), s8[q], d8[q], w3);
                    if (k < lqw)                // the LDS part of the segment
                        *lds128w_t(lq + 16u * k) = v4u{ent.x, ent.y, ent.z, ent.w};
                    else if (k - lqw < gqw)
                        GQ[k - lqw] = ent;
                    else    // the segment is full (a fixed size per wave): classify in place
                        other2(s8[q], d8[q], p8[q], p8[4 + q], w0[q], w1[q], o_at != 0u);
                }
        }
        if (wbytes == 1u) {                             // both results of the 4 connections: 4 bytes
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v |= ((w0[q] & 3u) | (w1[q] & 3u) << 2) << (8 * q);
            reinterpret_cast<uint32_t*>(out)[g] = v;
        } else if (wbytes == 2u) {                      // SYN | SYN-ACK << 16 per connection: 16 bytes
            OS[g] = make_uint4(w0[0] | w1[0] << 16, w0[1] | w1[1] << 16, w0[2] | w1[2] << 16, w0[3] | w1[3] << 16);
        } else {
            OS[g] = make_uint4(w0[0], w0[1], w0[2], w0[3]);
            OA[g] = make_uint4(w1[0], w1[1], w1[2], w1[3]);
        }
    }
    for (uint32_t i = nsteps * 4u + tid; i < uint32_t(p.n); i += nthreads) {
        const uint32_t s = p.src[i], d = p.dst[i], dp = p.dport[i], sp = sport[i], pr = p.proto[i];
        uint32_t w0, w1;
        if (!kO4 && pr > 2u) {
            other2(s, d, dp, sp, w0, w1, o_at != 0u);
        } else {
            const uint32_t sa[1] = {s}, da[1] = {d}, dpa[1] = {dp}, spa[1] = {sp}, ra[1] = {pr};
            uint32_t r[1], k[1];
            classify_n<1, true, kMode, kList, -1, kO4 ? 4 : 3>(im, t, sa, da, dpa, ra, r, k);
            w0 = r[0] | (key(k[0]) << 2);
            classify_n<1, true, kMode, kList, -1, kO4 ? 4 : 3>(im, t, da, sa, spa, ra, r, k);
            w1 = r[0] | (key(k[0]) << 2);
        }
        put(i, w0, w1);
    }
    if constexpr (kO4) return;
    // the wave's queued connections of protocol > 2, one per lane, their
    // fields from the queue entry (no gather from the connection arrays); the
    // wave's own main-loop stores of the same words complete first
    __threadfence_block();
    if (o_late) {                                       // uniform
        __syncthreads();                                // every wave is done with the main image
        lds_copy(smem, reinterpret_cast<const uint4*>(o.img), o.img_bytes / 16u);
        __syncthreads();
    }
    // lane 0's fill is current: the main loop's active lanes are a prefix
    const uint32_t nq = min(__builtin_amdgcn_readlane(wq, 0), lqw + gqw);
    for (uint32_t j = lane; j < nq; j += 64u) {
        uint4 e;
        if (j < lqw) {
            const v4u x = *lds128_t(lq + 16u * j);
            e = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            e = GQ[j - lqw];
        }
        uint32_t w0, w1;
        if (cdiv) {                                     // uniform: from the class rows
            const uint32_t r2[2] = {o.off_cells + (e.w & 0xFFFFu) * o.row_bytes, o.off_cells + (e.w >> 16) * o.row_bytes};
            const uint32_t d2[2] = {e.z, e.y}, z2[2] = {0u, 0u};
            uint32_t v2[2], k2[2];
            if (o_at | o_late) classify_n<2, true, 3, 0, -1>(im, o, r2, d2, z2, z2, v2, k2);
            else classify_n<2, false, 3, 0, -1>(og, o, r2, d2, z2, z2, v2, k2);
            w0 = v2[0] | (key(t.n_ctr + k2[0]) << 2);
            w1 = v2[1] | (key(t.n_ctr + k2[1]) << 2);
        } else {
            other2(e.y, e.z, e.w & 0xFFFFu, e.w >> 16, w0, w1, (o_at | o_late) != 0u);
        }
        put(e.x, w0, w1);
    }
}

template <int kMode, int kList, int kD, bool kO4>
void launch_pair_d(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                   uint32_t* out, uint64_t stride, uint32_t* oq, uint32_t oq_cap, const uint32_t* slot_rule,
                   uint32_t ctr_base, uint32_t wbytes, uint32_t lq_cap, bool o_late, uint32_t cdiv,
                   const PairMap& sm, const LaunchCfg& cfg) {
    const uint32_t q_lds = pair_queue_lds(t.img_bytes, o_at, o.img_bytes, o_late);   // the waves' LDS segments
    const size_t lds = std::max<size_t>(q_lds + size_t(lq_cap) * 16u * (kPairBlock / 64),
                                        sm.srl ? sm.srl + 16u * sm.n16 : 0u);
    lds_attr<classify4_pair<kMode, kList, kD, kO4>>();
    hipLaunchKernelGGL((classify4_pair<kMode, kList, kD, kO4>), dim3(cfg.grid), dim3(kClsBlock), lds, cfg.stream, t, o,
                       o_at, p, sport, out, stride, oq, oq_cap, q_lds, slot_rule, ctr_base, wbytes, lq_cap,
                       o_late ? 1u : 0u, cdiv, sm.map, sm.srl, sm.n16);
}

// sublist modes: the search depth as a template argument (the rendered
// global tables' one-length hash, as the hot classify kernel)
template <int kMode, int kList, bool kO4>
void launch_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p, const uint16_t* sport,
                 uint32_t* out, uint64_t stride, uint32_t* oq, uint32_t oq_cap, const uint32_t* slot_rule,
                 uint32_t ctr_base, uint32_t wbytes, uint32_t lq_cap, bool o_late, uint32_t cdiv,
                 const PairMap& sm, const LaunchCfg& cfg) {
    if constexpr (kMode == 2 && (kList == 3 || kList == 4)) {
        switch (t.bv_steps) {
        case 0: launch_pair_d<kMode, kList, 0, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        case 1: launch_pair_d<kMode, kList, 1, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        case 2: launch_pair_d<kMode, kList, 2, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        case 3: launch_pair_d<kMode, kList, 3, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        case 4: launch_pair_d<kMode, kList, 4, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        case 5: launch_pair_d<kMode, kList, 5, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, sm, cfg); return;
        default: break;
        }
    }
    launch_pair_d<kMode, kList, -1, kO4>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv,
                                    sm, cfg);
}

}  // namespace

hipError_t launch_classify4_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p,
                                 const uint16_t* sport, uint32_t* out, uint64_t stride, uint32_t* oq,
                                 uint32_t oq_cap, const uint32_t* slot_rule, uint32_t ctr_base, uint32_t wbytes,
                                 uint32_t lq_cap, bool o_late, uint32_t cdiv, bool o4, const PairMap& sm,
                                 const LaunchCfg& cfg) {
    if (!cls_dispatchable(t, true, false) || (!o4 && (o.mode != 0 || o.list_mode != 0))) return hipErrorInvalidValue;
    const int src = src_variant(t);
#define PAIR_CASE(S, M, L) \
    case 8 * S + L: \
        if (o4) launch_pair<M, L, true>(t, o, 0u, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, false, 0u, sm, cfg); \
        else launch_pair<M, L, false>(t, o, o_at, p, sport, out, stride, oq, oq_cap, slot_rule, ctr_base, wbytes, lq_cap, o_late, cdiv, PairMap{}, cfg); \
        break;
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
