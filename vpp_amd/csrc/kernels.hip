// gfx950 kernels of the batched first-match ACL classifier: the finish,
// stream-floor, linear, connection and traffic kernels and their launchers.
// The classify kernels (kernels_dev.hpp) are instantiated by k4_lds.hip,
// k4_glb.hip and k16.hip.
#include <cstdlib>

#include "kernels_dev.hpp"

namespace cls {

namespace {

// The classify kernels' HBM stream without the lookups (bench.py's measured
// floor): the same loads and stores, in the same order, on the same grid;
// the verdict is a mix of the packet's fields.
template <bool kPf, bool kNtPr>
__global__ __launch_bounds__(kClsBlock) void stream4_kernel(Pkts4 p, uint8_t* verdict) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nsteps = uint32_t(p.n / 4u);
    const uint4* S = reinterpret_cast<const uint4*>(p.src);
    const uint4* D = reinterpret_cast<const uint4*>(p.dst);
    const uint2* DP = reinterpret_cast<const uint2*>(p.dport);
    const uint32_t* PR = reinterpret_cast<const uint32_t*>(p.proto);
    struct Buf {
        uint4 s, d;
        uint2 dp;
        uint32_t pr;
    };
    auto load = [&](Buf& b, uint32_t g) {
        if (g < nsteps) {
            b.s = ldnt(at(S, g)); b.d = ldnt(at(D, g)); b.dp = ldnt(at(DP, g));
            b.pr = kNtPr ? ldnt(at(PR, g)) : *at(PR, g);
        }
    };
    auto step = [&](const Buf& b, uint32_t g) {
        const uint32_t v = (b.s.x ^ b.d.x ^ b.s.y ^ b.d.y ^ b.s.z ^ b.d.z ^ b.s.w ^ b.d.w ^ b.dp.x ^ b.dp.y ^ b.pr) &
                           0x03030303u;
        stnt(v, const_cast<uint32_t*>(at(reinterpret_cast<const uint32_t*>(verdict), g)));
    };
    if constexpr (kPf) {
        // as classify4_cls: whole grid steps with unconditional (clamped)
        // loads, so the next step's loads stay in flight; the rest after
        const uint32_t nfull = nsteps / nthreads * nthreads;
        auto loadc = [&](Buf& b, uint32_t g) {
            const uint32_t gi = min(g, nfull - 1u);
            b.s = ldnt(at(S, gi)); b.d = ldnt(at(D, gi)); b.dp = ldnt(at(DP, gi));
            b.pr = kNtPr ? ldnt(at(PR, gi)) : *at(PR, gi);
        };
        if (nfull) {
            Buf a, b;
            uint32_t g = tid;
            loadc(a, g);
            while (g < nfull) {
                loadc(b, g + nthreads);
                step(a, g);
                g += nthreads;
                if (g >= nfull) break;
                loadc(a, g + nthreads);
                step(b, g);
                g += nthreads;
            }
        }
        for (uint32_t g = nfull + tid; g < nsteps; g += nthreads) {
            Buf a;
            load(a, g);
            step(a, g);
        }
    } else {
        for (uint32_t g = tid; g < nsteps; g += nthreads) {
            Buf a;
            load(a, g);
            step(a, g);
        }
    }
}

__global__ __launch_bounds__(kClsBlock) void stream16_kernel(Pkts16 p, uint8_t* verdict) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nsteps = uint32_t(p.n / 256u) * 64u;
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        const uint32_t base = 4u * (g & ~63u) + (g & 63u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 s = ldnt(at(p.src, base + 64u * k)), d = ldnt(at(p.dst, base + 64u * k));
            const uint32_t dp = __builtin_nontemporal_load(p.dport + base + 64u * k);
            const uint32_t pr = __builtin_nontemporal_load(p.proto + base + 64u * k);
            __builtin_nontemporal_store(uint8_t((s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp ^ pr) & 3u),
                                        verdict + base + 64u * k);
        }
    }
}

// The connection batch's HBM stream without the evaluation (the connection
// path's floor, cls_stream_floor_conn): the 22 bytes of an IPv4 connection
// (src, dst, src_if, dst_if: 16-B loads; sport, dport: 8-B; proto: 4-B) read
// and its verdict byte written, 4 connections per lane.
__global__ __launch_bounds__(1024) void stream_conn_kernel(const uint4* src, const uint4* dst, const uint4* sif,
                                                           const uint4* dif, const uint2* sp, const uint2* dp,
                                                           const uint32_t* pr, uint32_t* out, uint32_t nsteps) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nsteps; g += gridDim.x * blockDim.x) {
        const uint4 a = ldnt(at(src, g)), b = ldnt(at(dst, g)), c = ldnt(at(sif, g)), d = ldnt(at(dif, g));
        const uint2 e = ldnt(at(sp, g)), f = ldnt(at(dp, g));
        const uint32_t p = ldnt(at(pr, g));
        const uint32_t v = (a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^
                            d.w ^ e.x ^ e.y ^ f.x ^ f.y ^ p) & 0x03030303u;
        stnt(v, const_cast<uint32_t*>(at(reinterpret_cast<const uint32_t*>(out), g)));
    }
}

constexpr uint32_t kOtherLds = 4096;   // finish launch: LDS histogram of the OTHER packets' rules

// One launch at the end of a classify call (kernels.hpp FinishArgs).  Blocks
// [0, ntile): 64 slots each -- the 16 waves sum the workgroups' partial rows
// (rows w, w + 16, ...: 256 contiguous bytes per load instruction), wave 0
// adds the slot's global counter and moves the total to its rule (hot rules:
// summed in LDS over the tile first, one atomic per tile).  Blocks after:
// one classify workgroup's OTHER queue segments each (its waves' packets),
// every lane on one packet, counted per rule in LDS (compact rule indices)
// and added once per (block, rule).  No block waits for another: the OTHER
// packets are counted straight into their rules, the tiles read only what
// the classify launch wrote.
constexpr uint32_t kFoldWaves = 16;
// A tile's rows may be split over f.split blocks (the host's fold_split),
// their sums added to the rules with device atomics: a few tiles each
// walking every row of a many-workgroup launch wait one memory latency per
// 64 rows.
__device__ __forceinline__ uint32_t fold_split(const FinishArgs& f) { return f.remap && f.part ? max(f.split, 1u) : 1u; }
template <typename Load>
__device__ __forceinline__ void finish_body(const FinishArgs& f, const Cls4Dev& o, uint8_t* verdict,
                                            const Load& load) {
    __shared__ unsigned long long acc[kFoldWaves][64];
    __shared__ unsigned long long hot[kMaxHotRules];
    __shared__ uint32_t h[kOtherLds];
    const uint32_t span = f.remap ? f.n_slots : (f.part ? f.n_lctr : 0u);
    const uint32_t split = fold_split(f);
    const uint32_t ntile = (span + 63u) / 64u * split;
    if (blockIdx.x < ntile) {
        const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
        const uint32_t piece = blockIdx.x % split;                 // this block's rows of the tile
        const uint32_t i = blockIdx.x / split * 64u + lane;
        if (threadIdx.x < f.n_hot) hot[threadIdx.x] = 0ull;
        unsigned long long s64 = 0;
        if (f.part && i < f.n_lctr) {
            const uint32_t n = f.n_lctr, per = (f.rows + split - 1u) / split;
            const uint32_t rows = min(f.rows, (piece + 1u) * per);
            const uint32_t* part = f.part;
            uint32_t w = piece * per + wave;
            for (; w + 3u * kFoldWaves < rows; w += 4u * kFoldWaves) {
                const uint32_t a = part[size_t(w) * n + i], b = part[size_t(w + kFoldWaves) * n + i];
                const uint32_t c = part[size_t(w + 2u * kFoldWaves) * n + i];
                const uint32_t d = part[size_t(w + 3u * kFoldWaves) * n + i];
                s64 += (unsigned long long)a + b + c + d;
            }
            for (; w < rows; w += kFoldWaves) s64 += part[size_t(w) * n + i];
        }
        acc[wave][lane] = s64;
        __syncthreads();
        if (wave == 0 && i < span) {
#pragma unroll
            for (uint32_t k = 1; k < kFoldWaves; ++k) s64 += acc[k][lane];
            if (f.remap) {
                if (piece == 0u) {                   // the slot's global counter: one block
                    const unsigned long long sv = f.slot_val[i];
                    if (sv) f.slot_val[i] = 0ull;
                    s64 += sv;
                }
                if (s64) {
                    const uint32_t e = f.slot_rule[i];
                    if (e & kHotRule) atomicAdd(&hot[e & ~kHotRule], s64);
                    else atomicAdd(&f.out[e], s64);
                }
            } else if (s64) {
                f.slot_val[i] += s64;            // an earlier chunk: this launch is the only writer
            }
        }
        __syncthreads();
        if (threadIdx.x < f.n_hot && hot[threadIdx.x])
            atomicAdd(&f.out[f.slot_rule[f.n_slots + threadIdx.x]], hot[threadIdx.x]);
        return;
    }
    const uint32_t r = blockIdx.x - ntile;
    if (!f.oq || r >= f.oq_rows) return;
    // the classify workgroup's kOtherSegs wave segments, taken as one list
    uint32_t cnt[kOtherSegs], n = 0;
#pragma unroll
    for (uint32_t w = 0; w < kOtherSegs; ++w) {
        cnt[w] = f.oq[r * kOtherSegs + w];
        n += cnt[w];
    }
    if (n == 0) return;                          // the usual case: no OTHER packet in this row
    const bool lds = f.n_orules <= kOtherLds;
    if (lds) {
        for (uint32_t i = threadIdx.x; i < f.n_orules; i += blockDim.x) h[i] = 0u;
        __syncthreads();
    }
    const Img<false> oim{reinterpret_cast<const uint8_t*>(o.img)};
    const uint32_t* orule = f.other_map + f.n_other;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t w = 0, at = i;
        while (at >= cnt[w]) at -= cnt[w++];     // i < n: stops inside a non-empty segment
        const uint32_t e = f.oq[f.oq_rows * kOtherSegs + (r * kOtherSegs + w) * f.oq_cap + at];
        // one packet, or (qmask) the packets 4 g + q of the entry's mask
        uint32_t mask = f.qmask ? e >> 28 : 1u;
        const uint32_t kb = f.qmask ? (e & 0x0FFFFFFFu) << 2 : e;
        while (mask) {
            const uint32_t k = kb + (f.qmask ? uint32_t(__builtin_ctz(mask)) : 0u);
            mask &= mask - 1u;
            uint32_t s1[1], d1[1], p1[1];
            load(k, s1[0], d1[0], p1[0]);
            const uint32_t z1[1] = {0u};
            uint32_t r1[1], k1[1];
            classify_n<1, false, 0, 0, -1>(oim, o, s1, d1, p1, z1, r1, k1);
            if (verdict) verdict[k] = uint8_t(r1[0]);
            const uint32_t c = f.other_map[k1[0]];
            if (lds) atomicAdd(&h[c], 1u);
            else wave_count(f.out, orule[c]);
        }
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < f.n_orules; i += blockDim.x)
            if (h[i]) atomicAdd(&f.out[orule[i]], (unsigned long long)h[i]);
    }
}

__global__ __launch_bounds__(1024) void finish4_kernel(FinishArgs f, Cls4Dev o, Pkts4 p, uint8_t* verdict) {
    finish_body(f, o, verdict, [&](uint32_t k, uint32_t& s, uint32_t& d, uint32_t& dp) {
        s = p.src[k];
        d = p.dst[k];
        dp = p.dport[k];
    });
}

// finish for 16-byte batches: the OTHER packets' reps from the front end in
// global memory (the image's copy; src_mode 1: the source interval table).
__global__ __launch_bounds__(1024) void finish16_kernel(FinishArgs f, Cls4Dev t, Cls4Dev o, Fe16 fe, Pkts16 p,
                                                       uint8_t* verdict) {
    const Img<false> gim{reinterpret_cast<const uint8_t*>(t.img)};
    finish_body(f, o, verdict, [&](uint32_t k, uint32_t& s, uint32_t& d, uint32_t& dp) {
        const uint4 s16[1] = {p.src[k]}, d16[1] = {p.dst[k]};
        uint32_t s1[1], d1[1];
        if (fe.src_mode >= 1) s1[0] = src_rep_global(fe.gsrc, fe.gval, fe.gtop, fe.gk8, s16[0]);
        else fe_rep(gim, fe.key[0], fe.val[0], fe.top[0], fe.k8[0], s16, s1);
        fe_rep(gim, fe.key[1], fe.val[1], fe.top[1], fe.k8[1], d16, d1);
        s = s1[0];
        d = d1[0];
        dp = p.dport[k];
    });
}

// slot_val[i] += the sum over the grid's rows of part[w][i], i < n: block b
// takes slots [64 b, 64 b + 64), wave w of its 16 the rows w, w + 16, ...
// (256 contiguous bytes per load instruction), then one wave adds the 16
// partial sums -- a plain read-modify-write, this launch being the only
// writer.  Blocks past the slot range zero `zero` (the call's rule counters):
// no separate memset launch.
__global__ __launch_bounds__(1024) void fold_kernel(const uint32_t* __restrict__ part, uint32_t rows, uint32_t n,
                                                    unsigned long long* __restrict__ slot_val,
                                                    unsigned long long* __restrict__ zero, uint32_t n_zero) {
    const uint32_t nb = (n + 63u) / 64u;
    if (blockIdx.x >= nb) {
        const uint32_t i = (blockIdx.x - nb) * blockDim.x + threadIdx.x;
        if (i < n_zero) zero[i] = 0ull;
        return;
    }
    __shared__ unsigned long long acc[kFoldWaves][64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 64u + lane;
    unsigned long long s64 = 0;
    if (i < n) {
        uint32_t w = wave;
        for (; w + 3u * kFoldWaves < rows; w += 4u * kFoldWaves) {
            const uint32_t a = part[size_t(w) * n + i], b = part[size_t(w + kFoldWaves) * n + i];
            const uint32_t c = part[size_t(w + 2u * kFoldWaves) * n + i];
            const uint32_t d = part[size_t(w + 3u * kFoldWaves) * n + i];
            s64 += (unsigned long long)a + b + c + d;
        }
        for (; w < rows; w += kFoldWaves) s64 += part[size_t(w) * n + i];
    }
    acc[wave][lane] = s64;
    __syncthreads();
    if (wave == 0 && i < n) {
#pragma unroll
        for (uint32_t k = 1; k < kFoldWaves; ++k) s64 += acc[k][lane];
        if (s64) slot_val[i] += s64;
    }
}

// rule_out (cls_classify_rules): each packet's terminating rule instead of
// the counters.
__global__ __launch_bounds__(kBlock) void classify4_linear(const LinRule4* __restrict__ rules,
                                                           uint32_t nr, uint32_t n_rules, Pkts4 p,
                                                           uint8_t* verdict,
                                                           unsigned long long* gslot, uint32_t* rule_out) {
    __shared__ uint32_t lctr[kLinLdsCounters];
    const bool lds = n_rules + 1 <= kLinLdsCounters && !rule_out;
    if (lds) {
        for (uint32_t i = threadIdx.x; i <= n_rules; i += blockDim.x) lctr[i] = 0u;
        __syncthreads();
    }
    const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t n_iter = (p.n + nthreads - 1) / nthreads;  // uniform trip count
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (uint64_t it = 0; it < n_iter; ++it) {
        const uint64_t i = it * nthreads + tid;
        const bool live = i < p.n;
        uint32_t s = 0, d = 0, dp = 0, pr = 0;
        if (live) { s = p.src[i]; d = p.dst[i]; dp = p.dport[i]; pr = p.proto[i]; }
        const uint32_t pi = pr <= 2u ? pr : 3u;
        bool done = !live;
        uint32_t res = 0, rule = n_rules;
        for (uint32_t r = 0; r < nr; ++r) {
            // wave-uniform rule: scalar loads
            const uint32_t sa = rules[r].src_addr, sm = rules[r].src_mask;
            const uint32_t da = rules[r].dst_addr, dm = rules[r].dst_mask;
            const uint32_t meta = rules[r].meta;
            const uint32_t pw = rules[r].port[pi];
            const uint32_t m = (meta >> (8 * pi)) & 0xFFu;
            if (!done && (m & 0x80u) && ((s ^ sa) & sm) == 0 && ((d ^ da) & dm) == 0 &&
                port_in(dp, pw)) {
                done = true;
                res = m & 3u;
                rule = rules[r].index;
            }
            if (__ballot(!done) == 0ull) break;   // every lane resolved: leave the scan
        }
        if (live) {
            if (verdict) verdict[i] = uint8_t(res);
            if (rule_out) rule_out[i] = rule;
            else if (lds) atomicAdd(&lctr[rule], 1u);
            else atomicAdd(&gslot[rule], 1ull);
        }
    }
    if (lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i <= n_rules; i += blockDim.x) {
            const uint32_t v = lctr[i];
            if (v) atomicAdd(&gslot[i], (unsigned long long)v);
        }
    }
}

// Slot-mode words -> each packet's ACLAction and terminating rule
// (cls_classify_rules): word = result | slot << 2, slot_rule = the image's
// slot -> rule map (the OTHER image's slots after the main image's); rule
// may alias words (each element is read before it is written).
__global__ __launch_bounds__(256) void slot_rules_kernel(const uint32_t* words, const uint32_t* __restrict__ slot_rule,
                                                         uint32_t n, uint8_t* __restrict__ verdict, uint32_t* rule) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t w = words[i];
        if (verdict) verdict[i] = uint8_t(w & 3u);
        rule[i] = slot_rule[w >> 2];
    }
}

// Slot counters -> rule counters, read and cleared (slot_val is all zero
// between calls).  csr: every slot once, grouped by rule, entry {slot, rule}.
// A wave sums the values of each run of equal rules among its 64 entries
// (suffix sums over the lanes) and the run's first lane adds the total: one
// atomic per (wave, rule).  out == nullptr: clear only.
__global__ __launch_bounds__(256) void remap_kernel(unsigned long long* __restrict__ slot_val,
                                                    const uint2* __restrict__ csr, uint32_t n,
                                                    unsigned long long* __restrict__ out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rule = 0xFFFFFFFFu;
    unsigned long long v = 0;
    if (k < n) {
        const uint2 e = csr[k];
        rule = e.y;
        v = slot_val[e.x];
        if (v) slot_val[e.x] = 0ull;
    }
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long w = __shfl_down(v, d);
        const uint32_t r2 = __shfl_down(rule, d);
        if (lane + uint32_t(d) < 64u && r2 == rule) v += w;
    }
    const uint32_t prev = __shfl_up(rule, 1);
    if (out && k < n && v && (lane == 0 || prev != rule)) atomicAdd(&out[rule], v);
}

// ---------------------------------------------------------------------------
// Connection batches: testConnection (aclengine_mock.go:394-471), one lane per
// connection, persistent grid.  Up to four evalACL calls per connection, in
// the reference's order and with its REFLECT short-cuts: SYN through the
// source interface's inbound then the destination's outbound ACL with
// (src, dst, dport); SYN-ACK through the destination's inbound then the
// source's outbound ACL with (dst, src, sport).  An ACL the host evaluated
// with the classifier (slot mode, both tuples of every connection) is read
// from its slot words; the others are scanned from the call's rule pool of
// compact rules (compile.hpp ConnRule4 / ConnRule16), staged in LDS when it
// fits -- every lane may scan a different ACL, so the scans are divergent,
// but LDS serves them without the global-memory latency of each step.
// Counting (CLS_F_COUNT): the terminating rule of every call made on a
// non-nil ACL -> the call's counter space (descriptor ctr_off + rule), in LDS
// (u32, folded into the u64 counters at the end) or with wave-aggregated
// global atomics.

template <bool k16> struct ConnT;
template <> struct ConnT<false> {
    typedef uint32_t A;
    typedef ConnRule4 R;
};
template <> struct ConnT<true> {
    typedef uint4 A;
    typedef ConnRule16 R;
};

template <bool kLds>
__device__ __forceinline__ ConnRule4 conn_rule(const ConnRule4* g, uint32_t i) {
    if constexpr (kLds) {                      // the pool at LDS address 0: two ds_read_b128
        const uint32_t a = i * uint32_t(sizeof(ConnRule4));
        const v4u x = *lds128_t(a), y = *lds128_t(a + 16u);
        ConnRule4 r;
        r.src_addr = x.x; r.src_mask = x.y; r.dst_addr = x.z; r.dst_mask = x.w;
        r.port[0] = y.x; r.port[1] = y.y; r.meta = y.z; r.index = y.w;
        return r;
    } else {
        return g[i];
    }
}
template <bool kLds>
__device__ __forceinline__ ConnRule16 conn_rule(const ConnRule16* g, uint32_t i) {
    if constexpr (kLds) {
        const uint32_t a = i * uint32_t(sizeof(ConnRule16));
        v4u w[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) w[k] = *lds128_t(a + 16u * k);
        ConnRule16 r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r.src[k] = w[0][k]; r.smask[k] = w[1][k]; r.dst[k] = w[2][k]; r.dmask[k] = w[3][k];
        }
        r.port[0] = w[4].x; r.port[1] = w[4].y; r.meta = w[4].z; r.index_fam = w[4].w;
        return r;
    } else {
        return g[i];
    }
}
__device__ __forceinline__ bool conn_match(const ConnRule4& r, uint32_t s, uint32_t d, bool, bool) {
    return (((s ^ r.src_addr) & r.src_mask) | ((d ^ r.dst_addr) & r.dst_mask)) == 0u;
}
// s4 / d4: the address is IPv4-mapped (Go's To4 succeeds)
__device__ __forceinline__ bool conn_match(const ConnRule16& r, const uint4& s, const uint4& d, bool s4, bool d4) {
    const uint32_t x = ((s.x ^ r.src[0]) & r.smask[0]) | ((s.y ^ r.src[1]) & r.smask[1]) |
                       ((s.z ^ r.src[2]) & r.smask[2]) | ((s.w ^ r.src[3]) & r.smask[3]) |
                       ((d.x ^ r.dst[0]) & r.dmask[0]) | ((d.y ^ r.dst[1]) & r.dmask[1]) |
                       ((d.z ^ r.dst[2]) & r.dmask[2]) | ((d.w ^ r.dst[3]) & r.dmask[3]);
    const uint32_t fam = r.index_fam & 3u;
    return x == 0u && !((fam & 1u) && s4) && !((fam & 2u) && d4);
}
__device__ __forceinline__ uint32_t conn_index(const ConnRule4& r) { return r.index; }
__device__ __forceinline__ uint32_t conn_index(const ConnRule16& r) { return r.index_fam >> 2; }
__device__ __forceinline__ bool mapped4(const uint4& a) { return (a.x | a.y) == 0u && a.z == 0xFFFF0000u; }

// The call's descriptor and interface tables: staged in LDS at a.meta_lds
// (descriptors, then the interfaces) when they fit, else read from global
// memory (a.meta_lds == ~0u; uniform branch).  Staged, a connection's
// interface and descriptor reads are LDS reads instead of dependent global
// loads in front of every evaluation.
template <bool kMeta = false>    // kMeta: the tables are in LDS (the kernel variant knows it)
__device__ __forceinline__ IfAcls conn_if(const ConnArgs& a, uint32_t j) {
    if (kMeta || a.meta_lds != 0xFFFFFFFFu) {
        const v4u v = *lds128_t(a.meta_lds + a.n_desc * uint32_t(sizeof(ConnDesc)) + 16u * j);
        return IfAcls{int32_t(v.x), int32_t(v.y), int32_t(v.z), int32_t(v.w)};
    }
    return a.ifs[j];
}
template <bool kMeta = false>
__device__ __forceinline__ ConnDesc conn_desc(const ConnArgs& a, uint32_t j) {
    if (kMeta || a.meta_lds != 0xFFFFFFFFu) {
        const uint32_t b = a.meta_lds + j * uint32_t(sizeof(ConnDesc));
        const v4u x = *lds128_t(b), y = *lds128_t(b + 16u);
        ConnDesc d;
        d.rule_off = x.x; d.n = x.y; d.n_rules = x.z; d.ctr_off = x.w;
        d.pre_blk = int32_t(y.x); d.pad = y.y;
        d.slot_rule = reinterpret_cast<const uint32_t*>(uint64_t(y.z) | (uint64_t(y.w) << 32));
        const v4u z = *lds128_t(b + 32u);
        d.bm_off = z.x; d.bm_sd = z.y; d.bm_tu = z.z; d.bm_w = z.w;
        return d;
    }
    return a.desc[j];
}

// The linear scan of one evalACL call over an ACL of the rule pool: ACLAction
// and the terminating rule (R: default DENY, aclengine_mock.go:667).
template <bool k16, bool kLds>
__device__ __forceinline__ uint32_t conn_scan(const ConnArgs& a, const ConnDesc& D,
                                              const typename ConnT<k16>::A& s, const typename ConnT<k16>::A& d,
                                              bool s4, bool d4, uint32_t port, uint32_t p, uint32_t& rule) {
    typedef typename ConnT<k16>::R R;
    const R* g = static_cast<const R*>(a.rules);
    uint32_t res = 0u;
    rule = D.n_rules;
    for (uint32_t r = 0; r < D.n; ++r) {
        const R x = conn_rule<kLds>(g, D.rule_off + r);
        const uint32_t meta = (x.meta >> (8u * p)) & 0xFFu;
        const uint32_t pw = p == 0u ? x.port[0] : p == 1u ? x.port[1] : 0xFFFF0000u;   // ICMP / OTHER: any port
        if ((meta & 0x80u) && conn_match(x, s, d, s4, d4) && port_in(port, pw)) {
            res = meta & 3u;
            rule = conn_index(x);
            break;
        }
    }
    return res;
}

// One evalACL call on the bitmap form of an IPv4 ACL (kernels.hpp
// kConnBmHeader; engine.cpp conn_bitmap4): three interval searches (source,
// destination, the protocol's destination port; ICMP and OTHER have one
// interval) give three bit rows, and the lowest bit set in all three is the
// first rule that matches -- the scan's answer in a fixed number of reads,
// so the lanes of a wave no longer wait for the longest scan among them.
template <bool kLds>
__device__ __forceinline__ uint32_t bm_u32(const uint8_t* g, uint32_t a) {
    if constexpr (kLds) return *lds32_t(a);
    else return *reinterpret_cast<const uint32_t*>(g + a);
}
template <bool kLds>
__device__ __forceinline__ uint32_t conn_bm(const ConnArgs& a, const ConnDesc& D, uint32_t s, uint32_t d,
                                            uint32_t port, uint32_t p, uint32_t& rule) {
    const uint8_t* g = static_cast<const uint8_t*>(a.rules);
    const uint32_t W = D.bm_w, ns = D.bm_sd & 0xFFFFu, nd = D.bm_sd >> 16;
    const uint32_t n0 = D.bm_tu & 0xFFFFu, n1 = D.bm_tu >> 16;
    // the tables: src, dst, then the protocol tables (n2 = n3 = 1), then the rules
    const uint32_t os = D.bm_off + kConnBmHeader, od = os + 4u * ns * (1u + W), t0 = od + 4u * nd * (1u + W);
    const uint32_t t1 = t0 + 4u * n0 * (1u + W), t2 = t1 + 4u * n1 * (1u + W), t3 = t2 + 4u * (1u + W);
    const uint32_t orl = t3 + 4u * (1u + W);
    const uint32_t op = p == 0u ? t0 : p == 1u ? t1 : p == 2u ? t2 : t3;
    const uint32_t np = p == 0u ? n0 : p == 1u ? n1 : 1u;
    // the three branch-free lower bounds (last key <= x; key 0 first) in
    // lock-step, their reads in flight together: a finished search re-reads
    // its current key (h = 0), which still holds.  The trip count is the
    // launch's (a.bm_steps, the largest table's), the same for every lane: a
    // loop on each lane's own lengths costs the wave exec-mask work per trip
    uint32_t ps = 0, ls = ns, pd = 0, ld = nd, pp = 0, lp = np;
    for (uint32_t it = 0; it < a.bm_steps; ++it) {
        const uint32_t hs = ls >> 1, hd = ld >> 1, hp = lp >> 1;
        const uint32_t ks = bm_u32<kLds>(g, os + 4u * (ps + hs)), kd = bm_u32<kLds>(g, od + 4u * (pd + hd));
        const uint32_t kp = bm_u32<kLds>(g, op + 4u * (pp + hp));
        ps = ks <= s ? ps + hs : ps;
        pd = kd <= d ? pd + hd : pd;
        pp = kp <= port ? pp + hp : pp;
        ls -= hs; ld -= hd; lp -= hp;
    }
    const uint32_t sr = os + 4u * ns + 4u * W * ps, dr = od + 4u * nd + 4u * W * pd, pr = op + 4u * np + 4u * W * pp;
    for (uint32_t w = 0; w < W; ++w) {
        const uint32_t m = bm_u32<kLds>(g, sr + 4u * w) & bm_u32<kLds>(g, dr + 4u * w) & bm_u32<kLds>(g, pr + 4u * w);
        if (m) {
            const uint32_t i = 32u * w + uint32_t(__builtin_ctz(m));
            rule = bm_u32<kLds>(g, orl + 8u * i + 4u);
            return (bm_u32<kLds>(g, orl + 8u * i) >> (8u * p)) & 3u;
        }
    }
    rule = D.n_rules;
    return 0u;
}

// testConnection, one lane per connection, in two phases per iteration.
//
// 1. Evaluations.  A call on a large ACL reads the classifier's result word
//    for this connection (classify4_pair / the slot launches); a call on a
//    linear ACL is a *job*: the bitmap search (IPv4, conn_bm) or the rule
//    scan.  The jobs of all four possible calls of the wave's 64 connections
//    are packed (ranks from the calls' ballots, no LDS) and run 64 at a time,
//    every lane on one job with its connection's fields fetched from the
//    owning lane (ds_bpermute).  A lane-per-call loop would make the wave run the
//    search once per call index in which any of its lanes has a job -- four
//    passes per wave with ~0.6 jobs per connection -- where packing runs
//    one.  (Running a call index most lanes need in place, without the
//    shuffles, measured slower: 84 -> 90 us at 12 local ACLs, 192 -> 234 us
//    at 64, profiles/r04k_conn_dense_calls_ab.txt.)  Jobs are evaluated
//    whether or not testConnection reaches the call (the call order needs
//    the earlier results); only the calls it makes are counted.
// 2. The state machine: testConnection's order and REFLECT short-cuts
//    (aclengine_mock.go:394-471) over the four results: SYN through the
//    source's inbound then the destination's outbound ACL, SYN-ACK through
//    the destination's inbound then the source's outbound ACL.
//
// Counting (CLS_F_COUNT): the terminating rule of every call made on a
// non-nil ACL -> the call's counter space (descriptor ctr_off + rule), in LDS
// (u32, folded into the u64 counters at the end) or with wave-aggregated
// global atomics.
// Workgroup size (launch_connect): the kernel holds ~80 VGPRs (6 waves per
// SIMD), so 24 waves fit a CU -- three 512-thread workgroups where the LDS
// allows, else two 768-thread ones where it allows those (the bench's
// counted plan at 12 local ACLs: 88 -> 75 us, profiles/r06w768_*), else two
// 512-thread ones or one 1024-thread workgroup (16 waves rather than the 8
// of one 512-thread one); forcing 64 VGPRs spills to scratch.  The
// 16-byte LDS-counter variants (kCount 1, k16) take up to 128 VGPRs (at 80
// they spill) and at most two 512-thread workgroups per CU (the host's plan);
// the IPv4 ones fit 80 since the job ranks came from mbcnt (round 6: 89 with
// a lane mask held in registers), so they get the third workgroup wherever
// the LDS allows it.  (640-thread workgroups, 5 waves per SIMD, measured 125
// against 88 us: the second workgroup finds no SIMD with room for its third
// wave -- profiles/r06e_conn_tree_search_ab.txt.)
// kJobs (IPv4): the waves' job lists in LDS (a.job_lds); else the owner
// search and shuffles (16-byte batches, and IPv4 launches whose LDS is
// full: the job lists would displace LDS counters or bitmap forms)
// testConnection's order over the four call results (res: ACLAction of
// the SYN src-inbound, SYN dst-outbound, SYN-ACK dst-inbound and SYN-ACK
// src-outbound calls; a nil ACL's is PERMIT) and its REFLECT short-cuts
// (aclengine_mock.go:394-471): the verdict | the calls made << 2.  same: the
// two interfaces are one; !ok: an unknown interface (Failure, no calls).
__device__ __forceinline__ uint32_t conn_state(const uint32_t res[4], bool same, bool ok) {
    uint32_t v = 3u;                                                        // Failure (unknown interface)
    bool made[4];
    uint32_t r = res[0];                                                    // SYN: src inbound
    made[0] = ok;
    bool done = ok && (r == 3u || r == 0u);
    v = ok && r == 3u ? 3u : ok && r == 0u ? 0u : v;
    bool srefl = ok && r == 2u, drefl = srefl && same;
    made[1] = ok && !done && !drefl;                                        // SYN: dst outbound
    r = res[1];
    v = made[1] && r == 3u ? 3u : made[1] && r == 0u ? 0u : v;
    done = done || (made[1] && (r == 3u || r == 0u));
    const bool dr1 = made[1] && r == 2u;
    drefl = drefl || dr1;
    srefl = srefl || (dr1 && same);
    made[2] = ok && !done && !drefl;                                        // SYN-ACK: dst inbound
    r = res[2];
    v = made[2] && r == 3u ? 3u : made[2] && r == 0u ? 1u : v;
    done = done || (made[2] && (r == 3u || r == 0u));
    made[3] = ok && !done && !srefl;                                        // SYN-ACK: src outbound
    r = res[3];
    v = made[3] && r == 3u ? 3u : made[3] && r == 0u ? 1u : v;
    done = done || (made[3] && (r == 3u || r == 0u));
    v = ok && !done ? 2u : v;
    return v | uint32_t(made[0]) << 2 | uint32_t(made[1]) << 3 | uint32_t(made[2]) << 4 | uint32_t(made[3]) << 5;
}

template <bool k16, bool kLdsRules, int kCount, bool kJobs>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(kCount == 1 && k16 ? 4 : 6))) void connect_kernel(
    ConnArgs a) {
    typedef typename ConnT<k16>::A A;
    extern __shared__ uint4 smem[];
    typedef __attribute__((address_space(3))) uint32_t* lctr_t;
    const uint32_t lane = __lane_id();
    // 32-bit connection indices (the host splits batches at 2^30): SGPR base
    // + 32-bit VGPR offset addressing, no 64-bit index arithmetic per load
    const uint32_t n = uint32_t(a.n);
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t n_iter = (n + nthreads - 1u) / nthreads;     // uniform trip count (ballots below)
    const uint32_t stride = uint32_t(a.pre_stride);
    if constexpr (kLdsRules) lds_copy(smem, static_cast<const uint4*>(a.rules), a.rules_bytes / 16u);
    if constexpr (kCount == 1) {
        const uint32_t nw = a.ctr16 ? (a.n_ctr + 1u) / 2u : a.n_ctr;
        for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) *lctr_t(a.ctr_lds + 4u * j) = 0u;
    }
    // this workgroup's copy of the call counters
    unsigned long long* const gctr = a.ctr + uint64_t(blockIdx.x % kConnCtrCopies) * a.n_ctr;
    // the state machine's table (kConnStateEntries bytes): entry res0 | res1
    // << 2 | res2 << 4 | res3 << 6 | same << 8 | !ok << 9
    for (uint32_t x = threadIdx.x; x < kConnStateEntries; x += blockDim.x) {
        const uint32_t r4[4] = {x & 3u, (x >> 2) & 3u, (x >> 4) & 3u, (x >> 6) & 3u};
        *reinterpret_cast<__attribute__((address_space(3))) uint8_t*>(a.sm_lds + x) =
            uint8_t(conn_state(r4, (x >> 8) & 1u, !((x >> 9) & 1u)));
    }
    if (a.meta_lds != 0xFFFFFFFFu) {
        const uint32_t nd = a.n_desc * uint32_t(sizeof(ConnDesc)) / 4u;
        const uint32_t* gd = reinterpret_cast<const uint32_t*>(a.desc);
        const uint32_t* gi = reinterpret_cast<const uint32_t*>(a.ifs);
        for (uint32_t j = threadIdx.x; j < nd; j += blockDim.x) *lctr_t(a.meta_lds + 4u * j) = gd[j];
        for (uint32_t j = threadIdx.x; j < 4u * a.n_ifs; j += blockDim.x) *lctr_t(a.meta_lds + 4u * (nd + j)) = gi[j];
    }
    __syncthreads();
    const A* src = static_cast<const A*>(a.src);
    const A* dst = static_cast<const A*>(a.dst);
    // IPv4: this wave's job list in LDS, 64 entries of 8 B {owner lane | call
    // << 6 | descriptor << 8, port | protocol << 16}; a job's lane writes its
    // result word over the entry's first word
    const uint32_t jq = __builtin_amdgcn_readfirstlane(a.job_lds + (threadIdx.x >> 6) * 512u);
    for (uint32_t it = 0; it < n_iter; ++it) {
        const uint32_t i = it * nthreads + blockIdx.x * blockDim.x + threadIdx.x;
        const bool live = i < n;
        const uint32_t ic = live ? i : 0u;                      // loads stay in bounds
        // every field's load first, together -- with the large ACLs' result
        // words when there are at most kConnEarlyBlocks of them (wave-uniform)
        uint32_t si, dj, sp, dp, pr;
        A sa, da;
        // (u8 / u16 words, packed: one register per block)
        const bool early = a.n_big == 0u || (a.n_big <= kConnEarlyBlocks && a.pre_bytes <= 2u);
        uint32_t ew[kConnEarlyBlocks] = {};                    // [block]: SYN | SYN-ACK << (8 or 16)
        {
            si = *at(a.src_if, ic);
            dj = *at(a.dst_if, ic);
            sa = *at(src, ic);
            da = *at(dst, ic);
            sp = *at(a.sport, ic);
            dp = *at(a.dport, ic);
            pr = *at(a.proto, ic);
            if (early) {
#pragma unroll
                for (uint32_t b = 0; b < kConnEarlyBlocks; ++b)
                    if (b < a.n_big) {
                        if (a.pre_bytes == 1u) ew[b] = reinterpret_cast<const uint8_t*>(a.pre)[uint64_t(b) * stride + ic];
                        else ew[b] = a.pre[uint64_t(b) * stride + ic];      // SYN | SYN-ACK << 16
                    }
            }
        }
        const bool ok = live && si < a.n_ifs && dj < a.n_ifs;   // unknown interface id: Failure
        // both lookups unconditional (an in-range index), the unknown case selected after
        const IfAcls S0 = conn_if(a, ok ? si : 0u), D0 = conn_if(a, ok ? dj : 0u);
        const IfAcls S = ok ? S0 : IfAcls{-1, -1, -1, -1};
        const IfAcls Dif = ok ? D0 : IfAcls{-1, -1, -1, -1};
        const uint32_t p = pr <= 2u ? pr : 3u;
        // the four calls in testConnection's order
        const int32_t di[4] = {S.in, Dif.out, Dif.in, S.out};
        const int32_t bi[4] = {S.in_pre, Dif.out_pre, Dif.in_pre, S.out_pre};
        // result words of the calls on large ACLs, loaded together (a call
        // without one reads a valid dummy word: unconditional loads measured
        // faster than the same loads under a branch)
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            w[k] = early ? ((bi[k] == 1 ? ew[1] : ew[0]) >> ((k >> 1) * (a.pre_bytes == 1u ? 2u : 16u))) &
                               (a.pre_bytes == 1u ? 0xFFu : 0xFFFFu)
                 : a.pre_bytes == 1u
                       ? uint32_t(*(bi[k] >= 0 ? reinterpret_cast<const uint8_t*>(a.pre) + uint64_t(uint32_t(bi[k])) * stride + ic
                                               : reinterpret_cast<const uint8_t*>(a.src_if) + ic)) >> (2 * (k >> 1))
                   : a.pre_bytes == 2u
                       ? (*(bi[k] >= 0 ? a.pre + uint64_t(uint32_t(bi[k])) * stride + ic : at(a.src_if, ic)) >>
                          (16u * uint32_t(k >> 1))) & 0xFFFFu
                       : *(bi[k] >= 0 ? a.pre + (uint64_t(2u * uint32_t(bi[k]) + uint32_t(k >> 1)) * stride + ic)
                                      : at(a.src_if, ic));
        // ---- the jobs of the wave, packed ----
        // job j of the wave is call k of owner lane o: the ballots of the four
        // calls give every job a rank; the jobs run 64 at a time, every lane
        // on one job
        // The jobs of the calls with a linear ACL.  When they need more than
        // one pass of the wave (more than 64), the calls that are never made
        // are dropped first: the SYN calls' large-ACL results end the
        // evaluation on DENY or FAILURE, and conn_state leaves calls 2 and 3
        // unmade after a terminal call 0 or 1 whether or not call 1 itself
        // was made (a REFLECT of call 0 on one interface skips all three);
        // call 2's result is not used (a REFLECT of call 1 skips call 2 but
        // not call 3).  At 64 local ACLs: 2.27 -> 1.98 passes per wave,
        // connect_kernel 154 -> 135 us (profiles/r06y_conn_skip_ab.txt); at
        // 12 one pass either way, and the test costs nothing there.
        bool job[4];
        uint64_t m[4];
        uint32_t c[5], jpos[4];
        auto pack = [&](bool skip) {
            c[0] = 0;
            bool ended = false;                                 // a large SYN result ended the evaluation
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                job[k] = di[k] >= 0 && bi[k] < 0 && !ended;
                if (skip) ended = ended || (k < 2 && bi[k] >= 0 && ((w[k] + 1u) & 3u) <= 1u);   // DENY 0, FAILURE 3
                m[k] = __ballot(job[k]);
                // (the set bits of m[k] below this lane: mbcnt, no lane mask held in registers)
                jpos[k] = c[k] + __builtin_amdgcn_mbcnt_hi(uint32_t(m[k] >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m[k]), 0u));
                c[k + 1] = c[k] + uint32_t(__popcll(m[k]));
            }
        };
        pack(false);
        if (c[4] > 64u) pack(true);                             // wave-uniform
        const uint32_t nj = c[4];
        uint32_t rj[4] = {0u, 0u, 0u, 0u};
        for (uint32_t j0 = 0; j0 < nj; j0 += 64u) {             // wave-uniform
            const uint32_t j = j0 + lane;
            const bool act = j < nj;
            uint32_t out = 0u;
            if constexpr (kJobs) {
                // IPv4: the owners write their jobs into the wave's LDS list
                // (entry = rank - j0), the lane of a rank reads its entry and
                // takes the owner's addresses with two shuffles -- where a
                // search of the ballots for the owner (nth_set_bit) and nine
                // shuffles cost ~60 VALU instructions per pass
                typedef __attribute__((address_space(3))) v2u* lds64w_t;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (job[k] && jpos[k] - j0 < 64u)
                        *lds64w_t(jq + 8u * (jpos[k] - j0)) =
                            v2u{lane | uint32_t(k) << 6 | uint32_t(di[k]) << 8, (k < 2 ? dp : sp) | (p << 16)};
                const v2u e = *lds64_t(jq + 8u * lane);
                const uint32_t o = act ? (e.x & 63u) : lane, kk = (e.x >> 6) & 3u;
                const uint32_t xs = __shfl(uint32_t(sa), int(o)), xd = __shfl(uint32_t(da), int(o));
                if (act) {
                    const ConnDesc D = conn_desc(a, e.x >> 8);
                    const uint32_t port = e.y & 0xFFFFu, xp = e.y >> 16;
                    const uint32_t s1 = kk < 2u ? xs : xd, d1 = kk < 2u ? xd : xs;
                    uint32_t res, rule;
                    if (D.bm_off != 0xFFFFFFFFu) res = conn_bm<kLdsRules>(a, D, s1, d1, port, xp, rule);
                    else res = conn_scan<false, kLdsRules>(a, D, A(s1), A(d1), true, true, port, xp, rule);
                    out = res | ((D.ctr_off + rule) << 2);
                }
                // the result over the entry's first word, then the owners read it
                if (act) *(__attribute__((address_space(3))) uint32_t*)(jq + 8u * lane) = out;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (job[k] && jpos[k] - j0 < 64u)
                        rj[k] = *(const __attribute__((address_space(3))) uint32_t*)(jq + 8u * (jpos[k] - j0));
            } else {
                const uint32_t k = uint32_t(j >= c[1]) + uint32_t(j >= c[2]) + uint32_t(j >= c[3]);
                const uint64_t mk = k == 0u ? m[0] : k == 1u ? m[1] : k == 2u ? m[2] : m[3];
                const uint32_t ck = k == 0u ? c[0] : k == 1u ? c[1] : k == 2u ? c[2] : c[3];
                const uint32_t o = act ? nth_set_bit(mk, j - ck) : lane;
                // the owning lane's connection (every lane takes part in the shuffles)
                A xs, xd;
                if constexpr (k16) {
                    xs = make_uint4(__shfl(sa.x, int(o)), __shfl(sa.y, int(o)), __shfl(sa.z, int(o)), __shfl(sa.w, int(o)));
                    xd = make_uint4(__shfl(da.x, int(o)), __shfl(da.y, int(o)), __shfl(da.z, int(o)), __shfl(da.w, int(o)));
                } else {
                    xs = __shfl(sa, int(o));
                    xd = __shfl(da, int(o));
                }
                const uint32_t xdp = __shfl(dp, int(o)), xsp = __shfl(sp, int(o)), xp = __shfl(p, int(o));
                const int32_t d0 = __shfl(di[0], int(o)), d1 = __shfl(di[1], int(o));
                const int32_t d2 = __shfl(di[2], int(o)), d3 = __shfl(di[3], int(o));
                if (act) {
                    const ConnDesc D = conn_desc(a, uint32_t(k == 0u ? d0 : k == 1u ? d1 : k == 2u ? d2 : d3));
                    const bool syn = k < 2u;
                    uint32_t res, rule;
                    if constexpr (!k16) {
                        if (D.bm_off != 0xFFFFFFFFu)
                            res = conn_bm<kLdsRules>(a, D, syn ? xs : xd, syn ? xd : xs, syn ? xdp : xsp, xp, rule);
                        else
                            res = conn_scan<false, kLdsRules>(a, D, syn ? xs : xd, syn ? xd : xs, true, true,
                                                              syn ? xdp : xsp, xp, rule);
                    } else {
                        const bool x4s = mapped4(xs), x4d = mapped4(xd);
                        res = syn ? conn_scan<k16, kLdsRules>(a, D, xs, xd, x4s, x4d, xdp, xp, rule)
                                  : conn_scan<k16, kLdsRules>(a, D, xd, xs, x4d, x4s, xsp, xp, rule);
                    }
                    out = res | ((D.ctr_off + rule) << 2);
                }
                // the owners take their results of this pass
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const uint32_t r = __shfl(out, int((jpos[kk] - j0) & 63u));
                    if (job[kk] && jpos[kk] >= j0 && jpos[kk] < j0 + 64u) rj[kk] = r;
                }
            }
        }
        // ---- testConnection over the four results ----
        uint32_t res[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) res[k] = di[k] < 0 ? 1u : job[k] ? (rj[k] & 3u) : (w[k] & 3u);   // nil ACL: PERMIT (:476-478)
        // the state machine from the workgroup's table: one LDS byte for the
        // verdict and the calls made (a ~60-instruction select chain per lane
        // otherwise)
        const uint32_t sm = *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
            a.sm_lds + (res[0] | res[1] << 2 | res[2] << 4 | res[3] << 6 | uint32_t(si == dj) << 8 |
                        uint32_t(!ok) << 9));
        const uint32_t v = sm & 3u;
        bool made[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) made[k] = (sm >> (2 + k)) & 1u;
        if (live) a.out[i] = uint8_t(v);
        if constexpr (kCount != 0) {
            uint32_t key[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                key[k] = 0xFFFFFFFFu;
                if (made[k] && di[k] >= 0) {                    // nil ACLs are not counted
                    if (job[k]) {
                        key[k] = rj[k] >> 2;
                    } else if (a.pre_rules) {            // a large ACL: the word's counter index
                        key[k] = w[k] >> 2;
                    } else {                                    // ... or its slot's rule
                        const ConnDesc D = conn_desc(a, uint32_t(di[k]));
                        key[k] = D.ctr_off + D.slot_rule[w[k] >> 2];
                    }
                }
            }
            if constexpr (kCount == 1) {
                // (aggregating a wave's equal keys first measured slower:
                // 136.5 -> 142.5 us at 12 local ACLs, profiles/r04l_conn_ab.txt)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t kk = key[k], add = 1u;
                    if (kk != 0xFFFFFFFFu)
                        __hip_atomic_fetch_add(lctr_t(a.ctr_lds + 4u * (a.ctr16 ? kk >> 1 : kk)),
                                               a.ctr16 ? add << (16u * (kk & 1u)) : add, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) wave_count(gctr, key[k]);
            }
        }
    }
    if constexpr (kCount == 1) {
        __syncthreads();
        if (a.ctr_rows) {
            // the words as this workgroup's row: plain coalesced stores, summed
            // by the rows launch (device atomics from every workgroup at the
            // end of the launch serialise per address)
            const uint32_t nw = a.ctr16 ? (a.n_ctr + 1u) / 2u : a.n_ctr;
            uint32_t* row = a.ctr_rows + uint64_t(blockIdx.x) * nw;
            for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) row[j] = *lctr_t(a.ctr_lds + 4u * j);
        } else if (a.ctr16) {
            for (uint32_t j = threadIdx.x; j < (a.n_ctr + 1u) / 2u; j += blockDim.x) {
                const uint32_t c = *lctr_t(a.ctr_lds + 4u * j);
                if (c & 0xFFFFu) atomicAdd(&gctr[2u * j], (unsigned long long)(c & 0xFFFFu));
                if (c >> 16) atomicAdd(&gctr[2u * j + 1u], (unsigned long long)(c >> 16));
            }
        } else {
            for (uint32_t j = threadIdx.x; j < a.n_ctr; j += blockDim.x) {
                const uint32_t c = *lctr_t(a.ctr_lds + 4u * j);
                if (c) atomicAdd(&gctr[j], (unsigned long long)c);
            }
        }
    }
}

// The call's counters -> the tables' connection counters, cleared for the
// next call (so the call counters stay zero between calls).  Workgroup
// (x, y): descriptor x (a table has one descriptor per call), counters
// 256 y .. 256 y + 255 -- one counter per thread, not a loop per table.
__global__ __launch_bounds__(256) void conn_scatter_kernel(const ConnDesc* __restrict__ desc,
                                                           unsigned long long* const* __restrict__ table_ctr,
                                                           unsigned long long* __restrict__ call_ctr,
                                                           uint32_t n_slabs, uint32_t clear, uint32_t n_ctr) {
    const ConnDesc D = desc[blockIdx.x];
    const uint32_t r = blockIdx.y * blockDim.x + threadIdx.x;
    if (r > D.n_rules) return;
    unsigned long long v = 0;
#pragma unroll 16
    for (uint32_t c = 0; c < n_slabs; ++c) {                // the slabs: copies or partial sums
        unsigned long long* p = call_ctr + uint64_t(c) * n_ctr + D.ctr_off + r;
        const unsigned long long x = *p;
        v += x;
        if (clear && x) *p = 0ull;
    }
    if (v) atomicAdd(&table_ctr[blockIdx.x][r], v);
}

// Rows -> the tables' connection counters: thread (word w, slab g) sums word
// w over rows g kConnRowsPerSlab .. + kConnRowsPerSlab - 1 (the loads in
// flight together, coalesced over w) and adds each nonzero counter of the
// word to its table's counter (the descriptor found by bisection over the
// ascending counter bases) -- at most one add per slab and counter.
__device__ __forceinline__ void conn_ctr_add(const ConnDesc* __restrict__ desc, uint32_t n_desc,
                                             unsigned long long* const* __restrict__ table_ctr, uint32_t c,
                                             unsigned long long v) {
    uint32_t lo = 0, hi = n_desc;                    // the last descriptor with ctr_off <= c
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (desc[mid].ctr_off <= c) lo = mid;
        else hi = mid;
    }
    atomicAdd(&table_ctr[lo][c - desc[lo].ctr_off], v);
}
__global__ __launch_bounds__(256) void conn_rows_kernel(const uint32_t* __restrict__ rows, uint32_t n_rows,
                                                        uint32_t nw, uint32_t ctr16, uint32_t n_ctr,
                                                        const ConnDesc* __restrict__ desc, uint32_t n_desc,
                                                        unsigned long long* const* __restrict__ table_ctr) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    const uint32_t r0 = blockIdx.y * kConnRowsPerSlab;
    uint32_t x[kConnRowsPerSlab];
#pragma unroll
    for (uint32_t k = 0; k < kConnRowsPerSlab; ++k) x[k] = r0 + k < n_rows ? rows[uint64_t(r0 + k) * nw + w] : 0u;
    unsigned long long lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < kConnRowsPerSlab; ++k) {
        lo += ctr16 ? (x[k] & 0xFFFFu) : x[k];
        hi += x[k] >> 16;
    }
    if (ctr16) {
        if (lo) conn_ctr_add(desc, n_desc, table_ctr, 2u * w, lo);
        if (hi && 2u * w + 1u < n_ctr) conn_ctr_add(desc, n_desc, table_ctr, 2u * w + 1u, hi);
    } else if (lo) {
        conn_ctr_add(desc, n_desc, table_ctr, w, lo);
    }
}


constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += kGolden;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void gen4_kernel(TrafficDev t, uint64_t first, uint64_t n, uint32_t* src,
                            uint32_t* dst, uint16_t* sport, uint16_t* dport, uint8_t* proto) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n; k += stride) {
        const uint64_t i = first + k;
        uint64_t w[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) w[j] = mix64(t.seed ^ ((8ull * i + uint64_t(j)) * kGolden));
        const uint32_t a0 = uint32_t(w[0]), b0 = uint32_t(w[0] >> 32);
        uint8_t pr;
        if (a0 % 100u < t.pct_icmp) pr = 2;
        else pr = (b0 & 1u) ? 1 : 0;
        uint32_t s;
        if (t.n_pods && ((b0 >> 1) % 100u) < t.pct_pod) s = t.pods[uint32_t(w[1] >> 32) % t.n_pods];
        else s = uint32_t(w[1]);
        const uint32_t a2 = uint32_t(w[2]), b2 = uint32_t(w[2] >> 32);
        uint32_t d;
        if (t.n_dst && (a2 % 100u) < t.pct_dst) {
            const uint32_t j = b2 % t.n_dst;
            const uint32_t len = t.dst_lens[j];
            const uint32_t mask = len ? (0xFFFFFFFFu << (32 - len)) : 0u;
            d = (t.dst_addrs[j] & mask) | (uint32_t(w[3]) & ~mask);
        } else {
            d = uint32_t(w[3]);
        }
        const uint32_t a4 = uint32_t(w[4]), b4 = uint32_t(w[4] >> 32);
        uint16_t dp;
        if (t.n_ports && (a4 % 100u) < t.pct_port) dp = t.ports[b4 % t.n_ports];
        else dp = uint16_t(w[5]);
        const uint16_t sp = uint16_t(1024u + (uint32_t(w[5] >> 32) % 64512u));
        if (src) src[k] = s;
        if (dst) dst[k] = d;
        if (sport) sport[k] = sp;
        if (dport) dport[k] = dp;
        if (proto) proto[k] = pr;
    }
}

// (hi, lo) address -> the 16 network-order bytes as stored (little-endian words)
__device__ __forceinline__ uint4 store16(uint64_t hi, uint64_t lo) {
    return make_uint4(__builtin_bswap32(uint32_t(hi >> 32)), __builtin_bswap32(uint32_t(hi)),
                      __builtin_bswap32(uint32_t(lo >> 32)), __builtin_bswap32(uint32_t(lo)));
}

__global__ void gen16_kernel(TrafficDev16 t, uint64_t first, uint64_t n, uint4* src, uint4* dst,
                             uint16_t* sport, uint16_t* dport, uint8_t* proto) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t fd00 = 0xFD00ull << 48, mapped = 0xFFFFull << 32;
    for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n; k += stride) {
        const uint64_t i = first + k;
        uint64_t w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = mix64(t.seed ^ ((8ull * i + uint64_t(j)) * kGolden));
        const uint32_t a0 = uint32_t(w[0]), b0 = uint32_t(w[0] >> 32);
        uint8_t pr;
        if (a0 % 100u < t.pct_icmp) pr = 2;
        else pr = (b0 & 1u) ? 1 : 0;
        uint64_t sh, sl;
        const uint32_t b1 = uint32_t(w[1] >> 32);
        if (t.n_pods && ((b0 >> 1) % 100u) < t.pct_pod) {
            const uint32_t j = b1 % t.n_pods;
            sh = t.pods[2 * j];
            sl = t.pods[2 * j + 1];
        } else if (b1 & 1u) {
            sh = fd00; sl = w[6];
        } else {
            sh = 0; sl = mapped | uint32_t(w[1]);
        }
        const uint32_t a2 = uint32_t(w[2]), b2 = uint32_t(w[2] >> 32);
        uint64_t dh, dl;
        if (t.n_dst && (a2 % 100u) < t.pct_dst) {
            const uint32_t j = b2 % t.n_dst;
            const uint32_t len = t.dst_lens[j];
            const uint64_t mh = len == 0 ? 0ull : len >= 64 ? ~0ull : ~0ull << (64 - len);
            const uint64_t ml = len <= 64 ? 0ull : len >= 128 ? ~0ull : ~0ull << (128 - len);
            dh = (t.dst_addrs[2 * j] & mh) | (w[3] & ~mh);
            dl = (t.dst_addrs[2 * j + 1] & ml) | (w[7] & ~ml);
        } else if (b2 & 1u) {
            dh = fd00; dl = w[7];
        } else {
            dh = 0; dl = mapped | uint32_t(w[3]);
        }
        const uint32_t a4 = uint32_t(w[4]), b4 = uint32_t(w[4] >> 32);
        uint16_t dp;
        if (t.n_ports && (a4 % 100u) < t.pct_port) dp = t.ports[b4 % t.n_ports];
        else dp = uint16_t(w[5]);
        const uint16_t sp = uint16_t(1024u + (uint32_t(w[5] >> 32) % 64512u));
        if (src) src[k] = store16(sh, sl);
        if (dst) dst[k] = store16(dh, dl);
        if (sport) sport[k] = sp;
        if (dport) dport[k] = dp;
        if (proto) proto[k] = pr;
    }
}

}  // namespace

int max_lds_bytes() { return kLdsMax; }
int cls_block() { return kClsBlock; }

hipError_t launch_classify4_linear(const LinRule4* rules, uint32_t n_lin, uint32_t n_rules,
                                   const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                                   const LaunchCfg& cfg, uint32_t* rule_out) {
    hipLaunchKernelGGL(classify4_linear, dim3(cfg.grid), dim3(kBlock), 0, cfg.stream, rules, n_lin,
                       n_rules, p, verdict, gslot, rule_out);
    return hipGetLastError();
}

hipError_t launch_slot_rules(const uint32_t* words, const uint32_t* slot_rule, uint32_t n, uint8_t* verdict,
                             uint32_t* rule, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t grid = std::min<uint32_t>((n + 255u) / 256u, 8192u);
    hipLaunchKernelGGL(slot_rules_kernel, dim3(grid), dim3(256), 0, s, words, slot_rule, n, verdict, rule);
    return hipGetLastError();
}

hipError_t launch_fold(const uint32_t* part, uint32_t rows, uint32_t n, unsigned long long* slot_val,
                       unsigned long long* zero, uint32_t n_zero, hipStream_t s) {
    if (rows == 0) n = 0;
    if (!zero) n_zero = 0;
    const uint32_t blocks = (n + 63u) / 64u + (n_zero + 1023u) / 1024u;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(fold_kernel, dim3(blocks), dim3(1024), 0, s, part, rows, n, slot_val, zero, n_zero);
    return hipGetLastError();
}

hipError_t launch_remap(unsigned long long* slot_val, const uint2* csr, uint32_t n, unsigned long long* out,
                        hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(remap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slot_val, csr, n, out);
    return hipGetLastError();
}

static uint32_t finish_grid(const FinishArgs& f) {
    const uint32_t span = f.remap ? f.n_slots : (f.part ? f.n_lctr : 0u);
    return (span + 63u) / 64u * (f.remap && f.part ? std::max(f.split, 1u) : 1u) + (f.oq ? f.oq_rows : 0u);
}

hipError_t launch_finish4(const FinishArgs& f, const Cls4Dev& o, const Pkts4& p, uint8_t* verdict, hipStream_t s) {
    const uint32_t g = finish_grid(f);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(finish4_kernel, dim3(g), dim3(1024), 0, s, f, o, p, verdict);
    return hipGetLastError();
}

hipError_t launch_finish16(const FinishArgs& f, const Cls4Dev& t, const Cls4Dev& o, const Fe16& fe, const Pkts16& p,
                           uint8_t* verdict, hipStream_t s) {
    const uint32_t g = finish_grid(f);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(finish16_kernel, dim3(g), dim3(1024), 0, s, f, t, o, fe, p, verdict);
    return hipGetLastError();
}

hipError_t launch_stream(const Pkts4* p4, const Pkts16* p16, uint8_t* verdict, int grid, int variant,
                         hipStream_t s) {
    if (p4) {
        switch (variant) {
        case 0: hipLaunchKernelGGL((stream4_kernel<true, true>), dim3(grid), dim3(kClsBlock), 0, s, *p4, verdict); break;
        case 1: hipLaunchKernelGGL((stream4_kernel<false, true>), dim3(grid), dim3(kClsBlock), 0, s, *p4, verdict); break;
        case 2: hipLaunchKernelGGL((stream4_kernel<true, false>), dim3(grid), dim3(kClsBlock), 0, s, *p4, verdict); break;
        default: hipLaunchKernelGGL((stream4_kernel<false, false>), dim3(grid), dim3(kClsBlock), 0, s, *p4, verdict);
        }
    } else {
        hipLaunchKernelGGL(stream16_kernel, dim3(grid), dim3(kClsBlock), 0, s, *p16, verdict);
    }
    return hipGetLastError();
}

hipError_t launch_stream_conn(const ConnArgs& a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(stream_conn_kernel, dim3(grid), dim3(1024), 0, s, static_cast<const uint4*>(a.src),
                       static_cast<const uint4*>(a.dst), reinterpret_cast<const uint4*>(a.src_if),
                       reinterpret_cast<const uint4*>(a.dst_if), reinterpret_cast<const uint2*>(a.sport),
                       reinterpret_cast<const uint2*>(a.dport), reinterpret_cast<const uint32_t*>(a.proto),
                       reinterpret_cast<uint32_t*>(a.out), uint32_t(a.n / 4u));
    return hipGetLastError();
}

hipError_t launch_connect(const ConnArgs& a, bool k16, bool lds_rules, int count, int grid, int block, size_t lds,
                          hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const bool jobs = a.job_lds != 0xFFFFFFFFu;
#define CONN_CASE(K16, L, C, J)                                                                            \
    if (k16 == K16 && lds_rules == L && count == C && jobs == J) {                                         \
        lds_attr<connect_kernel<K16, L, C, J>>();                                                          \
        hipLaunchKernelGGL((connect_kernel<K16, L, C, J>), dim3(grid), dim3(block), lds, s, a);            \
        return hipGetLastError();                                                                          \
    }
    CONN_CASE(false, false, 0, true) CONN_CASE(false, false, 1, true) CONN_CASE(false, false, 2, true)
    CONN_CASE(false, true, 0, true) CONN_CASE(false, true, 1, true) CONN_CASE(false, true, 2, true)
    CONN_CASE(false, false, 0, false) CONN_CASE(false, false, 1, false) CONN_CASE(false, false, 2, false)
    CONN_CASE(false, true, 0, false) CONN_CASE(false, true, 1, false) CONN_CASE(false, true, 2, false)
    CONN_CASE(true, false, 0, false) CONN_CASE(true, false, 1, false) CONN_CASE(true, false, 2, false)
    CONN_CASE(true, true, 0, false) CONN_CASE(true, true, 1, false) CONN_CASE(true, true, 2, false)
#undef CONN_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_conn_rows(const uint32_t* rows, uint32_t n_rows, uint32_t nw, bool ctr16, uint32_t n_ctr,
                            const ConnDesc* desc, uint32_t n_desc, unsigned long long* const* table_ctr,
                            hipStream_t s) {
    if (n_rows == 0 || nw == 0 || n_desc == 0) return hipSuccess;
    hipLaunchKernelGGL(conn_rows_kernel, dim3((nw + 255u) / 256u, (n_rows + kConnRowsPerSlab - 1u) / kConnRowsPerSlab),
                       dim3(256), 0, s, rows, n_rows, nw, ctr16 ? 1u : 0u, n_ctr, desc, n_desc, table_ctr);
    return hipGetLastError();
}

hipError_t launch_conn_scatter(const ConnDesc* desc, unsigned long long* const* table_ctr, uint32_t n_desc,
                               uint32_t max_rules, unsigned long long* call_ctr, uint32_t n_slabs, bool clear,
                               uint32_t n_ctr, hipStream_t s) {
    if (n_desc == 0) return hipSuccess;
    hipLaunchKernelGGL(conn_scatter_kernel, dim3(n_desc, max_rules / 256u + 1u), dim3(256), 0, s, desc, table_ctr,
                       call_ctr, n_slabs, clear ? 1u : 0u, n_ctr);
    return hipGetLastError();
}

hipError_t launch_gen16(const TrafficDev16& t, uint64_t first, uint64_t n, uint4* src, uint4* dst,
                        uint16_t* sport, uint16_t* dport, uint8_t* proto, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen16_kernel, dim3(uint32_t(blocks)), dim3(256), 0, s, t, first, n, src, dst, sport,
                       dport, proto);
    return hipGetLastError();
}

hipError_t launch_gen4(const TrafficDev& t, uint64_t first, uint64_t n, uint32_t* src,
                       uint32_t* dst, uint16_t* sport, uint16_t* dport, uint8_t* proto,
                       hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen4_kernel, dim3(uint32_t(blocks)), dim3(256), 0, s, t, first, n, src, dst,
                       sport, dport, proto);
    return hipGetLastError();
}

}  // namespace cls
