// gfx950 kernels of the batched first-match ACL classifier.
//
// classify4_cls  -- the hot path.  Persistent grid-stride kernel; every
//   workgroup stages the read-only classifier image (compile.hpp, Cls4Image)
//   into LDS once with 16-B loads, zeroes its LDS slot counters, then streams
//   packets: 4 packets per lane per step with 16-B (src, dst), 8-B (dport) and
//   4-B (proto) coalesced loads and one 4-B verdict store.  Per packet:
//   branch-free binary search of the source boundaries (LDS) -> class ->
//   (class, protocol) cell -> scan of the cell's candidate templates (dst
//   prefix + port range) to the first match.  One LDS atomic per packet
//   counts the terminating slot; counters are flushed to global u64 slots
//   once per workgroup.  Integer compare work only -- no MFMA.
// classify4_linear -- the ballot kernel: every lane walks the rule list in
//   order with wave-uniform (scalar) rule loads and the wave leaves as soon
//   as the ballot of unfinished lanes is empty.  Small tables, GPU cross-check,
//   and the protocol>2 fallback of classify4_cls.
// connect4 -- testConnection (aclengine_mock.go:394-471) for a batch.
// gen4 -- the counter-based splitmix64 traffic stream, generated in HBM.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace cls {

namespace {

constexpr int kBlock = 1024;
constexpr int kLdsMax = 160 * 1024;
constexpr uint32_t kLinLdsCounters = 16384;  // linear kernel: LDS counters up to R+1 <= this

__device__ __forceinline__ bool port_in(uint32_t dport, uint32_t pw) {
    return ((dport - (pw & 0xFFFFu)) & 0xFFFFu) <= (pw >> 16);
}

// first match over the linear rule list for one lane (protocol > 2 fallback)
__device__ __forceinline__ void linear_one(const LinRule4* __restrict__ rules, uint32_t nr,
                                           uint32_t n_rules, uint32_t src, uint32_t dst,
                                           uint32_t dport, uint32_t p, uint32_t& res,
                                           uint32_t& rule) {
    res = 0;
    rule = n_rules;
    for (uint32_t r = 0; r < nr; ++r) {
        const LinRule4& R = rules[r];
        const uint32_t meta = (R.meta >> (8 * p)) & 0xFFu;
        if ((meta & 0x80u) && ((src ^ R.src_addr) & R.src_mask) == 0 &&
            ((dst ^ R.dst_addr) & R.dst_mask) == 0 && port_in(dport, R.port[p])) {
            res = meta & 3u;
            rule = R.index;
            return;
        }
    }
}

// Source class of N packets, interleaved (N independent LDS chains per lane).
template <int N, int kMode>
__device__ __forceinline__ void src_class(const uint8_t* base, const Cls4Dev& t,
                                          const uint32_t (&src)[N], uint32_t (&cls)[N]) {
    if constexpr (kMode == 1) {
        // hash LPM: one cuckoo probe pair per prefix length, lengths ascending so
        // the longest hit wins
#pragma unroll
        for (int q = 0; q < N; ++q) cls[q] = t.default_class;
        // Constant indices into the kernel arguments: the parameters are loaded
        // into SGPRs once, outside the packet loop.  (A runtime index would
        // re-issue s_load + s_waitcnt lgkmcnt(0) every step, which also drains
        // the previous step's LDS counter atomics.)
#pragma unroll
        for (uint32_t i = 0; i < kMaxHashLens; ++i) {
            if (i >= t.n_hash) break;
            const uint2* __restrict__ tab = reinterpret_cast<const uint2*>(base + t.off_hash[i]);
            const uint32_t mask = t.hash_mask[i], shift = t.hash_shift[i], cap = t.hash_cap[i];
            uint2 e0[N], e1[N];
            uint32_t key[N];
#pragma unroll
            for (int q = 0; q < N; ++q) {
                key[q] = src[q] & mask;
                e0[q] = tab[lpm_h0(key[q], shift)];
                e1[q] = tab[cap + lpm_h1(key[q], shift)];
            }
#pragma unroll
            for (int q = 0; q < N; ++q) {
                // empty slots hold keys that never probe them: a key compare is
                // the whole hit test (two compares, two selects)
                cls[q] = e1[q].x == key[q] ? e1[q].y : cls[q];
                cls[q] = e0[q].x == key[q] ? e0[q].y : cls[q];
            }
        }
    } else {
        // branch-free binary search over the padded interval boundaries
        const uint32_t* __restrict__ b = reinterpret_cast<const uint32_t*>(base + t.off_bounds);
        uint32_t k[N];
#pragma unroll
        for (int q = 0; q < N; ++q) k[q] = 0;
#pragma unroll 1
        for (uint32_t s = t.search_top; s; s >>= 1) {
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint32_t c = k[q] + s;
                k[q] = (b[c] <= src[q]) ? c : k[q];
            }
        }
        const uint16_t* __restrict__ ic = reinterpret_cast<const uint16_t*>(base + t.off_iclass);
#pragma unroll
        for (int q = 0; q < N; ++q) cls[q] = ic[k[q]];
    }
}

// First match of N packets (protocols 0-2) against their cells' candidate
// lists.  The N scans advance in lockstep with predication: a finished packet
// keeps re-reading a valid entry instead of branching, so the lane issues N
// independent LDS reads per step.
template <int N, int kMode, int kList>
__device__ __forceinline__ void classify_n(const uint8_t* base, const Cls4Dev& t,
                                           const uint32_t (&src)[N], const uint32_t (&dst)[N],
                                           const uint32_t (&dport)[N], const uint32_t (&proto)[N],
                                           uint32_t (&res)[N], uint32_t (&slot)[N]) {
    uint32_t pc[N];
    if constexpr (kList == 2) {
        // global port class (list mode 2): top[port >> 8] = sub-table offset |
        // base class << 20, class = base + sub[port & 255].  Independent of the
        // source lookup: these reads go out together with the hash probes.
        const uint32_t* __restrict__ ptop = reinterpret_cast<const uint32_t*>(base + t.off_ptop);
        uint32_t tp[N];
#pragma unroll
        for (int q = 0; q < N; ++q) tp[q] = ptop[dport[q] >> 8];
#pragma unroll
        for (int q = 0; q < N; ++q) pc[q] = (tp[q] >> 20) + base[(tp[q] & 0xFFFFFu) + (dport[q] & 0xFFu)];
    }
    uint32_t cls[N];
    if (t.ablate & 4u) {
#pragma unroll
        for (int q = 0; q < N; ++q) cls[q] = src[q] & 1u;
    } else {
        src_class<N, kMode>(base, t, src, cls);
    }
    const uint2* __restrict__ cells = reinterpret_cast<const uint2*>(base + t.off_cells);
    if constexpr (kList >= 1) {
        // Bit vectors: the entries of the cell's list that cover the packet's
        // dst interval AND its port interval; the first such entry (lowest
        // set bit) is the first match of the ordered list.  Both interval
        // searches are branch-free, t.bv_steps steps for every lane, and
        // track the byte address of the current interval: the step sizes
        // are compile-time constants (unrolled, uniform guard), so a probe
        // is one ds_read_b64 {bound, mask} with an immediate offset (b64 and
        // b32 reads cost the same LDS cycles on gfx950: 2 x 32 lanes).
        // cell = dst array offset / 8 | counter base << 16; an array is 2^S
        // {bound, mask} pairs, the port array follows the dst array; the bound
        // word of entry 0 (never probed) holds the result bits, lo / hi
        const uint32_t* __restrict__ cells1 = reinterpret_cast<const uint32_t*>(base + t.off_cells);
        const uint32_t S = t.bv_steps;
        uint32_t cb[N], ad[N], ap[N], rlo[N], rhi[N], md[N], mp[N];
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t cell = cells1[cls[q] * 3u + min(proto[q], 2u)];
            cb[q] = cell >> 16;
            ad[q] = (cell & 0xFFFFu) * 8u;
            ap[q] = ad[q] + (8u << S);
        }
        if constexpr (kList == 1) {
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint2 d0 = *reinterpret_cast<const uint2*>(base + ad[q]);
                const uint2 p0 = *reinterpret_cast<const uint2*>(base + ap[q]);
                rlo[q] = d0.x;
                md[q] = d0.y;
                rhi[q] = p0.x;
                mp[q] = p0.y;
            }
        } else {
            // mode 2: after the dst array, the result-hi word and one mask per
            // global port class
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint2 d0 = *reinterpret_cast<const uint2*>(base + ad[q]);
                rlo[q] = d0.x;
                md[q] = d0.y;
                mp[q] = *reinterpret_cast<const uint32_t*>(base + ap[q] + 4u + pc[q] * 4u);
                rhi[q] = 0u;
            }
            if (t.bv_wide) {
#pragma unroll
                for (int q = 0; q < N; ++q) rhi[q] = *reinterpret_cast<const uint32_t*>(base + ap[q]);
            }
        }
        if (!(t.ablate & 2u)) {
#pragma unroll
            for (int i = int(kMaxBvSteps) - 1; i >= 0; --i) {
                if (uint32_t(i) >= S) continue;
                const uint32_t step = 8u << i;
#pragma unroll
                for (int q = 0; q < N; ++q) {
                    const uint2 ed = *reinterpret_cast<const uint2*>(base + ad[q] + step);
                    const bool td = ed.x <= dst[q];
                    ad[q] = td ? ad[q] + step : ad[q];
                    md[q] = td ? ed.y : md[q];
                    if constexpr (kList == 1) {
                        const uint2 ep = *reinterpret_cast<const uint2*>(base + ap[q] + step);
                        const bool tp = ep.x <= dport[q];
                        ap[q] = tp ? ap[q] + step : ap[q];
                        mp[q] = tp ? ep.y : mp[q];
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t m = md[q] & mp[q];
            const uint32_t j = uint32_t(__ffs(m)) - 1u;               // m == 0 handled below
            const uint32_t bits = uint32_t(((uint64_t(rhi[q]) << 32) | rlo[q]) >> ((2u * j) & 63u));
            res[q] = m ? (bits & 3u) : 0u;            // default DENY (aclengine_mock.go:667)
            slot[q] = m ? cb[q] + j : 0u;
        }
        return;
    }
    const uint16_t* __restrict__ L = reinterpret_cast<const uint16_t*>(base + t.off_lists);
    const uint4* __restrict__ T = reinterpret_cast<const uint4*>(base + t.off_tmpl);
    uint32_t start[N], len[N], cb[N];
    bool act[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const uint32_t pp = proto[q] <= 2u ? proto[q] : 0u;
        const uint2 cell = cells[cls[q] * 3u + pp];
        start[q] = cell.x & 0xFFFFu;
        len[q] = proto[q] <= 2u ? (cell.x >> 16) : 0u;
        cb[q] = cell.y;
        res[q] = 0u;      // default DENY (aclengine_mock.go:667)
        slot[q] = 0u;     // slot 0 = default DENY counter
        act[q] = len[q] != 0u;
    }
    bool any = false;
#pragma unroll
    for (int q = 0; q < N; ++q) any |= act[q];
    if (t.ablate & 2u) {
#pragma unroll
        for (int q = 0; q < N; ++q) res[q] = len[q] & 3u;
        any = false;
    }
    for (uint32_t j = 0; any; ++j) {
        any = false;
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t idx = start[q] + (act[q] ? j : 0u);
            const uint4 tm = T[L[idx]];
            const bool m = act[q] && ((dst[q] ^ tm.x) & tm.y) == 0u && port_in(dport[q], tm.z);
            res[q] = m ? tm.w : res[q];
            slot[q] = m ? cb[q] + j : slot[q];
            act[q] = act[q] && !m && (j + 1u < len[q]);
            any |= act[q];
        }
    }
}

template <int N, bool kLds, int kMode>
__device__ __forceinline__ void run_n(const uint8_t* base, const Cls4Dev& t, uint32_t* lctr,
                                      unsigned long long* gslot, uint32_t hot_lane,
                                      uint32_t& hot0, const uint32_t (&s)[N],
                                      const uint32_t (&d)[N], const uint32_t (&dp)[N],
                                      const uint32_t (&pr)[N], uint32_t (&res)[N]) {
    uint32_t slot[N];
    classify_n<N, (kMode & 1), (kMode >> 1)>(base, t, s, d, dp, pr, res, slot);
    if (t.ablate & 1u) return;
    // One LDS atomic per packet, no branch.  Hot slots (< n_hot: default DENY
    // and the cells of the widest source class) would have many lanes adding
    // to one word -- serialised -- so they are counted in this lane's own
    // row (hot_lane + slot * 64: one bank per lane) and folded at the end.
    uint32_t idx[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        if constexpr (kLds) {
            idx[q] = slot[q] < t.n_hot ? hot_lane + slot[q] * 64u : slot[q];
            atomicAdd(&lctr[idx[q]], 1u);
        } else if (pr[q] <= 2u) {
            if (slot[q] == 0u) ++hot0;
            else atomicAdd(&gslot[slot[q]], 1ull);
        }
    }
    // Protocols outside TCP/UDP/ICMP fall through evalACL's switch
    // (aclengine_mock.go:508-664): networks alone decide.  Rare; taken per
    // wave only when some lane holds such a packet.
    bool other = false;
#pragma unroll
    for (int q = 0; q < N; ++q) other |= pr[q] > 2u;
    if (__any(other)) {
#pragma unroll
        for (int q = 0; q < N; ++q) {
            if (pr[q] > 2u) {
                if constexpr (kLds) atomicSub(&lctr[idx[q]], 1u);   // undo the cell count
                uint32_t rule;
                linear_one(t.lin, t.n_lin, t.n_rules, s[q], d[q], dp[q], 3u, res[q], rule);
                atomicAdd(&gslot[t.n_ctr + rule], 1ull);
            }
        }
    }
}

#ifndef CLS_GROUPS
#define CLS_GROUPS 1
#endif
constexpr int kG = CLS_GROUPS;     // 16-B packet groups per lane per step

template <bool kLds, bool kVec, int kMode>
__global__ __launch_bounds__(kBlock) void classify4_cls(Cls4Dev t, Pkts4 p, uint8_t* verdict,
                                                        unsigned long long* gslot) {
    extern __shared__ uint4 smem[];
    const uint8_t* base;
    uint32_t* lctr = nullptr;
    if constexpr (kLds) {
        const uint4* src4 = reinterpret_cast<const uint4*>(t.img);
        const uint32_t n4 = t.img_bytes / 16u;
        for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) smem[i] = src4[i];
        lctr = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(smem) + t.img_bytes);
        for (uint32_t i = threadIdx.x; i < (t.lds_bytes - t.img_bytes) / 4u; i += blockDim.x) lctr[i] = 0u;
        __syncthreads();
        base = reinterpret_cast<const uint8_t*>(smem);
    } else {
        base = reinterpret_cast<const uint8_t*>(t.img);
    }

    const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    uint32_t hot0 = 0;                                     // global-image variant only
    const uint32_t hot_lane = (t.off_hot - t.img_bytes) / 4u + (threadIdx.x & 63u);
    uint64_t tail_from = 0;
    if constexpr (kVec) {
        // kG x 4 packets per lane per step (kG contiguous 16-B groups), next
        // step's loads issued before this step's lookups (software pipelining
        // of the HBM stream)
        constexpr int kN = 4 * kG;
        const uint64_t nsteps = p.n / kN;
        const uint4* S = reinterpret_cast<const uint4*>(p.src);
        const uint4* D = reinterpret_cast<const uint4*>(p.dst);
        const uint2* DP = reinterpret_cast<const uint2*>(p.dport);
        const uint32_t* PR = reinterpret_cast<const uint32_t*>(p.proto);
        uint64_t g = tid;
        uint4 s[kG], d[kG];
        uint2 dp[kG];
        uint32_t pr[kG];
#pragma unroll
        for (int k = 0; k < kG; ++k) {
            s[k] = make_uint4(0, 0, 0, 0); d[k] = s[k]; dp[k] = make_uint2(0, 0); pr[k] = 0;
        }
        if (g < nsteps) {
#pragma unroll
            for (int k = 0; k < kG; ++k) {
                s[k] = S[g * kG + k]; d[k] = D[g * kG + k]; dp[k] = DP[g * kG + k]; pr[k] = PR[g * kG + k];
            }
        }
        while (g < nsteps) {
            const uint64_t gn = g + nthreads;
            uint4 s2[kG], d2[kG];
            uint2 dp2[kG];
            uint32_t pr2[kG];
#pragma unroll
            for (int k = 0; k < kG; ++k) { s2[k] = s[k]; d2[k] = d[k]; dp2[k] = dp[k]; pr2[k] = pr[k]; }
            if (gn < nsteps) {
#pragma unroll
                for (int k = 0; k < kG; ++k) {
                    s2[k] = S[gn * kG + k]; d2[k] = D[gn * kG + k]; dp2[k] = DP[gn * kG + k]; pr2[k] = PR[gn * kG + k];
                }
            }
            uint32_t sa[kN], da[kN], pa[kN], ra[kN];
#pragma unroll
            for (int k = 0; k < kG; ++k) {
                sa[4 * k + 0] = s[k].x; sa[4 * k + 1] = s[k].y; sa[4 * k + 2] = s[k].z; sa[4 * k + 3] = s[k].w;
                da[4 * k + 0] = d[k].x; da[4 * k + 1] = d[k].y; da[4 * k + 2] = d[k].z; da[4 * k + 3] = d[k].w;
                pa[4 * k + 0] = dp[k].x & 0xFFFFu; pa[4 * k + 1] = dp[k].x >> 16;
                pa[4 * k + 2] = dp[k].y & 0xFFFFu; pa[4 * k + 3] = dp[k].y >> 16;
                ra[4 * k + 0] = pr[k] & 0xFFu; ra[4 * k + 1] = (pr[k] >> 8) & 0xFFu;
                ra[4 * k + 2] = (pr[k] >> 16) & 0xFFu; ra[4 * k + 3] = pr[k] >> 24;
            }
            uint32_t v[kN];
            run_n<kN, kLds, kMode>(base, t, lctr, gslot, hot_lane, hot0, sa, da, pa, ra, v);
            if (verdict && !(t.ablate & 8u)) {
#pragma unroll
                for (int k = 0; k < kG; ++k)
                    reinterpret_cast<uint32_t*>(verdict)[g * kG + k] =
                        v[4 * k] | (v[4 * k + 1] << 8) | (v[4 * k + 2] << 16) | (v[4 * k + 3] << 24);
            }
#pragma unroll
            for (int k = 0; k < kG; ++k) { s[k] = s2[k]; d[k] = d2[k]; dp[k] = dp2[k]; pr[k] = pr2[k]; }
            g = gn;
        }
        tail_from = nsteps * kN;
    }
    for (uint64_t i = tail_from + tid; i < p.n; i += nthreads) {
        const uint32_t sa[1] = {p.src[i]}, da[1] = {p.dst[i]}, pa[1] = {p.dport[i]}, ra[1] = {p.proto[i]};
        uint32_t v[1];
        run_n<1, kLds, kMode>(base, t, lctr, gslot, hot_lane, hot0, sa, da, pa, ra, v);
        if (verdict) verdict[i] = uint8_t(v[0]);
    }

    if constexpr (!kLds) {
        if (hot0) atomicAdd(&gslot[0], (unsigned long long)hot0);
    }
    if constexpr (kLds) {
        __syncthreads();
        // fold the per-lane hot rows into their slots
        const uint32_t* hrow = lctr + (t.off_hot - t.img_bytes) / 4u;
        for (uint32_t i = threadIdx.x; i < t.n_hot * 64u; i += blockDim.x) {
            const uint32_t v = hrow[i];
            if (v) atomicAdd(&lctr[i >> 6], v);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < t.n_ctr; i += blockDim.x) {
            const uint32_t v = lctr[i];
            if (v) atomicAdd(&gslot[i], (unsigned long long)v);
        }
    }
}

__global__ __launch_bounds__(kBlock) void classify4_linear(const LinRule4* __restrict__ rules,
                                                           uint32_t nr, uint32_t n_rules, Pkts4 p,
                                                           uint8_t* verdict,
                                                           unsigned long long* gslot) {
    __shared__ uint32_t lctr[kLinLdsCounters];
    const bool lds = n_rules + 1 <= kLinLdsCounters;
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
            if (lds) atomicAdd(&lctr[rule], 1u);
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

__global__ void remap_kernel(const unsigned long long* __restrict__ slot,
                             const uint32_t* __restrict__ map, uint32_t n,
                             unsigned long long* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const unsigned long long v = slot[i];
        if (v) atomicAdd(&out[map[i]], v);
    }
}

// evalACL on one ACL from global memory; returns ACLAction (nil ACL: PERMIT)
__device__ uint32_t eval_acl4(const AclDesc* __restrict__ acls, int32_t a, uint32_t src,
                              uint32_t dst, uint32_t port, uint32_t p) {
    if (a < 0) return 1u;
    const AclDesc A = acls[a];
    if (!A.valid) return 1u;
    uint32_t res, rule;
    linear_one(A.rules, A.n, 0xFFFFFFFFu, src, dst, port, p, res, rule);
    return res;
}

__global__ void connect4_kernel(const AclDesc* __restrict__ acls, const IfAcls* __restrict__ ifs,
                                const uint32_t* __restrict__ src_if,
                                const uint32_t* __restrict__ dst_if,
                                const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
                                const uint16_t* __restrict__ sport,
                                const uint16_t* __restrict__ dport,
                                const uint8_t* __restrict__ proto, uint64_t n,
                                uint8_t* __restrict__ out) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t si = src_if[i], di = dst_if[i];
    const IfAcls S = ifs[si], D = ifs[di];
    const bool same = si == di;
    const uint32_t sa = src[i], da = dst[i], sp = sport[i], dp = dport[i];
    const uint32_t p = proto[i] <= 2 ? proto[i] : 3u;
    bool srefl = false, drefl = false;
    uint32_t a = eval_acl4(acls, S.in, sa, da, dp, p);            // SYN: src inbound
    if (a == 3u) { out[i] = 3; return; }
    if (a == 0u) { out[i] = 0; return; }
    if (a == 2u) { srefl = true; if (same) drefl = true; }
    if (!drefl) {                                                 // SYN: dst outbound
        a = eval_acl4(acls, D.out, sa, da, dp, p);
        if (a == 3u) { out[i] = 3; return; }
        if (a == 0u) { out[i] = 0; return; }
        if (a == 2u) { drefl = true; if (same) srefl = true; }
    }
    if (!drefl) {                                                 // SYN-ACK: dst inbound
        a = eval_acl4(acls, D.in, da, sa, sp, p);
        if (a == 3u) { out[i] = 3; return; }
        if (a == 0u) { out[i] = 1; return; }
    }
    if (!srefl) {                                                 // SYN-ACK: src outbound
        a = eval_acl4(acls, S.out, da, sa, sp, p);
        if (a == 3u) { out[i] = 3; return; }
        if (a == 0u) { out[i] = 1; return; }
    }
    out[i] = 2;
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

}  // namespace

int max_lds_bytes() { return kLdsMax; }

template <bool kLds, bool kVec, int kMode>
static void launch_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                       const LaunchCfg& cfg) {
    const size_t lds = kLds ? t.lds_bytes : 0;
    if (kLds)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(classify4_cls<kLds, kVec, kMode>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    hipLaunchKernelGGL((classify4_cls<kLds, kVec, kMode>), dim3(cfg.grid), dim3(kBlock), lds, cfg.stream,
                       t, p, verdict, gslot);
}

hipError_t launch_classify4_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict,
                                unsigned long long* gslot, bool lds_resident, bool vec,
                                const LaunchCfg& cfg) {
    // variant bits: 1 = hash LPM source lookup, 2 = bit-vector candidate lists
    const int var = (t.mode == 1 ? 1 : 0) | (int(t.list_mode) << 1);
#define CLS_DISPATCH(L, V)                                                       \
    switch (var) {                                                               \
    case 0: launch_cls<L, V, 0>(t, p, verdict, gslot, cfg); break;               \
    case 1: launch_cls<L, V, 1>(t, p, verdict, gslot, cfg); break;               \
    case 2: launch_cls<L, V, 2>(t, p, verdict, gslot, cfg); break;               \
    case 3: launch_cls<L, V, 3>(t, p, verdict, gslot, cfg); break;               \
    case 4: launch_cls<L, V, 4>(t, p, verdict, gslot, cfg); break;               \
    default: launch_cls<L, V, 5>(t, p, verdict, gslot, cfg); break;              \
    }
    if (lds_resident) {
        if (vec) { CLS_DISPATCH(true, true) } else { CLS_DISPATCH(true, false) }
    } else {
        if (vec) { CLS_DISPATCH(false, true) } else { CLS_DISPATCH(false, false) }
    }
#undef CLS_DISPATCH
    return hipGetLastError();
}

hipError_t launch_classify4_linear(const LinRule4* rules, uint32_t n_lin, uint32_t n_rules,
                                   const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                                   const LaunchCfg& cfg) {
    hipLaunchKernelGGL(classify4_linear, dim3(cfg.grid), dim3(kBlock), 0, cfg.stream, rules, n_lin,
                       n_rules, p, verdict, gslot);
    return hipGetLastError();
}

hipError_t launch_remap(const unsigned long long* slot, const uint32_t* map, uint32_t n,
                        unsigned long long* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(remap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, slot, map, n, out);
    return hipGetLastError();
}

hipError_t launch_connect4(const AclDesc* acls, const IfAcls* ifs, const uint32_t* src_if,
                           const uint32_t* dst_if, const uint32_t* src, const uint32_t* dst,
                           const uint16_t* sport, const uint16_t* dport, const uint8_t* proto,
                           uint64_t n, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(connect4_kernel, dim3(uint32_t((n + 255) / 256)), dim3(256), 0, s, acls, ifs,
                       src_if, dst_if, src, dst, sport, dport, proto, n, out);
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
