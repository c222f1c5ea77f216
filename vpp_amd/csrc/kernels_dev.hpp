// Device code of the gfx950 classifier kernels shared by the kernel
// translation units (kernels.hip, k4_lds.hip, k4_glb.hip, k16.hip): the
// classify templates and their dispatchers.  Each unit instantiates only
// its own variants, so the units compile in parallel.
#pragma once

// gfx950 kernels of the batched first-match ACL classifier.
//
// classify4_cls  -- the hot path.  Persistent grid-stride kernel; every
//   workgroup stages the read-only classifier image (compile.hpp, Cls4Image)
//   into LDS once with 16-B loads, zeroes its LDS slot counters, then streams
//   packets: 4 packets per lane per step with 16-B (src, dst), 8-B (dport) and
//   4-B (proto) coalesced non-temporal loads and one 4-B verdict store, the
//   next step's loads in flight during this step's lookups.  Per packet:
//   source lookup (cuckoo hash LPM or interval search) -> the (class,
//   protocol) cell -> the cell's candidate list evaluated against dst address
//   and dst port (list modes 0-3, compile.hpp) -> verdict and the terminating
//   slot.  One LDS atomic per packet counts the slot; counters are flushed to
//   global u64 slots once per workgroup.  Integer compare work only -- no MFMA.
//
//   Cost model (measured on MI355X, config 3): the kernel is bound by VALU
//   issue plus LDS bank conflicts, ~0.006 ms per VALU op per packet and
//   ~0.03 ms per LDS read per packet at 256 Mi packets, both above the HBM
//   stream's 0.53 ms floor.  So LDS is addressed with absolute 32-bit
//   addresses (no base add), table values are stored pre-scaled to the byte
//   addresses the next lookup needs, and list mode 3 searches with a single
//   state word per packet.
// classify4_linear -- the ballot kernel: every lane walks the rule list in
//   order with wave-uniform (scalar) rule loads and the wave leaves as soon
//   as the ballot of unfinished lanes is empty.  Small tables, GPU cross-check,
//   and the protocol>2 fallback of classify4_cls.
// connect4 -- testConnection (aclengine_mock.go:394-471) for a batch.
// gen4 -- the counter-based splitmix64 traffic stream, generated in HBM.
#include <hip/hip_runtime.h>

#include <hip/hip_ext.h>

#include "kernels.hpp"

#include <atomic>
#include <utility>

namespace cls {

namespace {

constexpr int kBlock = 1024;      // linear kernel
constexpr int kClsBlock = 1024;   // classifier workgroup (one LDS image per workgroup)
constexpr int kLdsMax = 160 * 1024;
constexpr uint32_t kLinLdsCounters = 16384;  // linear kernel: LDS counters up to R+1 <= this

// Streamed packet fields are read once and verdicts written once: non-temporal
// loads/stores keep them from churning L2 / the Infinity Cache (measured on
// MI355X with tools/stream_bench.hip: 0.53 ms vs 0.61 ms for 256 Mi packets).
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ldnt(const uint4* p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ldnt(const uint2* p) {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t ldnt(const uint32_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt(uint32_t v, uint32_t* p) { __builtin_nontemporal_store(v, p); }
// element i of a streamed array by 32-bit byte offset: SGPR base + VGPR offset
template <typename T>
__device__ __forceinline__ const T* at(const T* base, uint32_t i) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + i * uint32_t(sizeof(T)));
}

// The classifier image, read either from LDS (staged at LDS address 0: the
// kernel has no static __shared__ data, so its dynamic LDS starts there) by
// absolute 32-bit address -- ds_read with no base add -- or, for images too
// large for LDS, from global memory.
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"   // 32-bit LDS addresses
typedef const __attribute__((address_space(3))) uint8_t* lds8_t;
typedef const __attribute__((address_space(3))) uint16_t* lds16_t;
typedef const __attribute__((address_space(3))) uint32_t* lds32_t;
typedef const __attribute__((address_space(3))) v2u* lds64_t;
typedef const __attribute__((address_space(3))) v4u* lds128_t;
typedef __attribute__((address_space(3))) v4u* lds128w_t;
template <bool kLds>
struct Img {
    const uint8_t* g;
    __device__ __forceinline__ uint32_t u8(uint32_t a) const {
        if constexpr (kLds) return *lds8_t(a); else return g[a];
    }
    __device__ __forceinline__ uint32_t u16(uint32_t a) const {
        if constexpr (kLds) return *lds16_t(a); else return *reinterpret_cast<const uint16_t*>(g + a);
    }
    __device__ __forceinline__ uint32_t u32(uint32_t a) const {
        if constexpr (kLds) return *lds32_t(a); else return *reinterpret_cast<const uint32_t*>(g + a);
    }
    __device__ __forceinline__ uint2 u64(uint32_t a) const {
        if constexpr (kLds) {
            const v2u v = *lds64_t(a);
            return make_uint2(v.x, v.y);
        } else {
            return *reinterpret_cast<const uint2*>(g + a);
        }
    }
    __device__ __forceinline__ uint4 u128(uint32_t a) const {
        if constexpr (kLds) {
            const v4u v = *lds128_t(a);
            return make_uint4(v.x, v.y, v.z, v.w);
        } else {
            return *reinterpret_cast<const uint4*>(g + a);
        }
    }
};

// A kernel's dynamic-LDS ceiling (hipFuncSetAttribute), raised once per
// (kernel, device) to the CU's whole LDS less the kernel's static LDS: the
// attribute is only a ceiling (a launch's occupancy follows the LDS it asks
// for), so no launch needs a host call, a lock or a lookup -- one static
// bit mask per kernel instantiation, a bit per device.  The attribute is the
// current device's (a multi-device engine launches the same kernels on
// every device).
template <auto K>
inline void lds_attr() {
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return;
    const void* f = reinterpret_cast<const void*>(K);
    hipFuncAttributes fa{};
    const size_t st = hipFuncGetAttributes(&fa, f) == hipSuccess ? fa.sharedSizeBytes : 0;
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, int(size_t(kLdsMax) - st));
    done.fetch_or(bit, std::memory_order_release);
}

// Position of the r-th set bit (0-based) of a 64-bit lane mask: six halving
// steps on popcounts (wave-level job packing without LDS: a lane finds the
// job it runs from the ballots of the lanes that own jobs).
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t r) {
    uint32_t lo = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint32_t c = uint32_t(__popcll((m >> lo) & ((1ull << w) - 1ull)));
        if (c <= r) {
            r -= c;
            lo += uint32_t(w);
        }
    }
    return lo;
}

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

// One probe step I of the sublist search for N packets (list modes 3, 4).
template <int I, int N, bool kLds>
__device__ __forceinline__ void sub_step(const Img<kLds>& im, const uint32_t (&dst)[N],
                                         uint32_t (&st)[N]) {
    uint2 e[N];
#pragma unroll
    for (int q = 0; q < N; ++q) e[q] = im.u64((st[q] >> 13) + (8u << I));
#pragma unroll
    for (int q = 0; q < N; ++q) st[q] = e[q].x < dst[q] ? e[q].y : st[q];
}

// Source lookup of N packets, interleaved (N independent LDS chains per lane).
// Result: the byte address of the packet's class row of cells.  kMode: 0
// interval search, 1 hash LPM over t.n_hash prefix lengths, 2 hash LPM over
// exactly one length (pod /32s: the common rendered table; fewer live SGPRs),
// 4 source trie (compile.cpp build_trie).
template <int N, bool kLds, int kMode>
__device__ __forceinline__ void src_row(const Img<kLds>& im, const Cls4Dev& t,
                                        const uint32_t (&src)[N], uint32_t (&row)[N]) {
    if constexpr (kMode == 4) {
        // level 1 -> node -> leaf {byte address << 8 | m - 1}; then the leaf's
        // branch-free lower bound for t.trie_depth steps (uniform): steps
        // past a lane's own ceil(log2 m) have h = 0 and re-test the current
        // entry (already taken, or entry 0: key 0xFFFF), so no per-lane branch
        uint32_t a[N], len[N], x[N];
#pragma unroll
        for (int q = 0; q < N; ++q) a[q] = im.u32(t.off_trie + ((src[q] >> 22) & 0x3FCu));
#pragma unroll
        for (int q = 0; q < N; ++q) a[q] = im.u32(a[q] + ((src[q] >> 14) & 0x3FCu));
#pragma unroll
        for (int q = 0; q < N; ++q) {
            len[q] = (a[q] & 0xFFu) + 1u;
            a[q] >>= 8;
            x[q] = src[q] & 0xFFFFu;
        }
#pragma unroll
        for (int i = 0; i < int(kMaxTrieDepth); ++i) {
            if (uint32_t(i) >= t.trie_depth) break;              // uniform
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint32_t h = len[q] >> 1, c = a[q] + 4u * h;
                a[q] = (im.u32(c) & 0xFFFFu) < x[q] ? c : a[q];
                len[q] -= h;
            }
        }
#pragma unroll
        for (int q = 0; q < N; ++q) row[q] = t.off_cells + (im.u32(a[q]) >> 16) * t.row_bytes;
    } else if constexpr (kMode == 3) {
        // the caller found the rows (16-byte path, host-route hashes)
#pragma unroll
        for (int q = 0; q < N; ++q) row[q] = src[q];
    } else if constexpr (kMode >= 1) {
        // Hash LPM: one cuckoo probe pair per prefix length, lengths ascending
        // so the longest hit wins.  Entries {key, row}; empty slots hold keys
        // that never probe them, so a key compare is the whole hit test.  The
        // parameters are indexed by constants: loaded into SGPRs once.
#pragma unroll
        for (int q = 0; q < N; ++q) row[q] = t.default_row;
#pragma unroll
        for (uint32_t i = 0; i < (kMode == 2 ? 1u : kMaxHashLens); ++i) {
            if (kMode == 1 && i >= t.n_hash) break;
            // one multiply per key: table 0 probes the top L bits of key x
            // mul, table 1 the next L bits (compile.hpp lpm_h0 / lpm_h1)
            const uint32_t tab = t.off_hash[i], mask = t.hash_mask[i], mul = t.hash_mul[i];
            const uint32_t s0 = t.hash_shift[i], s1 = t.hash_shift1[i], L = 32u - s0;
            const uint32_t tab1 = __builtin_amdgcn_readfirstlane(tab + 8u * t.hash_cap[i]);
            uint2 e0[N], e1[N];
            uint32_t key[N];
#pragma unroll
            for (int q = 0; q < N; ++q) {
                key[q] = src[q] & mask;
                const uint32_t h = key[q] * mul;
                e0[q] = im.u64(tab + 8u * (h >> s0));
                e1[q] = im.u64(tab1 + 8u * __builtin_amdgcn_ubfe(h, s1, L));
            }
#pragma unroll
            for (int q = 0; q < N; ++q) {
                row[q] = e1[q].x == key[q] ? e1[q].y : row[q];
                row[q] = e0[q].x == key[q] ? e0[q].y : row[q];
            }
        }
    } else {
        // branch-free binary search over the padded interval boundaries
        uint32_t k[N];
#pragma unroll
        for (int q = 0; q < N; ++q) k[q] = 0;
#pragma unroll 1
        for (uint32_t s = t.search_top; s; s >>= 1) {
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint32_t c = k[q] + s;
                k[q] = (im.u32(t.off_bounds + 4u * c) <= src[q]) ? c : k[q];
            }
        }
#pragma unroll
        for (int q = 0; q < N; ++q)
            row[q] = t.off_cells + im.u16(t.off_iclass + 2u * k[q]) * t.row_bytes;
    }
}

// First match of N packets (protocols 0-2) against their cells' candidate
// lists: verdict (ACLAction) and the terminating counter slot (0 = default
// DENY, aclengine_mock.go:667).
// row_out (optional): the packets' class rows (byte address of the row of
// cells), for a caller that classifies some of them again on the OTHER
// image, whose classes are the same (k4_pair.hip).  kCells: cells per class
// row -- 3 (TCP, UDP, ICMP; protocols > 2 go to the OTHER image), or 4 (the
// pair launch's image, compile.hpp Cls4Opts::with_other: the fourth cell for
// protocols > 2).
template <int N, bool kLds, int kMode, int kList, int kD, int kCells = 3>
__device__ __forceinline__ void classify_n(const Img<kLds>& im, const Cls4Dev& t,
                                           const uint32_t (&src)[N], const uint32_t (&dst)[N],
                                           const uint32_t (&dport)[N], const uint32_t (&proto)[N],
                                           uint32_t (&res)[N], uint32_t (&slot)[N],
                                           uint32_t (*row_out)[N] = nullptr) {
    // list modes 5, 6: 4, 3 with the wide cells in global memory (t.gcells)
    constexpr bool kWide = kList >= 5;
    constexpr int kPort = kList == 5 ? 4 : kList == 6 ? 3 : kList;
    uint32_t pc[N];
    if constexpr (kPort == 4) {
        // Port class from the perfect hash at image address 0: one probe at
        // byte address mulhi(port, mul) & mask4, e = {port | class x 4 << 16};
        // ports absent from it are in the default class (rendered tables:
        // every port no rule names).
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t e = im.u32(__umulhi(dport[q], t.port_mul) & t.port_mask4);
            pc[q] = (e & 0xFFFFu) == dport[q] ? e >> 16 : t.port_dflt;
        }
    } else if constexpr (kPort >= 2) {
        // Global port class from the radix at image address 0: top[port >> 8]
        // = byte address of a 256-byte window, class = window[port & 255]
        // (class x 4 in mode 3).  Independent of the source lookup: these
        // reads go out with the probes.
        uint32_t tp[N];
#pragma unroll
        for (int q = 0; q < N; ++q) tp[q] = im.u32(((dport[q] >> 8) & 0xFFu) * 4u);
#pragma unroll
        for (int q = 0; q < N; ++q) pc[q] = im.u8(tp[q] + (dport[q] & 0xFFu));
    }
    uint32_t row[N];
    src_row<N, kLds, kMode>(im, t, src, row);
    if (row_out) {
#pragma unroll
        for (int q = 0; q < N; ++q) (*row_out)[q] = row[q];
    }

    if constexpr (kList >= 3) {
        // Port-filtered sublists.  cell = {pointer table word address | counter
        // base << 14} (slot base + 0: the cell's own no-match slot, counted as
        // default DENY); the pointer table holds, per global port
        // class, the initial search state of the sublist deciding first-match
        // for that class: state = outcome | 8-B slot of the current entry << 16,
        // outcome = result | (j + 1) << 2 (0: no entry, default DENY), so
        // state >> 13 is the entry's byte address.  A probe of step i reads
        // {start - 1, state} 8 << i bytes further and the state moves to the
        // entry when start - 1 < dst: one shift, one compare, one select.
        uint32_t cell[N], st[N];
        if constexpr (kWide) {
            // cell = {pointer table byte address, counter base}; cell[q] keeps
            // the base (the slot below)
            uint2 wc[N];
#pragma unroll
            for (int q = 0; q < N; ++q)
                wc[q] = *reinterpret_cast<const uint2*>(t.gcells + row[q] + 8u * min(proto[q], uint32_t(kCells - 1)));
#pragma unroll
            for (int q = 0; q < N; ++q) {
                cell[q] = wc[q].y;
                st[q] = im.u32(wc[q].x + pc[q]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < N; ++q) cell[q] = im.u32(row[q] + 4u * min(proto[q], uint32_t(kCells - 1)));
#pragma unroll
            for (int q = 0; q < N; ++q) st[q] = im.u32(((cell[q] & 0x3FFFu) << 2) + pc[q]);
        }
        // kD >= 0: the table's depth is a template argument -- straight-line
        // probes.  kD < 0 (scalar tail, global-image variants): guarded steps
        // (the compiler materialises those uniform guards as lane masks, a
        // few VALU ops per step).
        static_assert(kMaxBvSteps == 7, "step chain below");
        if constexpr (kD > 6) sub_step<6>(im, dst, st);
        if constexpr (kD > 5) sub_step<5>(im, dst, st);
        if constexpr (kD > 4) sub_step<4>(im, dst, st);
        if constexpr (kD > 3) sub_step<3>(im, dst, st);
        if constexpr (kD > 2) sub_step<2>(im, dst, st);
        if constexpr (kD > 1) sub_step<1>(im, dst, st);
        if constexpr (kD > 0) sub_step<0>(im, dst, st);
        if constexpr (kD < 0) {
            if (t.bv_steps > 6) sub_step<6>(im, dst, st);
            if (t.bv_steps > 5) sub_step<5>(im, dst, st);
            if (t.bv_steps > 4) sub_step<4>(im, dst, st);
            if (t.bv_steps > 3) sub_step<3>(im, dst, st);
            if (t.bv_steps > 2) sub_step<2>(im, dst, st);
            if (t.bv_steps > 1) sub_step<1>(im, dst, st);
            if (t.bv_steps > 0) sub_step<0>(im, dst, st);
        }
#pragma unroll
        for (int q = 0; q < N; ++q) {
            res[q] = st[q] & 3u;                                      // DENY when no entry
            slot[q] = (kWide ? cell[q] : cell[q] >> 14) + ((st[q] >> 2) & 63u);   // base + j + 1 (0: no entry)
        }
    } else if constexpr (kList >= 1) {
        // Bit vectors: the entries of the cell's list covering the packet's dst
        // interval AND its port interval; the lowest set bit is the first match.
        // cell = block / 8 | counter base << 16.  Block: dst array of 2^S
        // {interval start, mask} (entry 0, never probed, = {result bits lo,
        // mask of interval 0}), then mode 1: the port array likewise (entry 0 =
        // {result bits hi, mask}); mode 2: result bits hi, one mask per global
        // port class.  The searches track the byte address of the current
        // entry; the steps are constants, so a probe is one ds_read_b64 with an
        // immediate offset.
        const uint32_t S = t.bv_steps;
        uint32_t cb[N], ad[N], ap[N], rlo[N], rhi[N], md[N], mp[N];
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t cell = im.u32(row[q] + 4u * min(proto[q], uint32_t(kCells - 1)));
            cb[q] = cell >> 16;
            ad[q] = (cell & 0xFFFFu) * 8u;
            ap[q] = ad[q] + (8u << S);
        }
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint2 d0 = im.u64(ad[q]);
            rlo[q] = d0.x;
            md[q] = d0.y;
            if constexpr (kList == 1) {
                const uint2 p0 = im.u64(ap[q]);
                rhi[q] = p0.x;
                mp[q] = p0.y;
            } else {
                mp[q] = im.u32(ap[q] + 4u + pc[q] * 4u);
                rhi[q] = t.bv_wide ? im.u32(ap[q]) : 0u;
            }
        }
#pragma unroll
        for (int i = int(kMaxBvSteps) - 1; i >= 0; --i) {
            if (uint32_t(i) >= S) continue;
            const uint32_t step = 8u << i;
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint2 ed = im.u64(ad[q] + step);
                const bool td = ed.x <= dst[q];
                ad[q] = td ? ad[q] + step : ad[q];
                md[q] = td ? ed.y : md[q];
                if constexpr (kList == 1) {
                    const uint2 ep = im.u64(ap[q] + step);
                    const bool tq = ep.x <= dport[q];
                    ap[q] = tq ? ap[q] + step : ap[q];
                    mp[q] = tq ? ep.y : mp[q];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint32_t m = md[q] & mp[q];
            const uint32_t j = uint32_t(__ffs(m)) - 1u;               // m == 0 handled below
            const uint32_t bits = uint32_t(((uint64_t(rhi[q]) << 32) | rlo[q]) >> ((2u * j) & 63u));
            res[q] = m ? (bits & 3u) : 0u;
            slot[q] = m ? cb[q] + j : 0u;
        }
    } else {
        // Template scan (lists > 32 entries): cell = {list start | length << 16,
        // counter base}; entries are 16-bit ids of 16-B templates {dst, dst
        // mask, port lo | width << 16, result}.  The N scans advance in
        // lockstep with predication.
        uint32_t start[N], len[N], cb[N];
        bool act[N];
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint2 cell = im.u64(row[q] + 8u * min(proto[q], uint32_t(kCells - 1)));
            start[q] = cell.x & 0xFFFFu;
            len[q] = cell.x >> 16;
            cb[q] = cell.y;
            res[q] = 0u;
            slot[q] = 0u;
            act[q] = len[q] != 0u;
        }
        bool any = false;
#pragma unroll
        for (int q = 0; q < N; ++q) any |= act[q];
        for (uint32_t j = 0; any; ++j) {
            any = false;
#pragma unroll
            for (int q = 0; q < N; ++q) {
                const uint32_t idx = start[q] + (act[q] ? j : 0u);
                const uint4 tm = im.u128(t.off_tmpl + 16u * im.u16(t.off_lists + 2u * idx));
                const bool m = act[q] && ((dst[q] ^ tm.x) & tm.y) == 0u && port_in(dport[q], tm.z);
                res[q] = m ? tm.w : res[q];
                slot[q] = m ? cb[q] + j : slot[q];
                act[q] = act[q] && !m && (j + 1u < len[q]);
                any |= act[q];
            }
        }
    }
}

// Global slot counters from a wave: lanes holding the same slot are summed
// across the wave first (ballot per distinct slot, one atomic by the lowest
// lane), so a hot slot costs one atomic per wave, not 64.  key ~0u: nothing.
__device__ __forceinline__ void wave_count(unsigned long long* gslot, uint32_t key) {
    unsigned long long pending = __ballot(key != 0xFFFFFFFFu);
    while (pending) {
        const int leader = __builtin_ctzll(pending);
        const uint32_t sk = __shfl(key, leader);
        const unsigned long long same = __ballot(key == sk);
        if (int(__lane_id()) == leader) atomicAdd(&gslot[sk], (unsigned long long)__popcll(same));
        pending &= ~same;
    }
}

// Global slot counters of the cold tier (slots past the LDS counters):
// spread keys, so one aggregation round for the leader's key (a popular slot
// costs one atomic) and direct atomics for the rest, instead of one ballot
// round per distinct key.
__device__ __forceinline__ void wave_count_cold(unsigned long long* gslot, uint32_t key) {
    const unsigned long long pending = __ballot(key != 0xFFFFFFFFu);
    if (!pending) return;
    const int leader = __builtin_ctzll(pending);
    const uint32_t sk = __shfl(key, leader);
    const unsigned long long same = __ballot(key == sk);
    if (int(__lane_id()) == leader) atomicAdd(&gslot[sk], (unsigned long long)__popcll(same));
    else if (key != 0xFFFFFFFFu && key != sk) atomicAdd(&gslot[key], 1ull);
}

// Classify N packets and count their slots.  kCtr (LDS-resident image): 0 --
// every slot has a u32 LDS counter; 1 -- u16 LDS counters for slots <
// n_lctr (compile.hpp Cls4Image counter tiers), global counters above.
// pr_any: some packet of the group has a protocol outside TCP/UDP/ICMP; those
// packets are queued for the finish launch (counting) or classified on the
// OTHER image `o` in place (slot mode, full queue) from sl(q): packet q's
// source, or on the 16-byte path its rep -- computed only for those.
// The OTHER queue row of this wave, and the first entry after the fills.
__device__ __forceinline__ uint32_t queue_row() { return blockIdx.x * kOtherSegs + (threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t queue_row0() { return gridDim.x * kOtherSegs; }

template <int N, bool kLds, int kMode, int kList, int kD, int kCtr, bool kMaskQ = false, typename SrcOf>
__device__ __forceinline__ void run_n(const Img<kLds>& im, const Cls4Dev& t, const Cls4Dev& o, uint32_t hot_lane,
                                      unsigned long long* gslot, uint32_t& hot0,
                                      const uint32_t (&s)[N], const uint32_t (&d)[N],
                                      const uint32_t (&dp)[N], const uint32_t (&pr)[N],
                                      bool pr_any, uint32_t (&res)[N], const SrcOf& sl,
                                      const uint32_t (&idx)[N], uint32_t oq_lds, uint32_t& wq) {
    uint32_t slot[N];
    classify_n<N, kLds, kMode, kList, kD>(im, t, s, d, dp, pr, res, slot);
    // One LDS atomic per packet, no branch.  Hot slots (< n_hot: default DENY
    // and the cells of the widest source class) would have many lanes adding
    // to one word -- serialised -- so they are counted in this lane's own row
    // (hot_lane + slot * 256 bytes: one bank per lane) and folded at the end.
    typedef __attribute__((address_space(3))) uint32_t* lctr_t;
    uint32_t addr[N];
    if constexpr (kCtr == 2) {
        // Slot mode (connection batches, cls_connect_batch): no counting; the
        // result word is res | slot << 2, OTHER packets classified in place
        // with their slots after the main image's (the caller maps slots to
        // rules for the evaluations testConnection actually makes).
#pragma unroll
        for (int q = 0; q < N; ++q) res[q] |= slot[q] << 2;
        if (__any(pr_any)) {
            const Img<false> oim{reinterpret_cast<const uint8_t*>(o.img)};
#pragma unroll
            for (int q = 0; q < N; ++q) {
                if (pr[q] > 2u) {
                    const uint32_t s1[1] = {sl(q)}, d1[1] = {d[q]}, p1[1] = {dp[q]}, z1[1] = {0u};
                    uint32_t r1[1], k1[1];
                    classify_n<1, false, 0, 0, -1>(oim, o, s1, d1, p1, z1, r1, k1);
                    res[q] = r1[0] | ((t.n_ctr + k1[0]) << 2);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
        if constexpr (kLds && kCtr == 0) {
            // a packet of protocol > 2 (counted by its OTHER evaluation) adds
            // to a spare word after the OTHER queue counter instead: no branch
            addr[q] = pr[q] > 2u ? oq_lds + 4u : slot[q] < t.n_hot ? hot_lane + slot[q] * 256u : t.img_bytes + slot[q] * 4u;
            __hip_atomic_fetch_add(lctr_t(addr[q]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if constexpr (kLds) {
            // Tiered counters.  A u16 counter lives in half of an LDS word; the
            // lane whose add takes it from 0x7FFF to 0x8000 moves 0x8000 to the
            // slot's global counter at once, so a half never carries into its
            // neighbour (that would need 0x8000 more adds to one slot in the
            // few instructions before the move).
            uint32_t key = 0xFFFFFFFFu;
            if (pr[q] <= 2u) {
                if (slot[q] < t.n_hot) {
                    __hip_atomic_fetch_add(lctr_t(hot_lane + slot[q] * 256u), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                } else if (slot[q] < t.n_lctr) {
                    const uint32_t w = t.img_bytes + ((slot[q] * 2u) & ~3u), sh = (slot[q] & 1u) * 16u;
                    const uint32_t old = __hip_atomic_fetch_add(lctr_t(w), 1u << sh, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
                        __hip_atomic_fetch_add(lctr_t(w), 0u - (0x8000u << sh), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        atomicAdd(&gslot[slot[q]], 0x8000ull);
                    }
                } else {
                    key = slot[q];
                }
            }
            wave_count_cold(gslot, key);
        } else {
            // Global counters (image not LDS-resident); slot 0 (default DENY,
            // the hottest) is counted per lane and added once at the end
            uint32_t key = pr[q] <= 2u ? slot[q] : 0xFFFFFFFFu;
            if (key == 0u) {
                ++hot0;
                key = 0xFFFFFFFFu;
            }
            wave_count(gslot, key);
        }
    }
    // Protocols outside TCP/UDP/ICMP fall through evalACL's switch
    // (aclengine_mock.go:508-664): networks alone decide.  Rare; taken per
    // wave only when some lane holds such a packet.  Such a packet's index
    // goes to its wave's segment of the OTHER queue (t.oq), which the finish
    // launch classifies on the OTHER image after this launch (verdict, count);
    // when the queue is full, here and now (the OTHER image's interval
    // search and candidate scan from global memory, its slots after the main
    // image's).
    if (__any(pr_any)) {
        if constexpr (kMaskQ) {
            // IPv4 launches (packets idx[q] = idx[0] + q, idx[0] a multiple of
            // 4, or one packet): one entry per lane holding OTHER packets,
            // (idx[0] >> 2) | their slots' mask << 28 (FinishArgs::qmask) --
            // one rank and one store per lane instead of one per slot
            uint32_t qm = 0u;
#pragma unroll
            for (int q = 0; q < N; ++q) qm |= (pr[q] > 2u ? 1u : 0u) << q;
            const uint32_t ent = N == 1 ? (idx[0] >> 2) | (qm << (28u + (idx[0] & 3u)))
                                        : (idx[0] >> 2) | (qm << 28);
            const uint64_t lb = __ballot(qm != 0u);
            const uint32_t base0 = __builtin_amdgcn_readfirstlane(wq), c = uint32_t(__popcll(lb));
            if (t.oq && base0 + c <= t.oq_cap) {                 // wave-uniform: room for all of them
                wq = base0 + c;
                if (qm) t.oq[queue_row0() + queue_row() * t.oq_cap + base0 +
                             uint32_t(__popcll(lb & ((1ull << __lane_id()) - 1ull)))] = ent;
                return;
            }
        }
        // one queue reservation for the wave's OTHER packets of all N slots
        uint64_t m[N];
        uint32_t pre[N + 1];
        pre[0] = 0u;
#pragma unroll
        for (int q = 0; q < N; ++q) {
            m[q] = __ballot(pr[q] > 2u);
            pre[q + 1] = pre[q] + uint32_t(__popcll(m[q]));
        }
        const uint64_t lt = (1ull << __lane_id()) - 1ull;
        // this wave's own queue segment, its fill a wave-uniform register:
        // no LDS atomic (and no wait for its return) per wave step; read
        // from the first active lane, so that the segment's address is
        // scalar (lanes done with a tail loop keep stale copies, but the
        // loops' active lanes are a prefix: lane 0 is current)
        const uint32_t base = __builtin_amdgcn_readfirstlane(wq);
        if (t.oq && base + pre[N] <= t.oq_cap) {          // wave-uniform: room for all of them
            wq = base + pre[N];
            uint32_t* seg = t.oq + queue_row0() + queue_row() * t.oq_cap + base;
#pragma unroll
            for (int q = 0; q < N; ++q)
                if (pr[q] > 2u)
                    seg[pre[q] + uint32_t(__popcll(m[q] & lt))] =
                        kMaskQ ? (idx[q] >> 2) | (1u << (28u + (idx[q] & 3u))) : idx[q];
        } else {
            // the segment is full (or there is none): what fits is queued,
            // the rest classified here and now (an out-of-line function for
            // this rare path cost config 3 11 %: the call changed the hot
            // loop's register allocation, profiles/r05k_bench_c3_noinline.json)
            if (t.oq) wq = min(base + pre[N], t.oq_cap);
#pragma unroll
            for (int q = 0; q < N; ++q) {
                bool now = pr[q] > 2u;
                if (t.oq && now) {
                    const uint32_t pos = base + pre[q] + uint32_t(__popcll(m[q] & lt));
                    if (pos < t.oq_cap) {
                        t.oq[queue_row0() + queue_row() * t.oq_cap + pos] =
                            kMaskQ ? (idx[q] >> 2) | (1u << (28u + (idx[q] & 3u))) : idx[q];
                        now = false;
                    }
                }
                if (__any(now)) {                              // here and now
                    uint32_t key = 0xFFFFFFFFu;
                    if (now) {                                 // only these lanes load
                        const Img<false> oim{reinterpret_cast<const uint8_t*>(o.img)};
                        const uint32_t s1[1] = {sl(q)}, d1[1] = {d[q]}, p1[1] = {dp[q]}, z1[1] = {0u};
                        uint32_t r1[1], k1[1];
                        classify_n<1, false, 0, 0, -1>(oim, o, s1, d1, p1, z1, r1, k1);
                        res[q] = r1[0];
                        key = t.n_ctr + k1[0];
                    }
                    wave_count(gslot, key);
                }
            }
        }
    }
}

// The OTHER queue: one segment of t.oq_cap entries per wave (kOtherSegs per
// workgroup), after the fills of all segments (kernels.hpp FinishArgs).
// queue_begin also clears a spare LDS word after the image's LDS (the launch
// adds 16 bytes of dynamic LDS): the hot loop counts protocol > 2 packets
// there instead of branching (they are counted by their OTHER evaluation).
template <bool kLds>
__device__ __forceinline__ uint32_t queue_begin(const Cls4Dev& t, uint4* smem) {
    const uint32_t a = kLds ? t.lds_bytes : 0u;
    if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(smem) + a) = 0u;
    if constexpr (!kLds) __syncthreads();
    return a;
}

// End of a launch: each wave's queue fill -> oq[its row] (the finish launch).
__device__ __forceinline__ void queue_end(const Cls4Dev& t, uint32_t wq) {
    if (t.oq && __lane_id() == 0u) t.oq[queue_row()] = min(wq, t.oq_cap);
}


// Copy n16 16-byte words from global memory into LDS, every thread's loads
// of a round in flight together (8 per thread: 128 KiB per round at 1024
// threads) before any is written -- a copy loop of one load and one store
// per trip waits a full memory latency per 16 KiB.
__device__ __forceinline__ void lds_copy(uint4* dst, const uint4* src, uint32_t n16) {
    constexpr int K = 8;
    for (uint32_t base = 0; base < n16; base += K * blockDim.x) {
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)          // (clamped, not guarded: the loads stay in registers)
            v[k] = src[min(base + uint32_t(k) * blockDim.x + threadIdx.x, n16 - 1u)];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = base + uint32_t(k) * blockDim.x + threadIdx.x;
            if (i < n16) dst[i] = v[k];
        }
    }
}

// Two source arrays into LDS in one round of loads where the block's
// threads can hold them (K = 10 16-B loads per thread, 160 KiB at 1024
// threads): n1 at dst, n2 at dst + at2 (16-B units).
__device__ __forceinline__ void lds_copy2(uint4* dst, const uint4* src1, uint32_t n1, uint32_t at2, const uint4* src2,
                                          uint32_t n2) {
    constexpr int K = 10;
    const uint32_t n = n1 + n2;
    for (uint32_t base = 0; base < n; base += K * blockDim.x) {
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {       // (clamped, not guarded: the loads stay in registers)
            const uint32_t i = min(base + uint32_t(k) * blockDim.x + threadIdx.x, n - 1u);
            v[k] = i < n1 ? src1[i] : src2[i - n1];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t i = base + uint32_t(k) * blockDim.x + threadIdx.x;
            if (i < n) dst[i < n1 ? i : at2 + (i - n1)] = v[k];
        }
    }
}

// Stage the read-only image into LDS (at address 0) and zero the counters.
__device__ __forceinline__ void stage_lds(const Cls4Dev& t, uint4* smem) {
    lds_copy(smem, reinterpret_cast<const uint4*>(t.img), t.img_bytes / 16u);
    uint32_t* lctr = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(smem) + t.img_bytes);
    for (uint32_t i = threadIdx.x; i < (t.lds_bytes - t.img_bytes) / 4u; i += blockDim.x) lctr[i] = 0u;
    __syncthreads();
}

// End of an LDS-resident launch: this workgroup's slot counters go plainly
// into its own row of the partials (fold_kernel sums the rows): no global
// atomics from every workgroup onto the same addresses at the end of the
// launch.  Hot slots: wave h sums slot h's per-lane row.
template <int kCtr>
__device__ __forceinline__ void flush_lds(const Cls4Dev& t, uint4* smem) {
    __syncthreads();
    const uint8_t* lds = reinterpret_cast<const uint8_t*>(smem);
    const uint32_t* lctr = reinterpret_cast<const uint32_t*>(lds + t.img_bytes);
    const uint32_t* hrow = reinterpret_cast<const uint32_t*>(lds + t.off_hot);
    uint32_t* part = t.part + size_t(blockIdx.x) * t.n_lctr;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (uint32_t h = wave; h < t.n_hot; h += blockDim.x >> 6) {
        uint32_t v = hrow[h * 64u + lane];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0 && h < t.n_lctr) part[h] = v + (kCtr == 0 ? lctr[h] : 0u);
    }
    for (uint32_t i = t.n_hot + threadIdx.x; i < t.n_lctr; i += blockDim.x) {
        if constexpr (kCtr == 0) part[i] = lctr[i];
        else part[i] = (lctr[i >> 1] >> ((i & 1u) * 16u)) & 0xFFFFu;
    }
}

template <bool kLds, bool kVec, int kMode, int kList, int kD, int kCtr>
__global__ __launch_bounds__(kClsBlock) void classify4_cls(Cls4Dev t, Cls4Dev o, Pkts4 p, uint8_t* verdict,
                                                           unsigned long long* gslot) {
    extern __shared__ uint4 smem[];
    if (t.zero)   // the call's rule counters, added to by the finish launch
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.n_zero; i += gridDim.x * blockDim.x)
            t.zero[i] = 0ull;
    Img<kLds> im{reinterpret_cast<const uint8_t*>(t.img)};
    const uint32_t oq_lds = queue_begin<kLds>(t, smem);
    uint32_t wq = 0;                                       // this wave's OTHER queue fill
    if constexpr (kLds) stage_lds(t, smem);

    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t hot0 = 0;                                     // global-image variant only
    const uint32_t hot_lane = t.off_hot + 4u * (threadIdx.x & 63u);
    uint32_t tail_from = 0;
    if constexpr (kVec) {
        // 4 packets per lane per step: 16-B (src, dst), 8-B (dport) and 4-B
        // (proto) loads, one 4-B verdict store.  32-bit indices: the host
        // splits batches at 2^30.
        const uint32_t nsteps = uint32_t(p.n / 4u);
        const uint4* S = reinterpret_cast<const uint4*>(p.src);
        const uint4* D = reinterpret_cast<const uint4*>(p.dst);
        const uint2* DP = reinterpret_cast<const uint2*>(p.dport);
        const uint32_t* PR = reinterpret_cast<const uint32_t*>(p.proto);
        auto step = [&](const uint4& s4, const uint4& d4, const uint2& p2, uint32_t pr, uint32_t g) {
            const uint32_t sa[4] = {s4.x, s4.y, s4.z, s4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
            const uint32_t pa[4] = {p2.x & 0xFFFFu, p2.x >> 16, p2.y & 0xFFFFu, p2.y >> 16};
            const uint32_t ra[4] = {pr & 0xFFu, (pr >> 8) & 0xFFu, (pr >> 16) & 0xFFu, pr >> 24};
            // some protocol byte > 2 (SWAR: bit 7 of each byte of x + 125,
            // computed without inter-byte carries)
            const bool other = ((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u;
            uint32_t v[4];
            const uint32_t ix[4] = {4u * g, 4u * g + 1u, 4u * g + 2u, 4u * g + 3u};
            run_n<4, kLds, kMode, kList, kD, kCtr, true>(im, t, o, hot_lane, gslot, hot0, sa, da, pa, ra, other, v,
                                                         [&](int q) { return sa[q]; }, ix, oq_lds, wq);
            if constexpr (kCtr == 2)                             // slot mode: 4 result words per lane
                reinterpret_cast<uint4*>(verdict)[g] = make_uint4(v[0], v[1], v[2], v[3]);
            else if (verdict)
                stnt(v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24),
                     const_cast<uint32_t*>(at(reinterpret_cast<const uint32_t*>(verdict), g)));
        };
        // Whole grid steps first (uniform trip count), plain load and use: the
        // CU's 16 waves overlap one another's loads and lookups.  (Register
        // prefetch one or two steps ahead measured slower, 0.566 / 0.583
        // against 0.559 ms, profiles/r02s4_prefetch_depth_ab_config3.txt: the
        // buffers' registers cost more than the overlap buys.)  The loads are
        // issued src, dst, dport, proto, as the stream kernel does (the
        // compiler otherwise issues proto first, for the protocol test): 0.551
        // against 0.558 ms, profiles/r03z_ab_load_order_config3.txt.  The
        // protocol stream is a cached load, the others non-temporal
        // (tools/nt_sweep.hip: the fastest of the 32 combinations).
        const uint32_t nfull = nsteps / nthreads * nthreads;
        for (uint32_t g = tid; g < nfull; g += nthreads) {
            const uint4 s4 = ldnt(at(S, g));
            __builtin_amdgcn_sched_barrier(0);
            const uint4 d4 = ldnt(at(D, g));
            __builtin_amdgcn_sched_barrier(0);
            const uint2 p2 = ldnt(at(DP, g));
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t pr = *at(PR, g);
            __builtin_amdgcn_sched_barrier(0);
            step(s4, d4, p2, pr, g);
        }
        // leftover groups one at a time
        for (uint32_t gi = nfull + tid; gi < nsteps; gi += nthreads) {
            const uint4 s4 = ldnt(at(S, gi)), d4 = ldnt(at(D, gi));
            const uint2 p2 = ldnt(at(DP, gi));
            const uint32_t pr = ldnt(at(PR, gi));
            const uint32_t sa[4] = {s4.x, s4.y, s4.z, s4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
            const uint32_t pa[4] = {p2.x & 0xFFFFu, p2.x >> 16, p2.y & 0xFFFFu, p2.y >> 16};
            const uint32_t ra[4] = {pr & 0xFFu, (pr >> 8) & 0xFFu, (pr >> 16) & 0xFFu, pr >> 24};
            uint32_t v[4];
            const uint32_t ix[4] = {4u * gi, 4u * gi + 1u, 4u * gi + 2u, 4u * gi + 3u};
            run_n<4, kLds, kMode, kList, -1, kCtr, true>(im, t, o, hot_lane, gslot, hot0, sa, da, pa, ra,
                                                         ((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u,
                                                         v, [&](int q) { return sa[q]; }, ix, oq_lds, wq);
            if constexpr (kCtr == 2)
                reinterpret_cast<uint4*>(verdict)[gi] = make_uint4(v[0], v[1], v[2], v[3]);
            else if (verdict)
                stnt(v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24),
                     const_cast<uint32_t*>(at(reinterpret_cast<const uint32_t*>(verdict), gi)));
        }
        tail_from = nsteps * 4u;
    }
    for (uint32_t i = tail_from + tid; i < uint32_t(p.n); i += nthreads) {
        const uint32_t sa[1] = {p.src[i]}, da[1] = {p.dst[i]}, pa[1] = {p.dport[i]}, ra[1] = {p.proto[i]};
        uint32_t v[1];
        const uint32_t ix[1] = {i};
        run_n<1, kLds, kMode, kList, -1, kCtr, true>(im, t, o, hot_lane, gslot, hot0, sa, da, pa, ra, ra[0] > 2u, v,
                                                     [&](int q) { return sa[q]; }, ix, oq_lds, wq);
        if constexpr (kCtr == 2) reinterpret_cast<uint32_t*>(verdict)[i] = v[0];   // slot mode: res | slot << 2
        else if (verdict) verdict[i] = uint8_t(v[0]);
    }

    if constexpr (kCtr == 2) return;
    if constexpr (!kLds) {
        if (hot0) atomicAdd(&gslot[0], (unsigned long long)hot0);
    }
    if constexpr (kLds) flush_lds<kCtr>(t, smem);
    queue_end(t, wq);
}

// ---------------------------------------------------------------------------
// 16-byte path (IPv6 and IPv4-mapped addresses, compile.hpp Cls16Image): the
// front end maps each 128-bit address to its 32-bit representative with one
// branch-free binary search over the elementary intervals (16-B keys: interval
// start - 1 as u64 hi, lo), then the IPv4 classifier runs on the reps.

// 128-bit address as loaded (network-order bytes in little-endian words)
// -> (hi, lo) u64 in address order
__device__ __forceinline__ void addr128(const uint4& a, uint64_t& hi, uint64_t& lo) {
    hi = (uint64_t(__builtin_bswap32(a.x)) << 32) | __builtin_bswap32(a.y);
    lo = (uint64_t(__builtin_bswap32(a.z)) << 32) | __builtin_bswap32(a.w);
}

template <int N, bool kLds>
__device__ __forceinline__ void fe_rep(const Img<kLds>& im, uint32_t off_key, uint32_t off_val,
                                       uint32_t top, uint32_t k8, const uint4 (&a)[N], uint32_t (&rep)[N]) {
    uint64_t kh[N], kl[N];
    uint32_t pos[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        addr128(a[q], kh[q], kl[q]);
        pos[q] = off_key;
    }
    if (k8) {
        // 8-B keys (compile.hpp key8): half the LDS bytes and one 64-bit compare per step
        constexpr uint64_t kLo = 1ull << 48, kHiMax = ~0ull - kLo;
        uint64_t k[N];
#pragma unroll
        for (int q = 0; q < N; ++q) k[q] = kh[q] == 0 ? min(kl[q], kLo) : kLo + min(kh[q], kHiMax);
#pragma unroll 1
        for (uint32_t s = top >> 1; s; s >>= 1) {
            const uint32_t step = 8u * s;
            uint2 e[N];
#pragma unroll
            for (int q = 0; q < N; ++q) e[q] = im.u64(pos[q] + step);
#pragma unroll
            for (int q = 0; q < N; ++q) pos[q] = ((uint64_t(e[q].y) << 32) | e[q].x) < k[q] ? pos[q] + step : pos[q];
        }
#pragma unroll
        for (int q = 0; q < N; ++q) rep[q] = im.u32(off_val + ((pos[q] - off_key) >> 1));
        return;
    }
#pragma unroll 1
    for (uint32_t s = top >> 1; s; s >>= 1) {
        const uint32_t step = 16u * s;
        uint4 e[N];
#pragma unroll
        for (int q = 0; q < N; ++q) e[q] = im.u128(pos[q] + step);
#pragma unroll
        for (int q = 0; q < N; ++q) {
            const uint64_t eh = (uint64_t(e[q].y) << 32) | e[q].x, el = (uint64_t(e[q].w) << 32) | e[q].z;
            const bool lt = eh < kh[q] || (eh == kh[q] && el < kl[q]);      // start - 1 < addr
            pos[q] = lt ? pos[q] + step : pos[q];
        }
    }
#pragma unroll
    for (int q = 0; q < N; ++q) rep[q] = im.u32(off_val + ((pos[q] - off_key) >> 2));
}

// Linear first match over the rules in rep space (the 16-byte path's GPU
// cross-check, CLS_F_FORCE_LINEAR): direct rule slots after the n_ctr slots.
template <int N>
__device__ __forceinline__ void lin_n(const Cls4Dev& t, unsigned long long* gslot, const uint32_t (&s)[N],
                                      const uint32_t (&d)[N], const uint32_t (&dp)[N],
                                      const uint32_t (&pr)[N], uint32_t (&res)[N]) {
#pragma unroll
    for (int q = 0; q < N; ++q) {
        uint32_t rule;
        linear_one(t.lin, t.n_lin, t.n_rules, s[q], d[q], dp[q], min(pr[q], 3u), res[q], rule);
        atomicAdd(&gslot[t.n_ctr + rule], 1ull);
    }
}

// Source rows of N 16-byte addresses from the host-route hashes (src_mode 1):
// both families' probes for every lane (a wave holds both), the family
// picked per lane.  IPv4-mapped = bytes 0-9 zero, bytes 10-11 0xFF (Go To4).
template <int N, bool kLds>
__device__ __forceinline__ void src_hash16(const Img<kLds>& im, const Fe16& fe, const uint4 (&a)[N],
                                           uint32_t (&row)[N]) {
    uint2 e0[N], e1[N];
    uint4 c0[N], c1[N];
    uint32_t v0[N], v1[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const uint32_t h = a[q].w * fe.mul4;
        e0[q] = im.u64(fe.h4 + 8u * (h >> fe.s4_0));
        e1[q] = im.u64(fe.h4 + 8u * fe.cap4 + 8u * __builtin_amdgcn_ubfe(h, fe.s4_1, fe.L4));
        const uint32_t g = fold6(a[q].x, a[q].y, a[q].z, a[q].w, fe.fold) * fe.mul6;
        const uint32_t p0 = g >> fe.s6_0, p1 = fe.cap6 + __builtin_amdgcn_ubfe(g, fe.s6_1, fe.L6);
        c0[q] = im.u128(fe.k6 + 16u * p0);
        c1[q] = im.u128(fe.k6 + 16u * p1);
        v0[q] = im.u32(fe.r6 + 4u * p0);
        v1[q] = im.u32(fe.r6 + 4u * p1);
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const uint4 x = a[q];
        const bool is4 = (x.x | x.y) == 0u && x.z == 0xFFFF0000u;
        uint32_t r4 = e1[q].x == x.w ? e1[q].y : fe.dflt4;
        r4 = e0[q].x == x.w ? e0[q].y : r4;
        const bool m1 = c1[q].x == x.x && c1[q].y == x.y && c1[q].z == x.z && c1[q].w == x.w;
        const bool m0 = c0[q].x == x.x && c0[q].y == x.y && c0[q].z == x.z && c0[q].w == x.w;
        uint32_t r6 = m1 ? v1[q] : fe.dflt6;
        r6 = m0 ? v0[q] : r6;
        row[q] = is4 ? r4 : r6;
    }
}

// Source rows of N 16-byte addresses, src_mode 2 (compile.hpp Cls16Image):
// IPv4-mapped addresses through the trie over their IPv4 word (the core's
// off_trie / trie_depth, leaves carrying core classes: src_row mode 4), the
// others through the interval search over the non-IPv4 intervals, whose
// values are rows -- taken only when some lane of the wave holds one.
template <int N, bool kLds>
__device__ __forceinline__ void src_trie16(const Img<kLds>& im, const Cls4Dev& t, const Fe16& fe, const uint4 (&a)[N],
                                           uint32_t (&row)[N]) {
    uint32_t ip[N];
    bool v6 = false;
#pragma unroll
    for (int q = 0; q < N; ++q) {
        ip[q] = __builtin_bswap32(a[q].w);
        v6 |= !((a[q].x | a[q].y) == 0u && a[q].z == 0xFFFF0000u);
    }
    src_row<N, kLds, 4>(im, t, ip, row);
    if (__any(v6)) {
        uint32_t r6[N];
        fe_rep(im, fe.key[0], fe.val[0], fe.top[0], fe.k8[0], a, r6);
#pragma unroll
        for (int q = 0; q < N; ++q)
            row[q] = ((a[q].x | a[q].y) == 0u && a[q].z == 0xFFFF0000u) ? row[q] : r6[q];
    }
}

// The source rep of one address from the global-memory interval table
// (src_mode 1 and 2, protocol > 2 lanes only): out of line, so the rare path
// costs the hot loop no registers.
[[maybe_unused]] __device__ __noinline__ uint32_t src_rep_global(const uint8_t* g, uint32_t gval, uint32_t top, uint32_t k8,
                                                uint4 a) {
    const uint4 a1[1] = {a};
    uint32_t r[1];
    fe_rep(Img<false>{g}, 0u, gval, top, k8, a1, r);
    return r[0];
}

template <bool kLds, int kMode, int kList, int kD, bool kLin, int kFe, int kCtr>
__global__ __launch_bounds__(kClsBlock) void classify16_cls(Cls4Dev t, Cls4Dev o, Fe16 fe, Pkts16 p,
                                                            uint8_t* verdict, unsigned long long* gslot) {
    extern __shared__ uint4 smem[];
    if (t.zero)   // the call's rule counters, added to by the finish launch
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < t.n_zero; i += gridDim.x * blockDim.x)
            t.zero[i] = 0ull;
    Img<kLds> im{reinterpret_cast<const uint8_t*>(t.img)};
    const uint32_t oq_lds = queue_begin<kLds>(t, smem);
    uint32_t wq = 0;                                       // this wave's OTHER queue fill
    if constexpr (kLds) stage_lds(t, smem);
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t hot0 = 0;
    const uint32_t hot_lane = t.off_hot + 4u * (threadIdx.x & 63u);
    // src_mode 1 and 2 keep the source interval table in global memory: reps
    // for the linear paths (protocol > 2 fallback, CLS_F_FORCE_LINEAR)
    const Img<false> gim{fe.gsrc};
    auto src_rep = [&](const auto& a, auto& out) {
        if constexpr (kFe >= 1) fe_rep(gim, 0u, fe.gval, fe.gtop, fe.gk8, a, out);
        else fe_rep(im, fe.key[0], fe.val[0], fe.top[0], fe.k8[0], a, out);
    };
    auto classify = [&](const auto& s16, const auto& d16, auto& pa, auto& ra, bool other, auto& v, const auto& ix) {
        constexpr int N = sizeof(v) / 4;
        uint32_t sa[N], da[N];
        fe_rep(im, fe.key[1], fe.val[1], fe.top[1], fe.k8[1], d16, da);
        if constexpr (kLin) {
            src_rep(s16, sa);
            lin_n(t, gslot + o.n_ctr, sa, da, pa, ra, v);   // direct rule slots after both images
        } else if constexpr (kFe >= 1) {
            if constexpr (kFe == 1) src_hash16(im, fe, s16, sa);   // class rows, not reps
            else src_trie16(im, t, fe, s16, sa);
            // protocols > 2 need the source's rep (the OTHER image is in rep
            // space): only for a packet classified in place, not queued
            run_n<N, kLds, kMode, kList, kD, kCtr>(
                im, t, o, hot_lane, gslot, hot0, sa, da, pa, ra, other, v,
                [&](int q) { return src_rep_global(fe.gsrc, fe.gval, fe.gtop, fe.gk8, s16[q]); }, ix, oq_lds, wq);
        } else {
            src_rep(s16, sa);
            run_n<N, kLds, kMode, kList, kD, kCtr>(im, t, o, hot_lane, gslot, hot0, sa, da, pa, ra, other, v,
                                                   [&](int q) { return sa[q]; }, ix, oq_lds, wq);
        }
    };
    // 4 packets per lane per step (vector dport / proto / verdict words).
    // Wave-contiguous packets: a wave's step covers 256 consecutive packets
    // and lane l takes packets base + 64k + l (k = 0..3), so each 16-B
    // address load instruction reads 1 KiB contiguous per wave (the
    // lane-owns-4-consecutive order strides 64 B per lane and fetched 25 %
    // more than the algorithmic bytes, profiles/r01_pmc_config5_lane4order.json);
    // dport / proto / verdict move one element per packet, also contiguous
    // per instruction.  Whole waves only (nsteps a multiple of 64 groups of 4,
    // wave-uniform); the rest goes to the per-packet tail.
    const uint32_t nsteps = uint32_t(p.n / 256u) * 64u;
    struct Step16 {
        uint4 s[4], d[4];
        uint32_t dp[4], pr[4];
    };
    auto load = [&](Step16& b, uint32_t g) {
        const uint32_t base = 4u * (g & ~63u) + (g & 63u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            b.s[k] = ldnt(at(p.src, base + 64u * k));
            b.d[k] = ldnt(at(p.dst, base + 64u * k));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            b.dp[k] = __builtin_nontemporal_load(p.dport + base + 64u * k);
            b.pr[k] = __builtin_nontemporal_load(p.proto + base + 64u * k);
        }
    };
    // The step's four packets, G at a time: with the host-route hashes
    // (src_mode 1) a 16-byte packet's lookups hold about twice the registers
    // of an IPv4 one, so two, to stay within 128 VGPRs (1024-thread
    // workgroups) without scratch; the trie and interval front ends fit all
    // four, whose LDS chains then run interleaved.  The CU's 16 waves overlap
    // one another's loads and lookups: the next step's loads held in
    // registers during this step's lookups (two at a time, in the order the
    // vmcnt counter can serve) measured no faster on the gen-policy lists
    // (profiles/r04j_genpolicy16_prefetch_ab.txt).
    constexpr int G = kFe == 1 ? 2 : 4;
    auto run = [&](const Step16& b, uint32_t g, uint32_t (&v)[4]) {
        const uint32_t base = 4u * (g & ~63u) + (g & 63u);
#pragma unroll
        for (int h = 0; h < 4 / G; ++h) {
            uint4 sg[G], dg[G];
            uint32_t pa[G], ra[G], vg[G], ix[G], any = 0u;
#pragma unroll
            for (int q = 0; q < G; ++q) {
                sg[q] = b.s[G * h + q];
                dg[q] = b.d[G * h + q];
                pa[q] = b.dp[G * h + q];
                ra[q] = b.pr[G * h + q];
                ix[q] = base + 64u * (G * h + q);
                any |= ra[q];
            }
            classify(sg, dg, pa, ra, any > 2u, vg, ix);
#pragma unroll
            for (int q = 0; q < G; ++q) v[G * h + q] = vg[q];
        }
    };
    auto put = [&](const uint32_t (&v)[4], uint32_t g) {
        const uint32_t base = 4u * (g & ~63u) + (g & 63u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (kCtr == 2) reinterpret_cast<uint32_t*>(verdict)[base + 64u * k] = v[k];   // slot mode: res | slot << 2
            else if (verdict) __builtin_nontemporal_store(uint8_t(v[k]), verdict + base + 64u * k);
        }
    };
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        Step16 b;
        uint32_t v[4];
        load(b, g);
        run(b, g, v);
        put(v, g);
    }
    for (uint32_t i = nsteps * 4u + tid; i < uint32_t(p.n); i += nthreads) {
        const uint4 s1[1] = {ldnt(at(p.src, i))}, d1[1] = {ldnt(at(p.dst, i))};
        uint32_t v[1];
        uint32_t pa[1] = {p.dport[i]}, ra[1] = {p.proto[i]};
        const uint32_t ix[1] = {i};
        classify(s1, d1, pa, ra, ra[0] > 2u, v, ix);
        if constexpr (kCtr == 2) reinterpret_cast<uint32_t*>(verdict)[i] = v[0];
        else if (verdict) verdict[i] = uint8_t(v[0]);
    }
    if constexpr (kCtr == 2) return;
    if constexpr (!kLds) {
        if (hot0) atomicAdd(&gslot[0], (unsigned long long)hot0);
    }
    if constexpr (kLds) flush_lds<kCtr>(t, smem);
    queue_end(t, wq);
}

}  // namespace

template <bool kLds, bool kVec, int kMode, int kList, int kD, int kCtr = 0>
static void launch_d(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                     const LaunchCfg& cfg) {
    const size_t lds = (kLds ? t.lds_bytes : 0) + 16;   // + the OTHER queue counter
    lds_attr<classify4_cls<kLds, kVec, kMode, kList, kD, kCtr>>();
    if (cfg.ev_start || cfg.ev_stop)
        hipExtLaunchKernelGGL((classify4_cls<kLds, kVec, kMode, kList, kD, kCtr>), dim3(cfg.grid), dim3(kClsBlock),
                              uint32_t(lds), cfg.stream, cfg.ev_start, cfg.ev_stop, 0u, t, cfg.other, p, verdict, gslot);
    else
        hipLaunchKernelGGL((classify4_cls<kLds, kVec, kMode, kList, kD, kCtr>), dim3(cfg.grid), dim3(kClsBlock), lds,
                           cfg.stream, t, cfg.other, p, verdict, gslot);
}

// The hot variants (LDS-resident image, vector loads, sublist lists, u32
// LDS counters) are specialised on the search depth; the others take it at
// run time.
template <bool kLds, bool kVec, int kMode, int kList>
static void launch_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                       const LaunchCfg& cfg) {
    if constexpr (kLds) {
        if (t.ctr16) {
            launch_d<kLds, kVec, kMode, kList, -1, 1>(t, p, verdict, gslot, cfg);
            return;
        }
    }
    if constexpr (kLds && kVec && (kList == 3 || kList == 4)) {
        switch (int(t.bv_steps)) {
        case 0: launch_d<kLds, kVec, kMode, kList, 0>(t, p, verdict, gslot, cfg); return;
        case 1: launch_d<kLds, kVec, kMode, kList, 1>(t, p, verdict, gslot, cfg); return;
        case 2: launch_d<kLds, kVec, kMode, kList, 2>(t, p, verdict, gslot, cfg); return;
        case 3: launch_d<kLds, kVec, kMode, kList, 3>(t, p, verdict, gslot, cfg); return;
        case 4: launch_d<kLds, kVec, kMode, kList, 4>(t, p, verdict, gslot, cfg); return;
        case 5: launch_d<kLds, kVec, kMode, kList, 5>(t, p, verdict, gslot, cfg); return;
        default: break;
        }
    }
    launch_d<kLds, kVec, kMode, kList, -1>(t, p, verdict, gslot, cfg);
}

// source lookup variant: 0 interval search, 1 hash LPM, 2 hash LPM with one
// length, 3 source trie (kMode 4)
static inline int src_variant(const Cls4Dev& t) {
    return t.mode == 4 ? 3 : t.mode != 1 ? 0 : t.n_hash == 1 ? 2 : 1;
}

// Whether the dispatchers below have a kernel for this image (kernels.hpp
// cls_kernel_exists: the engine refuses the others at put time, the
// launchers check again, so a combination without a case is an error, never
// another variant's kernel reading the image wrongly).
static inline bool cls_dispatchable(const Cls4Dev& t, bool lds, bool rep16) {
    return cls_kernel_exists(t.mode, t.list_mode, lds, rep16);
}

template <bool kLds, bool kVec>
static void dispatch_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                         const LaunchCfg& cfg) {
    const int src = src_variant(t);
    if constexpr (kLds) {
        // the source trie (sublist modes) and the wide cells (LDS-resident
        // images only)
        if (src == 3 || t.list_mode >= 5) {
#define CLS_TW_CASES(L)                                                                       \
    case 4 * L + 0: launch_cls<kLds, kVec, 0, L>(t, p, verdict, gslot, cfg); return;          \
    case 4 * L + 1: launch_cls<kLds, kVec, 1, L>(t, p, verdict, gslot, cfg); return;          \
    case 4 * L + 2: launch_cls<kLds, kVec, 2, L>(t, p, verdict, gslot, cfg); return;          \
    case 4 * L + 3: launch_cls<kLds, kVec, 4, L>(t, p, verdict, gslot, cfg); return;
            switch (src + 4 * int(t.list_mode)) {
                case 4 * 3 + 3: launch_cls<kLds, kVec, 4, 3>(t, p, verdict, gslot, cfg); return;
                case 4 * 4 + 3: launch_cls<kLds, kVec, 4, 4>(t, p, verdict, gslot, cfg); return;
                CLS_TW_CASES(5)
                CLS_TW_CASES(6)
            default: return;
            }
#undef CLS_TW_CASES
        }
    }
#define CLS_SRC_CASES(L)                                                                   \
    case 3 * L + 0: launch_cls<kLds, kVec, 0, L>(t, p, verdict, gslot, cfg); break;        \
    case 3 * L + 1: launch_cls<kLds, kVec, 1, L>(t, p, verdict, gslot, cfg); break;        \
    case 3 * L + 2: launch_cls<kLds, kVec, 2, L>(t, p, verdict, gslot, cfg); break;
    switch (src + 3 * int(t.list_mode)) {
        CLS_SRC_CASES(0)
        CLS_SRC_CASES(1)
        CLS_SRC_CASES(2)
        CLS_SRC_CASES(3)
        CLS_SRC_CASES(4)
    default: break;
    }
#undef CLS_SRC_CASES
}

template <bool kLds, int kMode, int kList, int kD, bool kLin, int kFe, int kCtr = 0>
static void launch16_d(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint8_t* verdict,
                       unsigned long long* gslot, const LaunchCfg& cfg) {
    const size_t lds = (kLds ? t.lds_bytes : 0) + 16;   // + the OTHER queue counter
    lds_attr<classify16_cls<kLds, kMode, kList, kD, kLin, kFe, kCtr>>();
    if (cfg.ev_start || cfg.ev_stop)
        hipExtLaunchKernelGGL((classify16_cls<kLds, kMode, kList, kD, kLin, kFe, kCtr>), dim3(cfg.grid),
                              dim3(kClsBlock), uint32_t(lds), cfg.stream, cfg.ev_start, cfg.ev_stop, 0u, t, cfg.other,
                              fe, p, verdict, gslot);
    else
        hipLaunchKernelGGL((classify16_cls<kLds, kMode, kList, kD, kLin, kFe, kCtr>), dim3(cfg.grid), dim3(kClsBlock),
                           lds, cfg.stream, t, cfg.other, fe, p, verdict, gslot);
}

template <bool kLds, int kMode, int kList, int kFe>
static void launch16_cls(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint8_t* verdict,
                         unsigned long long* gslot, const LaunchCfg& cfg) {
    if constexpr (kLds) {
        if (t.ctr16) {
            launch16_d<kLds, kMode, kList, -1, false, kFe, 1>(t, fe, p, verdict, gslot, cfg);
            return;
        }
    }
    if constexpr (kLds && (kList == 3 || kList == 4) && kFe != 2) {
        switch (int(t.bv_steps)) {
        case 0: launch16_d<kLds, kMode, kList, 0, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        case 1: launch16_d<kLds, kMode, kList, 1, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        case 2: launch16_d<kLds, kMode, kList, 2, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        case 3: launch16_d<kLds, kMode, kList, 3, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        case 4: launch16_d<kLds, kMode, kList, 4, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        case 5: launch16_d<kLds, kMode, kList, 5, false, kFe>(t, fe, p, verdict, gslot, cfg); return;
        default: break;
        }
    }
    launch16_d<kLds, kMode, kList, -1, false, kFe>(t, fe, p, verdict, gslot, cfg);
}

template <bool kLds>
static void dispatch16(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint8_t* verdict,
                       unsigned long long* gslot, bool lin, const LaunchCfg& cfg) {
    if (lin) {
        if (fe.src_mode >= 1) launch16_d<kLds, 0, 0, -1, true, 1>(t, fe, p, verdict, gslot, cfg);
        else launch16_d<kLds, 0, 0, -1, true, 0>(t, fe, p, verdict, gslot, cfg);
        return;
    }
    if (fe.src_mode == 1) {                      // rows from the host-route hashes (core mode 3)
        switch (t.list_mode) {
        case 0: launch16_cls<kLds, 3, 0, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 1: launch16_cls<kLds, 3, 1, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 2: launch16_cls<kLds, 3, 2, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 3: launch16_cls<kLds, 3, 3, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 4: launch16_cls<kLds, 3, 4, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 5: if constexpr (kLds) launch16_cls<kLds, 3, 5, 1>(t, fe, p, verdict, gslot, cfg); break;
        case 6: if constexpr (kLds) launch16_cls<kLds, 3, 6, 1>(t, fe, p, verdict, gslot, cfg); break;
        default: break;
        }
        return;
    }
    if (fe.src_mode == 2) {                      // rows from the IPv4 trie / non-IPv4 search (core mode 3)
        switch (t.list_mode) {
        case 0: launch16_cls<kLds, 3, 0, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 1: launch16_cls<kLds, 3, 1, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 2: launch16_cls<kLds, 3, 2, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 3: launch16_cls<kLds, 3, 3, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 4: launch16_cls<kLds, 3, 4, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 5: if constexpr (kLds) launch16_cls<kLds, 3, 5, 2>(t, fe, p, verdict, gslot, cfg); break;
        case 6: if constexpr (kLds) launch16_cls<kLds, 3, 6, 2>(t, fe, p, verdict, gslot, cfg); break;
        default: break;
        }
        return;
    }
    const int src = src_variant(t);
    if constexpr (kLds) {
        // the source trie over reps (sublist modes) and the wide cells (LDS-resident images only)
        if (src == 3 || t.list_mode >= 5) {
#define CLS16_TW_CASES(L)                                                                     \
    case 4 * L + 0: launch16_cls<kLds, 0, L, 0>(t, fe, p, verdict, gslot, cfg); return;       \
    case 4 * L + 1: launch16_cls<kLds, 1, L, 0>(t, fe, p, verdict, gslot, cfg); return;       \
    case 4 * L + 2: launch16_cls<kLds, 2, L, 0>(t, fe, p, verdict, gslot, cfg); return;       \
    case 4 * L + 3: launch16_cls<kLds, 4, L, 0>(t, fe, p, verdict, gslot, cfg); return;
            switch (src + 4 * int(t.list_mode)) {
                case 4 * 3 + 3: launch16_cls<kLds, 4, 3, 0>(t, fe, p, verdict, gslot, cfg); return;
                case 4 * 4 + 3: launch16_cls<kLds, 4, 4, 0>(t, fe, p, verdict, gslot, cfg); return;
                CLS16_TW_CASES(5)
                CLS16_TW_CASES(6)
            default: return;
            }
#undef CLS16_TW_CASES
        }
    }
#define CLS16_SRC_CASES(L)                                                                  \
    case 3 * L + 0: launch16_cls<kLds, 0, L, 0>(t, fe, p, verdict, gslot, cfg); break;      \
    case 3 * L + 1: launch16_cls<kLds, 1, L, 0>(t, fe, p, verdict, gslot, cfg); break;      \
    case 3 * L + 2: launch16_cls<kLds, 2, L, 0>(t, fe, p, verdict, gslot, cfg); break;
    switch (src + 3 * int(t.list_mode)) {
        CLS16_SRC_CASES(0)
        CLS16_SRC_CASES(1)
        CLS16_SRC_CASES(2)
        CLS16_SRC_CASES(3)
        CLS16_SRC_CASES(4)
    default: break;
    }
#undef CLS16_SRC_CASES
}

// Slot mode, run-time search depth: 4 packets per lane (vector loads, one
// 16-B result store) for an LDS-resident image on aligned arrays, else one
// packet per lane.
template <bool kLds>
static void dispatch_slots4(const Cls4Dev& t, const Pkts4& p, uint32_t* out, const LaunchCfg& cfg) {
    uint8_t* o = reinterpret_cast<uint8_t*>(out);
    const int src = src_variant(t);
    if constexpr (kLds) {
        auto al = [](const void* q, uintptr_t a) { return (reinterpret_cast<uintptr_t>(q) & (a - 1)) == 0; };
        if (src == 3 || t.list_mode >= 5) {           // source trie / wide cells
#define CLS_SLOTTW_CASES(L)                                                                        \
    case 4 * L + 0: launch_d<true, false, 0, L, -1, 2>(t, p, o, nullptr, cfg); return;             \
    case 4 * L + 1: launch_d<true, false, 1, L, -1, 2>(t, p, o, nullptr, cfg); return;             \
    case 4 * L + 2: launch_d<true, false, 2, L, -1, 2>(t, p, o, nullptr, cfg); return;             \
    case 4 * L + 3: launch_d<true, false, 4, L, -1, 2>(t, p, o, nullptr, cfg); return;
            switch (src + 4 * int(t.list_mode)) {
                case 4 * 3 + 3: launch_d<true, false, 4, 3, -1, 2>(t, p, o, nullptr, cfg); return;
                case 4 * 4 + 3: launch_d<true, false, 4, 4, -1, 2>(t, p, o, nullptr, cfg); return;
                CLS_SLOTTW_CASES(5)
                CLS_SLOTTW_CASES(6)
            default: return;
            }
#undef CLS_SLOTTW_CASES
        }
        if (al(p.src, 16) && al(p.dst, 16) && al(p.dport, 8) && al(p.proto, 4) && al(out, 16)) {
#define CLS_SLOTV_CASES(L)                                                                         \
    case 3 * L + 0: launch_d<true, true, 0, L, -1, 2>(t, p, o, nullptr, cfg); return;              \
    case 3 * L + 1: launch_d<true, true, 1, L, -1, 2>(t, p, o, nullptr, cfg); return;              \
    case 3 * L + 2: launch_d<true, true, 2, L, -1, 2>(t, p, o, nullptr, cfg); return;
            switch (src + 3 * int(t.list_mode)) {
                CLS_SLOTV_CASES(0)
                CLS_SLOTV_CASES(1)
                CLS_SLOTV_CASES(2)
                CLS_SLOTV_CASES(3)
                CLS_SLOTV_CASES(4)
            default: break;
            }
#undef CLS_SLOTV_CASES
        }
    }
#define CLS_SLOT_CASES(L)                                                                          \
    case 3 * L + 0: launch_d<kLds, false, 0, L, -1, 2>(t, p, o, nullptr, cfg); break;              \
    case 3 * L + 1: launch_d<kLds, false, 1, L, -1, 2>(t, p, o, nullptr, cfg); break;              \
    case 3 * L + 2: launch_d<kLds, false, 2, L, -1, 2>(t, p, o, nullptr, cfg); break;
    switch (src + 3 * int(t.list_mode)) {
        CLS_SLOT_CASES(0)
        CLS_SLOT_CASES(1)
        CLS_SLOT_CASES(2)
        CLS_SLOT_CASES(3)
        CLS_SLOT_CASES(4)
    default: break;
    }
#undef CLS_SLOT_CASES
}

template <bool kLds>
static void dispatch_slots16(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint32_t* out,
                             const LaunchCfg& cfg) {
    uint8_t* o = reinterpret_cast<uint8_t*>(out);
    if (fe.src_mode == 2) {
        switch (t.list_mode) {
        case 0: launch16_d<kLds, 3, 0, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 1: launch16_d<kLds, 3, 1, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 2: launch16_d<kLds, 3, 2, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 3: launch16_d<kLds, 3, 3, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 4: launch16_d<kLds, 3, 4, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 5: if constexpr (kLds) launch16_d<kLds, 3, 5, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        case 6: if constexpr (kLds) launch16_d<kLds, 3, 6, -1, false, 2, 2>(t, fe, p, o, nullptr, cfg); break;
        default: break;
        }
        return;
    }
    if (fe.src_mode == 1) {
        switch (t.list_mode) {
        case 0: launch16_d<kLds, 3, 0, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 1: launch16_d<kLds, 3, 1, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 2: launch16_d<kLds, 3, 2, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 3: launch16_d<kLds, 3, 3, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 4: launch16_d<kLds, 3, 4, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 5: if constexpr (kLds) launch16_d<kLds, 3, 5, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        case 6: if constexpr (kLds) launch16_d<kLds, 3, 6, -1, false, 1, 2>(t, fe, p, o, nullptr, cfg); break;
        default: break;
        }
        return;
    }
    const int src = src_variant(t);
    if constexpr (kLds) {
        if (src == 3 || t.list_mode >= 5) {
#define CLS16_SLOTTW_CASES(L)                                                                      \
    case 4 * L + 0: launch16_d<kLds, 0, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;    \
    case 4 * L + 1: launch16_d<kLds, 1, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;    \
    case 4 * L + 2: launch16_d<kLds, 2, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;    \
    case 4 * L + 3: launch16_d<kLds, 4, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;
            switch (src + 4 * int(t.list_mode)) {
                case 4 * 3 + 3: launch16_d<kLds, 4, 3, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;
                case 4 * 4 + 3: launch16_d<kLds, 4, 4, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); return;
                CLS16_SLOTTW_CASES(5)
                CLS16_SLOTTW_CASES(6)
            default: return;
            }
#undef CLS16_SLOTTW_CASES
        }
    }
#define CLS16_SLOT_CASES(L)                                                                        \
    case 3 * L + 0: launch16_d<kLds, 0, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); break;     \
    case 3 * L + 1: launch16_d<kLds, 1, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); break;     \
    case 3 * L + 2: launch16_d<kLds, 2, L, -1, false, 0, 2>(t, fe, p, o, nullptr, cfg); break;
    switch (src + 3 * int(t.list_mode)) {
        CLS16_SLOT_CASES(0)
        CLS16_SLOT_CASES(1)
        CLS16_SLOT_CASES(2)
        CLS16_SLOT_CASES(3)
        CLS16_SLOT_CASES(4)
    default: break;
    }
#undef CLS16_SLOT_CASES
}

// the LDS-resident vector-load variants of classify4_cls (k4_ldsv.hip)
hipError_t launch_cls4_lds_vec(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                               const LaunchCfg& cfg);

}  // namespace cls
