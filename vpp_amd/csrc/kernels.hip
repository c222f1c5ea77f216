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

template <typename Base>
__device__ __forceinline__ void cls4_one(Base base, const Cls4Dev& t, uint32_t src, uint32_t dst,
                                         uint32_t dport, uint32_t proto, uint32_t& res,
                                         uint32_t& slot) {
    const uint32_t* __restrict__ b = reinterpret_cast<const uint32_t*>(base + t.off_bounds);
    uint32_t k = 0;
#pragma unroll 1
    for (uint32_t s = t.search_top; s; s >>= 1) {
        const uint32_t c = k + s;
        k = (b[c] <= src) ? c : k;
    }
    const uint32_t cls = reinterpret_cast<const uint16_t*>(base + t.off_iclass)[k];
    const uint2 cell = reinterpret_cast<const uint2*>(base + t.off_cells)[cls * 3u + proto];
    const uint16_t* __restrict__ L = reinterpret_cast<const uint16_t*>(base + t.off_lists) + (cell.x & 0xFFFFu);
    const uint4* __restrict__ T = reinterpret_cast<const uint4*>(base + t.off_tmpl);
    const uint32_t len = cell.x >> 16;
    res = 0;
    slot = 0;
    for (uint32_t j = 0; j < len; ++j) {
        const uint4 tm = T[L[j]];
        if (((dst ^ tm.x) & tm.y) == 0 && port_in(dport, tm.z)) {
            res = tm.w;
            slot = cell.y + j;
            break;
        }
    }
}

template <bool kLds, bool kVec>
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
        for (uint32_t i = threadIdx.x; i < t.n_ctr; i += blockDim.x) lctr[i] = 0u;
        __syncthreads();
        base = reinterpret_cast<const uint8_t*>(smem);
    } else {
        base = reinterpret_cast<const uint8_t*>(t.img);
    }

    auto one = [&](uint32_t s, uint32_t d, uint32_t dp, uint32_t pr) -> uint32_t {
        uint32_t res, slot;
        if (pr <= 2u) {
            if constexpr (kLds)
                cls4_one(reinterpret_cast<const uint8_t*>(smem), t, s, d, dp, pr, res, slot);
            else
                cls4_one(base, t, s, d, dp, pr, res, slot);
            if constexpr (kLds)
                atomicAdd(&lctr[slot], 1u);
            else
                atomicAdd(&gslot[slot], 1ull);
        } else {
            uint32_t rule;
            linear_one(t.lin, t.n_lin, t.n_rules, s, d, dp, 3u, res, rule);
            atomicAdd(&gslot[t.n_ctr + rule], 1ull);
        }
        return res;
    };

    const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if constexpr (kVec) {
        const uint64_t ngroups = p.n / 4u;
        for (uint64_t g = tid; g < ngroups; g += nthreads) {
            const uint4 s = reinterpret_cast<const uint4*>(p.src)[g];
            const uint4 d = reinterpret_cast<const uint4*>(p.dst)[g];
            const uint2 dp = reinterpret_cast<const uint2*>(p.dport)[g];
            const uint32_t pr = reinterpret_cast<const uint32_t*>(p.proto)[g];
            const uint32_t v0 = one(s.x, d.x, dp.x & 0xFFFFu, pr & 0xFFu);
            const uint32_t v1 = one(s.y, d.y, dp.x >> 16, (pr >> 8) & 0xFFu);
            const uint32_t v2 = one(s.z, d.z, dp.y & 0xFFFFu, (pr >> 16) & 0xFFu);
            const uint32_t v3 = one(s.w, d.w, dp.y >> 16, pr >> 24);
            if (verdict)
                reinterpret_cast<uint32_t*>(verdict)[g] = v0 | (v1 << 8) | (v2 << 16) | (v3 << 24);
        }
        for (uint64_t i = ngroups * 4u + tid; i < p.n; i += nthreads) {
            const uint32_t v = one(p.src[i], p.dst[i], p.dport[i], p.proto[i]);
            if (verdict) verdict[i] = uint8_t(v);
        }
    } else {
        for (uint64_t i = tid; i < p.n; i += nthreads) {
            const uint32_t v = one(p.src[i], p.dst[i], p.dport[i], p.proto[i]);
            if (verdict) verdict[i] = uint8_t(v);
        }
    }

    if constexpr (kLds) {
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

hipError_t launch_classify4_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict,
                                unsigned long long* gslot, bool lds_resident, bool vec,
                                const LaunchCfg& cfg) {
    dim3 grid(cfg.grid), block(kBlock);
    if (lds_resident) {
        const size_t lds = t.lds_bytes;
        if (vec) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(classify4_cls<true, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
            hipLaunchKernelGGL((classify4_cls<true, true>), grid, block, lds, cfg.stream, t, p, verdict, gslot);
        } else {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(classify4_cls<true, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
            hipLaunchKernelGGL((classify4_cls<true, false>), grid, block, lds, cfg.stream, t, p, verdict, gslot);
        }
    } else {
        if (vec)
            hipLaunchKernelGGL((classify4_cls<false, true>), grid, block, 0, cfg.stream, t, p, verdict, gslot);
        else
            hipLaunchKernelGGL((classify4_cls<false, false>), grid, block, 0, cfg.stream, t, p, verdict, gslot);
    }
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
