// Can the classify kernel's IPv4 packet stream (src u32, dst u32, dport u16,
// proto u8 read, verdict u8 written: 12 B per packet) move faster through
// LDS-DMA (global_load_lds, no VGPR destination) than through register
// loads?  The lookups are left out; every variant runs on the classify grid
// (one 1024-thread workgroup per CU) over 256 Mi packets.
//   R0  register loads as classify4_cls: per lane 4 packets (16-B src, 16-B
//       dst nt, 8-B dport nt, 4-B proto), 4-B nt verdict store
//   R1  R0 without the verdict store (reads only)
//   D0  per wave: the step's 256 packets DMA'd into the wave's LDS slot
//       (src 1 KiB, dst 1 KiB, dport 512 B, proto 256 B; nt), vmcnt(0),
//       ds_read into the same registers as R0, verdict stored as R0
//   D1  D0 double-buffered: the next step's DMA issued before this step's reads
//   D2  D1 without the verdict store
//   D3  D1 with 128-packet steps (two lanes' worth of LDS per packet group)
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream_glds.bin tools/stream_glds.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_t;

__device__ __forceinline__ uint4 ldnt(const uint4* p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ldnt(const uint2* p) {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t mix(uint4 s, uint4 d, uint2 dp, uint32_t pr) {
    return (s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp.x ^ dp.y ^ pr) & 0x03030303u;
}

template <int M>
__global__ __launch_bounds__(1024) void k(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                          uint32_t* V, uint32_t ngroups, uint32_t* sink) {
    extern __shared__ uint4 smem[];
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t nfull = ngroups / nthreads * nthreads;
    uint32_t acc = 0;
    if constexpr (M <= 1) {
        for (uint32_t g = tid; g < nfull; g += nthreads) {
            const uint4 s = ldnt(S + g), d = ldnt(D + g);
            const uint2 dp = ldnt(DP + g);
            const uint32_t pr = PR[g];
            const uint32_t v = mix(s, d, dp, pr);
            if constexpr (M == 0) __builtin_nontemporal_store(v, V + g);
            else acc ^= v;
        }
    } else {
        // group index g of this lane; the wave's groups are g0 .. g0 + 63
        constexpr uint32_t kBuf = (M == 2) ? 1u : 2u;
        constexpr uint32_t kGpw = (M == 5) ? 32u : 64u;        // groups of 4 packets per wave-step
        constexpr uint32_t kSlot = kGpw * 44u;                  // src 16, dst 16, dport 8, proto 4 per group
        uint8_t* base = reinterpret_cast<uint8_t*>(smem) + wave * kBuf * kSlot;
        const uint32_t wspan = nthreads / 64u * kGpw;           // groups per grid-step over all waves
        const uint32_t wfirst = (blockIdx.x * (blockDim.x / 64u) + wave) * kGpw;
        auto issue = [&](uint32_t w0, uint32_t b) {
            uint8_t* sl = base + b * kSlot;
            const uint32_t gi = w0 + (lane % kGpw);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(S + gi), (lds_t)sl, 16, 0, 2);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(D + gi), (lds_t)(sl + 16u * kGpw), 16, 0, 2);
            // dport: 8 B per group = kGpw * 8 B; proto 4 B per group: 16-B lanes
            const uint32_t dq = min(lane, kGpw / 2u - 1u), pq = min(lane, kGpw / 4u - 1u);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(reinterpret_cast<const uint4*>(DP + w0) + dq),
                                             (lds_t)(sl + 32u * kGpw), 16, 0, 2);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(reinterpret_cast<const uint4*>(PR + w0) + pq),
                                             (lds_t)(sl + 40u * kGpw), 16, 0, 0);
        };
        auto use = [&](uint32_t w0, uint32_t b) {
            const uint8_t* sl = base + b * kSlot;
            const uint32_t j = lane % kGpw;
            const uint4 s = *reinterpret_cast<const uint4*>(sl + 16u * j);
            const uint4 d = *reinterpret_cast<const uint4*>(sl + 16u * kGpw + 16u * j);
            const uint2 dp = *reinterpret_cast<const uint2*>(sl + 32u * kGpw + 8u * j);
            const uint32_t pr = *reinterpret_cast<const uint32_t*>(sl + 40u * kGpw + 4u * j);
            const uint32_t v = mix(s, d, dp, pr);
            if (lane < kGpw) {
                if constexpr (M != 4) __builtin_nontemporal_store(v, V + w0 + j);
                else acc ^= v;
            }
        };
        const uint32_t wfull = nfull / wspan * wspan;
        if constexpr (M == 2) {
            for (uint32_t w0 = wfirst; w0 < wfull; w0 += wspan) {
                issue(w0, 0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                use(w0, 0);
            }
        } else {
            uint32_t w0 = wfirst, b = 0;
            if (w0 < wfull) issue(w0, 0);
            while (w0 < wfull) {
                const uint32_t nx = w0 + wspan;
                if (nx < wfull) {
                    issue(nx, b ^ 1u);
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // this step's 4 DMAs landed
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                use(w0, b);
                w0 = nx;
                b ^= 1u;
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// splitmix64 bytes: the stream over data like the benchmark's (a memset
// pattern toggles no bits and streams faster)
__global__ void fill_rand(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const bool rnd = argc > 1 && argv[1][0] == 'r';
    const uint64_t N = 1ull << 28;                 // packets
    const uint32_t G = uint32_t(N / 4);            // 4-packet groups
    uint4 *src, *dst;
    uint2* dp;
    uint32_t *pr, *v, *sink;
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, N * 4)); CK(hipMemset(dst, 2, N * 4)); CK(hipMemset(dp, 3, N * 2));
    CK(hipMemset(pr, 1, N)); CK(hipMemset(v, 0, N));
    if (rnd) {
        fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(src), N * 4 / 8, 1);
        fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dst), N * 4 / 8, 2);
        fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dp), N * 2 / 8, 3);
        fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(pr), N / 8, 4);
        CK(hipDeviceSynchronize());
        printf("random data\n");
    }
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](auto kern, int m, size_t lds, double bytes_per_pkt) -> int {
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        for (int rep = 0; rep < 3; ++rep) {
            for (int i = 0; i < 5; ++i) kern<<<ncu, 1024, lds>>>(src, dst, dp, pr, v, G, sink);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) kern<<<ncu, 1024, lds>>>(src, dst, dp, pr, v, G, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 10;
            printf("variant %d: %.4f ms %.1f GB/s\n", m, ms, bytes_per_pkt * N / ms / 1e6);
        }
        return 0;
    };
    // warm the clocks
    for (int i = 0; i < 200; ++i) k<0><<<ncu, 1024>>>(src, dst, (const uint2*)dp, pr, v, G, sink);
    CK(hipDeviceSynchronize());
    if (run(k<0>, 0, 0, 12.0)) return 1;
    if (run(k<1>, 1, 0, 11.0)) return 1;
    if (run(k<2>, 2, 16 * 64 * 44, 12.0)) return 1;
    if (run(k<3>, 3, 16 * 2 * 64 * 44, 12.0)) return 1;
    if (run(k<4>, 4, 16 * 2 * 64 * 44, 11.0)) return 1;
    if (run(k<5>, 5, 16 * 2 * 32 * 44, 12.0)) return 1;
    if (run(k<0>, 0, 0, 12.0)) return 1;
    return 0;
}
