// The 16-byte layout's stream (config 5: 16-B src and dst, u16 dport, u8
// proto read, u8 verdict written -- 36 B per packet) by shape of the three
// narrow fields (round 5).  src and dst are read wave-
// contiguous as classify16_cls does (lane l of a 256-packet wave step owns
// packets base + 64k + l, one 1 KiB 16-B load per wave-instruction).  The
// narrow fields:
//   A    as classify16_cls: one u16 / u8 load and one u8 store per packet
//        (128 / 64 / 64 B per wave-instruction)
//   A-RO A without the verdict store (read ceiling; opaque run-time flag)
//   AV   A's loads; the lane's four verdict bytes are moved with ds_bpermute
//        so that lane m stores packets base + 4m .. 4m + 3 as one 4-B word
//        (256 B per instruction)
//   X    dport (8 B), proto (4 B) and verdict (4 B) per lane in packet
//        order -- lane m owns packets base + 4m .. 4m + 3 -- moved to the
//        wave-contiguous owners with ds_bpermute (16 per lane per step)
//   T    the ideal if the layout is the engine's: the narrow fields stored
//        transposed per 256-packet block (element 4l + k is packet 64k + l),
//        8-B / 4-B / 4-B per lane, no exchange
// 256 Mi packets of random data, one 1024-thread workgroup per CU; A, AV and
// X checked against each other (same verdict bytes).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream16_shape.bin tools/stream16_shape.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 ldnt(const uint4* p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t mix(const uint4& s, const uint4& d, uint32_t dp, uint32_t pr) {
    return (s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp ^ pr) & 3u;
}
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src_lane << 2), int(v)));
}

template <int M>
__global__ __launch_bounds__(1024) void k16(const uint4* S, const uint4* D, const uint16_t* DP, const uint8_t* PR,
                                            uint8_t* V, uint32_t n, uint32_t magic) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t nsteps = n / 256u * 64u;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nsteps; g += nthreads) {
        const uint32_t base = 4u * (g & ~63u);               // the wave step's first packet
        uint4 s[4], d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[k] = ldnt(S + base + 64u * k + lane);
            d[k] = ldnt(D + base + 64u * k + lane);
        }
        uint32_t dp[4], pr[4], v[4];
        if constexpr (M <= 2) {                               // A, A-RO, AV
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                dp[k] = __builtin_nontemporal_load(DP + base + 64u * k + lane);
                pr[k] = __builtin_nontemporal_load(PR + base + 64u * k + lane);
            }
        } else if constexpr (M == 3) {                        // X: packet order, exchanged
            const v2u dw = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(DP + base) + lane);
            const uint32_t pw = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(PR + base) + lane);
            // packet base + 64k + lane is element (lane & 3) of lane 16k + lane / 4
            const uint32_t sh = 8u * (lane & 3u);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t from = 16u * k + (lane >> 2);
                const uint32_t x = bperm(dw.x, from), y = bperm(dw.y, from), z = bperm(pw, from);
                const uint32_t w = (lane & 2u) ? y : x;
                dp[k] = (lane & 1u) ? (w >> 16) : (w & 0xFFFFu);
                pr[k] = (z >> sh) & 0xFFu;
            }
        } else {                                              // T: transposed per block
            const v2u dw = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(DP + base) + lane);
            const uint32_t pw = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(PR + base) + lane);
            dp[0] = dw.x & 0xFFFFu; dp[1] = dw.x >> 16; dp[2] = dw.y & 0xFFFFu; dp[3] = dw.y >> 16;
#pragma unroll
            for (int k = 0; k < 4; ++k) pr[k] = (pw >> (8 * k)) & 0xFFu;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = mix(s[k], d[k], dp[k], pr[k]);
        if constexpr (M == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(uint8_t(v[k]), V + base + 64u * k + lane);
        } else if constexpr (M == 1) {
            if ((v[0] ^ v[1] ^ v[2] ^ v[3]) == magic) V[base + lane] = 1;   // never (magic > 3)
        } else if constexpr (M == 2 || M == 3) {
            // lane m stores packets base + 4m + j: packet q = 4m + j is byte
            // k = q / 64 of lane (q & 63)'s packed word
            const uint32_t packed = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
            const uint32_t kb = 8u * (lane >> 4);
            uint32_t out = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) out |= ((bperm(packed, (4u * lane + j) & 63u) >> kb) & 0xFFu) << (8 * j);
            __builtin_nontemporal_store(out, reinterpret_cast<uint32_t*>(V + base) + lane);
        } else {
            const uint32_t packed = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
            __builtin_nontemporal_store(packed, reinterpret_cast<uint32_t*>(V + base) + lane);
        }
    }
}

__global__ void fill_rand(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ void diff(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* bad) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1u);
}

int main() {
    const uint64_t N = 1ull << 28;
    uint4 *src, *dst;
    uint16_t* dp;
    uint8_t *pr, *v, *v0;
    uint32_t* bad;
    CK(hipMalloc(&src, N * 16)); CK(hipMalloc(&dst, N * 16)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N)); CK(hipMalloc(&v0, N)); CK(hipMalloc(&bad, 4));
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(src), N * 2, 1);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dst), N * 2, 2);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dp), N / 4, 3);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(pr), N / 8, 4);
    CK(hipDeviceSynchronize());
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = 36.0 * double(N);
    auto timed = [&](const char* name, auto launch) -> int {
        for (int rep = 0; rep < 3; ++rep) {
            for (int i = 0; i < 3; ++i) launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 8; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 8;
            printf("%-6s %.4f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
        }
        fflush(stdout);
        return 0;
    };
    const uint32_t n = uint32_t(N);
    for (int i = 0; i < 40; ++i) k16<0><<<ncu, 1024>>>(src, dst, dp, pr, v0, n, 7);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 2; ++round) {
        timed("A", [&] { k16<0><<<ncu, 1024>>>(src, dst, dp, pr, v0, n, 7); });
        timed("A-RO", [&] { k16<1><<<ncu, 1024>>>(src, dst, dp, pr, v, n, 7); });
        timed("AV", [&] { k16<2><<<ncu, 1024>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0) {
            CK(hipMemset(bad, 0, 4));
            diff<<<1024, 256>>>(v, v0, N, bad);
            uint32_t h = 0;
            CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
            printf("AV check against A: %u bytes differ\n", h);
        }
        timed("X", [&] { k16<3><<<ncu, 1024>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0) {
            CK(hipMemset(bad, 0, 4));
            diff<<<1024, 256>>>(v, v0, N, bad);
            uint32_t h = 0;
            CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
            printf("X check against A: %u bytes differ\n", h);
        }
        timed("T", [&] { k16<4><<<ncu, 1024>>>(src, dst, dp, pr, v, n, 7); });
    }
    return 0;
}
