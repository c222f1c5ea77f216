// The 16-byte layout's HBM stream (config 5: 16-B src and dst, u16 dport, u8
// proto read, u8 verdict written -- 36 B per packet) in several access shapes,
// timed alone (no lookups), on the classify kernel's grid (one 1024-thread
// workgroup per CU).  Which shape moves the 36 B fastest?
//   0  wave-contiguous addresses (lane l: packets base + 64k + l), dport /
//      proto / verdict one element per lane per instruction, all non-temporal
//      (the classify16 kernel today)
//   1  as 0, dport / proto cached loads
//   2  as 0, but dport (u64: 4 ports), proto (u32: 4) and verdict (u32: 4)
//      moved 4 consecutive packets per lane, transposed across the wave with
//      ds_bpermute
//   3  lane owns 4 consecutive packets: 16-B address loads at a 64-B lane
//      stride, cached; dport u64, proto u32, verdict u32 per lane
//   4  as 3 with non-temporal address loads
//   5  as 2, verdict one byte per lane (transpose the loads only)
//   6  as 0 with 2 workgroups per CU
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream16_sweep.bin tools/stream16_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
template <bool nt> __device__ __forceinline__ uint4 ld4(const uint4* p) {
    if constexpr (nt) { const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)); return make_uint4(v.x, v.y, v.z, v.w); }
    else return *p;
}
template <bool nt> __device__ __forceinline__ uint2 ld2(const uint2* p) {
    if constexpr (nt) { const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p)); return make_uint2(v.x, v.y); }
    else return *p;
}
template <bool nt, typename T> __device__ __forceinline__ T ld(const T* p) {
    if constexpr (nt) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ uint32_t perm(uint32_t lane, uint32_t v) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(lane * 4u), int(v)));
}
__device__ __forceinline__ uint32_t mix(const uint4& s, const uint4& d) { return s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w; }

template <int M>
__global__ __launch_bounds__(1024) void k(const uint4* S, const uint4* D, const uint16_t* DP, const uint8_t* PR,
                                          uint8_t* V, uint32_t n) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    if constexpr (M == 0 || M == 1 || M == 6) {
        constexpr bool ntp = M != 1;
        const uint32_t nsteps = n / 256u * 64u;
        for (uint32_t g = tid; g < nsteps; g += nthreads) {
            const uint32_t base = 4u * (g & ~63u) + (g & 63u);
            uint4 s[4], d[4];
            uint32_t dp[4], pr[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { s[q] = ld4<true>(S + base + 64u * q); d[q] = ld4<true>(D + base + 64u * q); }
#pragma unroll
            for (int q = 0; q < 4; ++q) { dp[q] = ld<ntp>(DP + base + 64u * q); pr[q] = ld<ntp>(PR + base + 64u * q); }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_nontemporal_store(uint8_t((mix(s[q], d[q]) ^ dp[q] ^ pr[q]) & 3u), V + base + 64u * q);
        }
    } else if constexpr (M == 2 || M == 5) {
        const uint32_t nsteps = n / 256u * 64u;
        for (uint32_t g = tid; g < nsteps; g += nthreads) {
            const uint32_t w = g & ~63u;                  // wave's first group: packets 4w .. 4w + 255
            const uint32_t base = 4u * w + lane;
            uint4 s[4], d[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { s[q] = ld4<true>(S + base + 64u * q); d[q] = ld4<true>(D + base + 64u * q); }
            // lane l holds dport / proto of packets 4w + 4l .. 4l + 3
            const uint2 dp4 = ld2<true>(reinterpret_cast<const uint2*>(DP) + w + lane);
            const uint32_t pr4 = ld<true>(reinterpret_cast<const uint32_t*>(PR) + w + lane);
            uint32_t v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // packet 64q + l lives in lane 16q + l/4, element l%4
                const uint32_t src = 16u * q + (lane >> 2), e = lane & 3u;
                const uint32_t wx = perm(src, dp4.x), wy = perm(src, dp4.y), p = perm(src, pr4);
                const uint32_t dw = (e & 2u) ? wy : wx;
                const uint32_t dport = (dw >> (16u * (e & 1u))) & 0xFFFFu, proto = (p >> (8u * e)) & 0xFFu;
                v[q] = (mix(s[q], d[q]) ^ dport ^ proto) & 3u;
            }
            if constexpr (M == 2) {
                // verdict of packet 4l + j: lane (4l + j) % 64, q = l / 16
                const uint32_t packed = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
                uint32_t out = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t x = perm((4u * lane + uint32_t(j)) & 63u, packed);
                    out |= ((x >> (8u * (lane >> 4))) & 0xFFu) << (8 * j);
                }
                __builtin_nontemporal_store(out, reinterpret_cast<uint32_t*>(V) + w + lane);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(uint8_t(v[q]), V + base + 64u * q);
            }
        }
    } else {
        constexpr bool nta = M == 4;
        const uint32_t nsteps = n / 4u;
        for (uint32_t g = tid; g < nsteps; g += nthreads) {
            uint4 s[4], d[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { s[q] = ld4<nta>(S + 4u * g + q); d[q] = ld4<nta>(D + 4u * g + q); }
            const uint2 dp4 = ld2<true>(reinterpret_cast<const uint2*>(DP) + g);
            const uint32_t pr4 = ld<true>(reinterpret_cast<const uint32_t*>(PR) + g);
            const uint32_t m = (mix(s[0], d[0]) & 3u) | ((mix(s[1], d[1]) & 3u) << 8) | ((mix(s[2], d[2]) & 3u) << 16) |
                               ((mix(s[3], d[3]) & 3u) << 24);
            __builtin_nontemporal_store((m ^ dp4.x ^ dp4.y ^ pr4) & 0x03030303u, reinterpret_cast<uint32_t*>(V) + g);
        }
    }
}

int main() {
    const uint64_t N = 1ull << 28;
    uint4 *src, *dst;
    uint16_t* dp;
    uint8_t *pr, *v;
    CK(hipMalloc(&src, N * 16)); CK(hipMalloc(&dst, N * 16)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N));
    CK(hipMemset(src, 1, N * 16)); CK(hipMemset(dst, 2, N * 16)); CK(hipMemset(dp, 3, N * 2));
    CK(hipMemset(pr, 1, N)); CK(hipMemset(v, 0, N));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](auto kern, int m, int grid) -> int {
        for (int rep = 0; rep < 3; ++rep) {
            for (int i = 0; i < 3; ++i) kern<<<grid, 1024>>>(src, dst, dp, pr, v, uint32_t(N));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) kern<<<grid, 1024>>>(src, dst, dp, pr, v, uint32_t(N));
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 10;
            printf("shape %d grid %d: %.4f ms %.1f GB/s\n", m, grid, ms, 36.0 * N / ms / 1e6);
        }
        return 0;
    };
    run(k<0>, 0, ncu); run(k<1>, 1, ncu); run(k<2>, 2, ncu); run(k<3>, 3, ncu);
    run(k<4>, 4, ncu); run(k<5>, 5, ncu); run(k<6>, 6, 2 * ncu);
    run(k<0>, 0, ncu); run(k<2>, 2, ncu);
    return 0;
}
