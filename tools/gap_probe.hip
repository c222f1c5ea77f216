// Where does classify4_cls lose 4-11 % against the plain packet stream when
// its evaluation is compiled out?  The stream kernel of
// the floor (src, dst, dport nt, proto cached, verdict nt; 4 packets per lane,
// one 1024-thread workgroup per CU) with one ingredient of the classify
// kernel added per variant, over 256 Mi packets of random data:
//   0  the stream kernel as bench.py's floor (no LDS)
//   1  + 125 KB dynamic LDS (the config-3 image's allocation)
//   2  + a 1 KiB by-value kernel argument read by every wave (Cls4Dev x 2)
//   3  + 68 live VGPRs per lane (the classify kernel's register count)
//   4  + the verdict packing of the classify loop (4 bytes, SWAR protocol test)
//   5  + clearing 80 KB of a global buffer at the start (the rule counters)
//      and a workgroup barrier at the end
//   6  all of 1-5
// build: hipcc -O3 --offload-arch=gfx950 -o tools/gap_probe.bin tools/gap_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

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

struct Big {                        // a kernel argument the size of two Cls4Dev
    uint32_t w[256];
};

// extra adds per step on R live registers (pacing), R * K adds
template <int R, int K>
__global__ __launch_bounds__(1024) void kp(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                           uint32_t* V, uint32_t nsteps, unsigned long long*, uint32_t, Big) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t r[R];
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = tid * uint32_t(i + 1);
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        const uint4 s = ldnt(S + g);
        const uint4 d = ldnt(D + g);
        const uint2 dp = ldnt(DP + g);
        const uint32_t pr = PR[g];
        const uint32_t v = (s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp.x ^ dp.y ^ pr) & 0x03030303u;
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int i = 0; i < R; ++i) r[i] = r[i] * 3u + v;
        }
        __builtin_nontemporal_store(v, V + g);
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) x ^= r[i];
    if (x == 0x9E3779B9u) V[0] = x;
}

template <bool kBigArg, bool kRegs, bool kPack, bool kZero>
__global__ __launch_bounds__(1024) void k(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                          uint32_t* V, uint32_t nsteps, unsigned long long* zero, uint32_t nzero,
                                          Big big) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if constexpr (kZero)
        for (uint32_t i = tid; i < nzero; i += nthreads) zero[i] = 0ull;
    uint32_t salt = 0;
    if constexpr (kBigArg) salt = big.w[threadIdx.x & 255u] & 0x01010101u;
    uint32_t r[48];
    if constexpr (kRegs) {
#pragma unroll
        for (int i = 0; i < 48; ++i) r[i] = tid * uint32_t(i + 1);
    }
    for (uint32_t g = tid; g < nsteps; g += nthreads) {
        const uint4 s = ldnt(S + g);
        const uint4 d = ldnt(D + g);
        const uint2 dp = ldnt(DP + g);
        const uint32_t pr = PR[g];
        uint32_t v;
        if constexpr (kPack) {
            const uint32_t other = ((pr | ((pr & 0x7F7F7F7Fu) + 0x7D7D7D7Du)) & 0x80808080u) != 0u;
            const uint32_t b0 = (s.x ^ d.x ^ (dp.x & 0xFFFFu) ^ (pr & 0xFFu) ^ other) & 3u;
            const uint32_t b1 = (s.y ^ d.y ^ (dp.x >> 16) ^ ((pr >> 8) & 0xFFu) ^ other) & 3u;
            const uint32_t b2 = (s.z ^ d.z ^ (dp.y & 0xFFFFu) ^ ((pr >> 16) & 0xFFu) ^ other) & 3u;
            const uint32_t b3 = (s.w ^ d.w ^ (dp.y >> 16) ^ (pr >> 24) ^ other) & 3u;
            v = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
        } else {
            v = (s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp.x ^ dp.y ^ pr) & 0x03030303u;
        }
        if constexpr (kRegs) {
#pragma unroll
            for (int i = 0; i < 48; ++i) r[i] += v;
        }
        __builtin_nontemporal_store(v ^ salt, V + g);
    }
    if constexpr (kRegs) {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 48; ++i) x ^= r[i];
        if (x == 0x9E3779B9u) V[0] = x;
    }
    if constexpr (kZero) __syncthreads();
}

__global__ void fill_rand(uint64_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main() {
    const uint64_t N = 1ull << 28;
    const uint32_t G = uint32_t(N / 4);
    uint4 *src, *dst;
    uint2* dp;
    uint32_t *pr, *v;
    unsigned long long* zero;
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N)); CK(hipMalloc(&zero, 80 * 1024));
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(src), N * 4 / 8, 1);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dst), N * 4 / 8, 2);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dp), N * 2 / 8, 3);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(pr), N / 8, 4);
    CK(hipDeviceSynchronize());
    Big big;
    for (int i = 0; i < 256; ++i) big.w[i] = uint32_t(i) * 0x01000193u;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint32_t nz = 80 * 1024 / 8;
    auto run = [&](auto kern, const char* name, size_t lds) -> int {
        if (lds) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        for (int rep = 0; rep < 3; ++rep) {
            for (int i = 0; i < 3; ++i) kern<<<ncu, 1024, lds>>>(src, dst, dp, pr, v, G, zero, nz, big);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) kern<<<ncu, 1024, lds>>>(src, dst, dp, pr, v, G, zero, nz, big);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-34s %.4f ms\n", name, ms / 10);
        }
        return 0;
    };
    const size_t L = 128320;
    for (int i = 0; i < 100; ++i) k<false, false, false, false><<<ncu, 1024>>>(src, dst, dp, pr, v, G, zero, nz, big);
    CK(hipDeviceSynchronize());
    if (run(k<false, false, false, false>, "0 stream", 0)) return 1;
    if (run(k<false, false, false, false>, "1 + 125 KB LDS", L)) return 1;
    if (run(k<true, false, false, false>, "2 + 1 KiB kernel argument", 0)) return 1;
    if (run(k<false, true, false, false>, "3 + 68 VGPRs", 0)) return 1;
    if (run(k<false, false, true, false>, "4 + verdict packing", 0)) return 1;
    if (run(k<false, false, false, true>, "5 + counter clearing, barrier", 0)) return 1;
    if (run(k<true, true, true, true>, "6 all of 1-5", L)) return 1;
    if (run(k<false, false, false, false>, "0 stream", 0)) return 1;
    // pacing: R registers x K rounds of mad per step
    if (run(kp<8, 1>, "p 8 regs x 1", 0)) return 1;
    if (run(kp<8, 4>, "p 8 regs x 4", 0)) return 1;
    if (run(kp<8, 12>, "p 8 regs x 12", 0)) return 1;
    if (run(kp<48, 1>, "p 48 regs x 1", 0)) return 1;
    if (run(kp<48, 2>, "p 48 regs x 2", 0)) return 1;
    if (run(kp<48, 4>, "p 48 regs x 4", 0)) return 1;
    if (run(kp<96, 1>, "p 96 regs x 1", 0)) return 1;
    if (run(k<false, false, false, false>, "0 stream", 0)) return 1;
    return 0;
}
