// Do the classify kernels' streams lose bandwidth because their arrays sit at
// power-of-two distances (the same HBM channel / bank for the same index)?
// The 16-byte stream (config 5 shape 0 of stream16_sweep) and the IPv4 stream
// (classify4 shape: 16-B src/dst, 8-B dport, 4-B proto and verdict per lane)
// over one allocation with each array starting `skew` bytes after a 1 GiB
// boundary multiple: skew 0 (aligned like separate hipMallocs) vs odd skews.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream_offset_sweep.bin tools/stream_offset_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld4(const uint4* p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)); return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld2(const uint2* p) {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p)); return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t mix(const uint4& s, const uint4& d) { return s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w; }

__global__ __launch_bounds__(1024) void s16(const uint4* S, const uint4* D, const uint16_t* DP, const uint8_t* PR,
                                            uint8_t* V, uint32_t n) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t nsteps = n / 256u * 64u;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nsteps; g += nthreads) {
        const uint32_t base = 4u * (g & ~63u) + (g & 63u);
        uint4 s[4], d[4];
        uint32_t dp[4], pr[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { s[q] = ld4(S + base + 64u * q); d[q] = ld4(D + base + 64u * q); }
#pragma unroll
        for (int q = 0; q < 4; ++q) { dp[q] = __builtin_nontemporal_load(DP + base + 64u * q); pr[q] = __builtin_nontemporal_load(PR + base + 64u * q); }
#pragma unroll
        for (int q = 0; q < 4; ++q) __builtin_nontemporal_store(uint8_t((mix(s[q], d[q]) ^ dp[q] ^ pr[q]) & 3u), V + base + 64u * q);
    }
}

__global__ __launch_bounds__(1024) void s4(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                           uint32_t* V, uint32_t nsteps) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nsteps; g += nthreads) {
        const uint4 s = ld4(S + g), d = ld4(D + g);
        const uint2 dp = ld2(DP + g);
        const uint32_t pr = PR[g];
        __builtin_nontemporal_store((mix(s, d) ^ dp.x ^ dp.y ^ pr) & 0x03030303u, V + g);
    }
}

int main() {
    const uint64_t N = 1ull << 28;
    const uint64_t GB = 1ull << 30;
    uint8_t* pool;
    const uint64_t bytes = 40 * GB;
    CK(hipMalloc(&pool, bytes));
    CK(hipMemset(pool, 1, bytes));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint64_t skews[] = {0, 4096 + 256, 65536 + 1024, 3 * 1024 * 1024 + 4096 + 512, 256};
    for (uint64_t sk : skews) {
        for (int v16 = 0; v16 < 2; ++v16) {
            // arrays at k * 8 GiB (v16) / k * 2 GiB (v4) + k * skew
            const uint64_t stride = v16 ? 8 * GB : 2 * GB;
            uint8_t* a[5];
            for (int k = 0; k < 5; ++k) a[k] = pool + k * stride + k * sk;
            auto launch = [&]() {
                if (v16) s16<<<ncu, 1024>>>((const uint4*)a[0], (const uint4*)a[1], (const uint16_t*)a[2], a[3], a[4], uint32_t(N));
                else s4<<<ncu, 1024>>>((const uint4*)a[0], (const uint4*)a[1], (const uint2*)a[2], (const uint32_t*)a[3], (uint32_t*)a[4], uint32_t(N / 4));
            };
            for (int rep = 0; rep < 2; ++rep) {
                for (int i = 0; i < 3; ++i) launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                for (int i = 0; i < 10; ++i) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= 10;
                const double b = (v16 ? 36.0 : 12.0) * N;
                printf("%s skew %llu: %.4f ms %.1f GB/s\n", v16 ? "v16" : "v4 ", (unsigned long long)sk, ms, b / ms / 1e6);
            }
        }
    }
    return 0;
}
