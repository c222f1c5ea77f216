// Which of the classify kernel's five streams want non-temporal accesses?
// stream_pp shape (one 4-packet group per lane per step, 32-bit offsets from
// uniform bases, no prefetch), every combination of nt per array.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/nt_sweep.bin tools/nt_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ const T* at(const T* base, uint32_t i) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + i * uint32_t(sizeof(T)));
}
template <bool nt> __device__ __forceinline__ uint4 ld4(const uint4* p) {
    if constexpr (nt) { const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)); return make_uint4(v.x, v.y, v.z, v.w); }
    else return *p;
}
template <bool nt> __device__ __forceinline__ uint2 ld2(const uint2* p) {
    if constexpr (nt) { const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p)); return make_uint2(v.x, v.y); }
    else return *p;
}
template <bool nt> __device__ __forceinline__ uint32_t ld1(const uint32_t* p) {
    if constexpr (nt) return __builtin_nontemporal_load(p);
    else return __builtin_amdgcn_readfirstlane(0) + *p;
}
template <int M>
__global__ __launch_bounds__(1024) void k(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                          uint32_t* V, uint32_t nsteps) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nsteps; g += nthreads) {
        const uint4 s = ld4<(M & 1) != 0>(at(S, g)), d = ld4<(M & 2) != 0>(at(D, g));
        const uint2 dp = ld2<(M & 4) != 0>(at(DP, g));
        const uint32_t pr = ld1<(M & 8) != 0>(at(PR, g));
        const uint32_t v = (s.x ^ d.x ^ s.y ^ d.y ^ s.z ^ d.z ^ s.w ^ d.w ^ dp.x ^ dp.y ^ pr) & 0x03030303u;
        uint32_t* o = const_cast<uint32_t*>(at(const_cast<const uint32_t*>(V), g));
        if constexpr ((M & 16) != 0) __builtin_nontemporal_store(v, o);
        else *o = v;
    }
}

int main() {
    const uint64_t N = 1ull << 28;
    uint32_t *src, *dst, *pr, *v;
    uint16_t* dp;
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N));
    CK(hipMemset(src, 1, N * 4)); CK(hipMemset(dst, 2, N * 4)); CK(hipMemset(dp, 3, N * 2));
    CK(hipMemset(pr, 1, N)); CK(hipMemset(v, 0, N));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](auto kern, int m, int grid) -> int {
        for (int rep = 0; rep < 2; ++rep) {
            for (int i = 0; i < 3; ++i) kern<<<grid, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, uint32_t(N / 4));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) kern<<<grid, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, uint32_t(N / 4));
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 10;
            printf("nt src %d dst %d dport %d proto %d store %d grid %d: %.4f ms %.1f GB/s\n", m & 1, (m >> 1) & 1,
                   (m >> 2) & 1, (m >> 3) & 1, (m >> 4) & 1, grid, ms, 12.0 * N / ms / 1e6);
        }
        return 0;
    };
#define R(M) run(k<M>, M, 256);
    R(0) R(1) R(2) R(3) R(4) R(5) R(6) R(7) R(8) R(9) R(10) R(11) R(12) R(13) R(14) R(15)
    R(16) R(17) R(18) R(19) R(20) R(21) R(22) R(23) R(24) R(25) R(26) R(27) R(28) R(29) R(30) R(31)
    return 0;
}
