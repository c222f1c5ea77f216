// Verdict-store shapes of the classify stream (round 5).  tools/stream_ring
// showed the LDS-DMA read stream at 6.8 TB/s of reads alone but 6.1 TB/s
// total once the 1 B/packet verdict stores are added -- the same as the
// register stream.  So: what do the stores cost, and does a wider store
// shape cost less?  Register loads as classify4_cls (16-B src / dst nt, 8-B
// dport nt, 4-B proto), one 1024-thread workgroup per CU, 256 Mi packets:
//   S4     the kernel's shape: 4 packets per lane per step, one 4-B nt store
//   RO     no store (read-only; an opaque run-time flag keeps the loads)
//   S16L   waves take 1024-packet chunks (4 sub-steps of 256); each sub-step's
//          verdict bytes go to the wave's 1 KiB LDS buffer and the chunk is
//          stored with one 16-B store per lane (1 KiB per instruction)
//   S16L-d the same with default-policy (not nt) stores
//   S4C    waves take 1024-packet chunks, 4-B stores (the chunk order alone)
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream_wshape.bin tools/stream_wshape.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#pragma clang diagnostic ignored "-Wint-to-pointer-cast"

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
__device__ __forceinline__ uint32_t mix(uint4 s, uint4 d, uint2 dp, uint32_t pr) {
    return (s.x ^ s.y ^ s.z ^ s.w ^ d.x ^ d.y ^ d.z ^ d.w ^ dp.x ^ dp.y ^ pr) & 0x03030303u;
}

// S4 / RO: grid-stride over 4-packet groups (store = 0: only when m == magic,
// which the host never makes true)
template <int kStore>   // 1: every group; 0: none; -4 / -16: one group in 4 / 16 (a quarter / sixteenth of the bytes)
__global__ __launch_bounds__(1024) void s4_kernel(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                                  uint32_t* V, uint32_t ngroups, uint32_t magic) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t nfull = ngroups / nthreads * nthreads;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nfull; g += nthreads) {
        const uint4 s = ldnt(S + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint4 d = ldnt(D + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint2 dp = ldnt(DP + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t pr = PR[g];
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t m = mix(s, d, dp, pr);
        // -4 / -16: sparse lanes (partial lines); -104 / -116: whole wave
        // instructions of one wave step in 4 / 16 (full lines, a quarter /
        // sixteenth of the bytes)
        const bool st = kStore == 1 ? true : kStore == 0 ? false
                        : kStore > -100 ? (g & uint32_t(-kStore - 1)) == 0u
                                        : ((g >> 6) & uint32_t(-kStore - 101)) == 0u;
        if (st || m == magic) __builtin_nontemporal_store(m, V + g);
    }
}

// S4 with the verdict stored by a buffer store of cache policy AUX (gfx950
// CPol bits: sc0 = 1, nt = 2, sc1 = 16)
template <int AUX>
__global__ __launch_bounds__(1024) void s4b_kernel(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                                   uint32_t* V, uint32_t ngroups) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(V, 0, 0x7FFFFFFF, 0x00020000);
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t nfull = ngroups / nthreads * nthreads;
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nfull; g += nthreads) {
        const uint4 s = ldnt(S + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint4 d = ldnt(D + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint2 dp = ldnt(DP + g);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t pr = PR[g];
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b32(mix(s, d, dp, pr), rs, 4u * g, 0, AUX);
    }
}

// chunked: wave w of the grid takes 1024-packet chunks w, w + nwaves, ...
// kMode 0: 4-B stores per sub-step; 1: LDS-staged 16-B nt store per chunk;
// 2: LDS-staged 16-B default-policy store
template <int kMode>
__global__ __launch_bounds__(1024) void chunk_kernel(const uint4* S, const uint4* D, const uint2* DP,
                                                     const uint32_t* PR, uint32_t* V, uint32_t nchunks) {
    __shared__ uint32_t buf[16][256];                 // 1 KiB per wave
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t c = blockIdx.x * (blockDim.x >> 6) + wv; c < nchunks; c += nwaves) {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t g = c * 256u + j * 64u + lane;    // 4-packet group
            const uint4 s = ldnt(S + g);
            __builtin_amdgcn_sched_barrier(0);
            const uint4 d = ldnt(D + g);
            __builtin_amdgcn_sched_barrier(0);
            const uint2 dp = ldnt(DP + g);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t pr = PR[g];
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t m = mix(s, d, dp, pr);
            if constexpr (kMode == 0) __builtin_nontemporal_store(m, V + g);
            else buf[wv][j * 64u + lane] = m;
        }
        if constexpr (kMode != 0) {
            // the chunk's 1 KiB of verdicts: lane l stores words 4l .. 4l + 3
            const v4u x = *reinterpret_cast<const v4u*>(&buf[wv][4u * lane]);
            v4u* o = reinterpret_cast<v4u*>(V + c * 256u) + lane;
            if constexpr (kMode == 1) __builtin_nontemporal_store(x, o);
            else *o = x;
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

__global__ void check(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR, const uint32_t* V,
                      uint32_t ngroups, uint32_t* bad) {
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += gridDim.x * blockDim.x)
        if (V[g] != mix(S[g], D[g], DP[g], PR[g])) atomicAdd(bad, 1u);
}

int main() {
    const uint64_t N = 1ull << 28;
    const uint32_t G = uint32_t(N / 4);
    uint4 *src, *dst;
    uint2* dp;
    uint32_t *pr, *v, *bad;
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N)); CK(hipMalloc(&bad, 4));
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(src), N * 4 / 8, 1);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dst), N * 4 / 8, 2);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dp), N * 2 / 8, 3);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(pr), N / 8, 4);
    CK(hipDeviceSynchronize());
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double bytes, bool chk, auto launch) -> int {
        for (int rep = 0; rep < 3; ++rep) {
            for (int i = 0; i < 5; ++i) launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int i = 0; i < 10; ++i) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 10;
            printf("%-10s %.4f ms  %.2f TB/s (%.0f B/packet)\n", name, ms, bytes / ms / 1e9, bytes / double(N));
        }
        if (chk) {
            CK(hipMemset(v, 0, N));
            CK(hipMemset(bad, 0, 4));
            launch();
            check<<<1024, 256>>>(src, dst, dp, pr, v, G, bad);
            uint32_t h = 0;
            CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
            printf("%-10s check: %u wrong groups\n", name, h);
        }
        fflush(stdout);
        return 0;
    };
    for (int i = 0; i < 200; ++i) s4_kernel<1><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0);
    CK(hipDeviceSynchronize());
    const double b12 = 12.0 * double(N), b11 = 11.0 * double(N);
    const uint32_t nch = uint32_t(N / 1024);
    for (int round = 0; round < 2; ++round) {
        timed("S4", b12, true, [&] { s4_kernel<1><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0); });
        timed("RO", b11, false, [&] { s4_kernel<0><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0xFFFFFFFFu); });
        timed("S4/4", b11 + double(N) / 4, false, [&] { s4_kernel<-4><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0xFFFFFFFFu); });
        timed("S4/16", b11 + double(N) / 16, false, [&] { s4_kernel<-16><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0xFFFFFFFFu); });
        timed("W4 full", b11 + double(N) / 4, false, [&] { s4_kernel<-104><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0xFFFFFFFFu); });
        timed("W16 full", b11 + double(N) / 16, false, [&] { s4_kernel<-116><<<ncu, 1024>>>(src, dst, dp, pr, v, G, 0xFFFFFFFFu); });
    }
    return 0;
}
