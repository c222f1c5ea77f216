// Streaming-skeleton microbenchmark for the classify kernel's HBM pattern:
// read src u32, dst u32, dport u16, proto u8 per packet, write one verdict
// byte.  No classification -- only the access pattern, to find the achievable
// floor on MI355X.  Build: hipcc -O3 --offload-arch=gfx950 -o stream_bench stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld(const uint4* p, bool nt) {
    if (!nt) return *p;
    v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld(const uint2* p, bool nt) {
    if (!nt) return *p;
    v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t ld(const uint32_t* p, bool nt) {
    return nt ? __builtin_nontemporal_load(p) : *p;
}
__device__ __forceinline__ void st(uint4 v, uint4* p) {
    v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(p));
}

// A: 4 packets per lane per step (16 B src/dst, 8 B dport, 4 B proto, 4 B store)
// kG groups per lane per step, group k of lane at index (g*kG... ) coalesced per instruction:
// step base b = (blk*steps ...) -- grid-stride over 4-packet groups, kG groups at stride nthreads.
template <int kG, bool kNtL, bool kNtS>
__global__ __launch_bounds__(1024) void stream4(const uint4* S, const uint4* D, const uint2* DP,
                                                const uint32_t* PR, uint32_t* V, uint64_t ngroups,
                                                uint32_t salt) {
    const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (uint64_t g = tid; g < ngroups; g += nthreads * kG) {
        uint4 s[kG], d[kG];
        uint2 dp[kG];
        uint32_t pr[kG];
#pragma unroll
        for (int k = 0; k < kG; ++k) {
            const uint64_t i = g + uint64_t(k) * nthreads;
            if (i < ngroups) {
                s[k] = ld(S + i, kNtL); d[k] = ld(D + i, kNtL); dp[k] = ld(DP + i, kNtL); pr[k] = ld(PR + i, kNtL);
            } else {
                s[k] = make_uint4(0, 0, 0, 0); d[k] = s[k]; dp[k] = make_uint2(0, 0); pr[k] = 0;
            }
        }
#pragma unroll
        for (int k = 0; k < kG; ++k) {
            const uint64_t i = g + uint64_t(k) * nthreads;
            uint32_t v = (s[k].x ^ d[k].x ^ s[k].y ^ d[k].y ^ s[k].z ^ d[k].z ^ s[k].w ^ d[k].w ^
                          dp[k].x ^ dp[k].y ^ pr[k] ^ salt) & 0x03030303u;
            if (i < ngroups) {
                if (kNtS) __builtin_nontemporal_store(v, V + i);
                else V[i] = v;
            }
        }
    }
}

// B: 16 packets per lane: src/dst as 4 coalesced 16-B loads each (lane-strided
// sub-blocks of a 1024-packet wave tile), dport 2 x 16 B, proto 16 B, verdict 16 B.
// Wave tile = 1024 packets: src words [t*1024 .. +1024): load j (0..3): lane l reads
// uint4 at (t*256 + j*64 + l) -> packets 4*(j*64+l)..+3.  dport: uint4 holds 8 ports:
// load j (0..1) lane l reads uint4 at t*128 + j*64 + l -> packets 8*(j*64+l)..+7.
// proto: uint4 at t*64 + l -> packets 16*l..+15.  Mismatched ownership is fine for a
// streaming floor (the classifier would reshuffle through LDS / DPP).
template <bool kNtL, bool kNtS>
__global__ __launch_bounds__(1024) void stream16(const uint4* S, const uint4* D, const uint4* DP,
                                                 const uint4* PR, uint4* V, uint64_t ntiles,
                                                 uint32_t salt) {
    const uint64_t nwaves = uint64_t(gridDim.x) * (blockDim.x / 64);
    const uint64_t w = uint64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t l = threadIdx.x & 63;
    for (uint64_t t = w; t < ntiles; t += nwaves) {
        uint4 s[4], d[4], dp[2], pr;
#pragma unroll
        for (int j = 0; j < 4; ++j) { s[j] = ld(S + t * 256 + j * 64 + l, kNtL); d[j] = ld(D + t * 256 + j * 64 + l, kNtL); }
#pragma unroll
        for (int j = 0; j < 2; ++j) dp[j] = ld(DP + t * 128 + j * 64 + l, kNtL);
        pr = ld(PR + t * 64 + l, kNtL);
        uint32_t x = salt;
#pragma unroll
        for (int j = 0; j < 4; ++j) x ^= s[j].x ^ s[j].y ^ s[j].z ^ s[j].w ^ d[j].x ^ d[j].y ^ d[j].z ^ d[j].w;
        x ^= dp[0].x ^ dp[0].y ^ dp[0].z ^ dp[0].w ^ dp[1].x ^ dp[1].y ^ dp[1].z ^ dp[1].w;
        uint4 v = make_uint4((x ^ pr.x) & 0x03030303u, (x ^ pr.y) & 0x03030303u, (x ^ pr.z) & 0x03030303u,
                             (x ^ pr.w) & 0x03030303u);
        if (kNtS) st(v, V + t * 64 + l);
        else V[t * 64 + l] = v;
    }
}

// D: the classify kernel's skeleton: 32-bit byte offsets from uniform bases
// (saddr loads), two buffers in turn (next step's loads in flight), nt loads
// and stores.  kPf = false: load and use in the same iteration.
template <typename T>
__device__ __forceinline__ const T* at(const T* base, uint32_t i) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + i * uint32_t(sizeof(T)));
}
struct Buf { uint4 s, d; uint2 dp; uint32_t pr; };
template <bool kPf>
__global__ __launch_bounds__(1024) void stream_pp(const uint4* S, const uint4* D, const uint2* DP,
                                                  const uint32_t* PR, uint32_t* V, uint32_t nsteps,
                                                  uint32_t salt) {
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    auto load = [&](Buf& b, uint32_t g) {
        if (g < nsteps) { b.s = ld(at(S, g), true); b.d = ld(at(D, g), true); b.dp = ld(at(DP, g), true); b.pr = ld(at(PR, g), true); }
    };
    auto step = [&](const Buf& b, uint32_t g) {
        const uint32_t v = (b.s.x ^ b.d.x ^ b.s.y ^ b.d.y ^ b.s.z ^ b.d.z ^ b.s.w ^ b.d.w ^ b.dp.x ^ b.dp.y ^ b.pr ^ salt) & 0x03030303u;
        __builtin_nontemporal_store(v, const_cast<uint32_t*>(at(const_cast<const uint32_t*>(V), g)));
    };
    if constexpr (kPf) {
        Buf a, b;
        uint32_t g = tid;
        load(a, g);
        while (g < nsteps) {
            load(b, g + nthreads);
            step(a, g);
            g += nthreads;
            if (g >= nsteps) break;
            load(a, g + nthreads);
            step(b, g);
            g += nthreads;
        }
    } else {
        for (uint32_t g = tid; g < nsteps; g += nthreads) { Buf a; load(a, g); step(a, g); }
    }
}

// C: pure read 11 B/pkt (no store) and pure float4 copy for reference
__global__ __launch_bounds__(1024) void copy16(const uint4* a, uint4* b, uint64_t n) {
    const uint64_t nt = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += nt) b[i] = a[i];
}

int main(int argc, char** argv) {
    const uint64_t N = 1ull << 28;  // packets
    uint32_t *src, *dst, *pr, *v;
    uint16_t* dp;
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N));
    CK(hipMemset(src, 1, N * 4)); CK(hipMemset(dst, 2, N * 4)); CK(hipMemset(dp, 3, N * 2));
    CK(hipMemset(pr, 1, N)); CK(hipMemset(v, 0, N));
    uint4 *ca, *cb;
    const uint64_t CN = 1ull << 30;  // bytes copied
    CK(hipMalloc(&ca, CN)); CK(hipMalloc(&cb, CN)); CK(hipMemset(ca, 0, CN));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    int ncu = 256;
    auto timeit = [&](const char* name, auto fn, double bytes) {
        for (int i = 0; i < 3; ++i) fn();
        CK(hipDeviceSynchronize());
        const int it = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; ++i) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-44s %8.4f ms  %7.1f GB/s  %6.1f Gpps\n", name, ms, bytes / ms / 1e6, N / ms / 1e6);
        fflush(stdout);
    };
    const double B12 = 12.0 * N;
    timeit("copy16 1 GiB (read+write bytes)", [&] { copy16<<<ncu * 8, 1024>>>(ca, cb, CN / 16); }, 2.0 * CN);
#define RUN4(G, NL, NS, GRID)                                                                              \
    {                                                                                                      \
        char nm[96];                                                                                       \
        snprintf(nm, sizeof nm, "stream4 kG=%d ntL=%d ntS=%d grid=%d", G, NL, NS, GRID);                  \
        timeit(nm, [&] { stream4<G, NL, NS><<<GRID, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, \
                                                          pr, v, N / 4, 7u); }, B12);                        \
    }
    RUN4(1, false, false, 256);
    RUN4(1, false, false, 512);
    RUN4(1, false, false, 2048);
    RUN4(1, true, false, 256);
    RUN4(1, false, true, 256);
    RUN4(1, true, true, 256);
    RUN4(2, false, false, 256);
    RUN4(2, false, false, 512);
    RUN4(4, false, false, 256);
    RUN4(2, true, true, 256);
    RUN4(2, false, true, 512);
#define RUN16(NL, NS, GRID)                                                                                \
    {                                                                                                      \
        char nm[96];                                                                                       \
        snprintf(nm, sizeof nm, "stream16 ntL=%d ntS=%d grid=%d", NL, NS, GRID);                          \
        timeit(nm, [&] { stream16<NL, NS><<<GRID, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint4*)dp, \
                                                       (const uint4*)pr, (uint4*)v, N / 1024, 7u); }, B12);  \
    }
    timeit("stream_pp prefetch grid=256", [&] { stream_pp<true><<<256, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, N / 4, 7u); }, B12);
    timeit("stream_pp no-prefetch grid=256", [&] { stream_pp<false><<<256, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, N / 4, 7u); }, B12);
    timeit("stream_pp prefetch grid=512", [&] { stream_pp<true><<<512, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, N / 4, 7u); }, B12);
    timeit("stream_pp no-prefetch grid=512", [&] { stream_pp<false><<<512, 1024>>>((const uint4*)src, (const uint4*)dst, (const uint2*)dp, pr, v, N / 4, 7u); }, B12);
    RUN16(false, false, 256);
    RUN16(false, false, 512);
    RUN16(false, false, 1024);
    RUN16(true, false, 256);
    RUN16(false, true, 256);
    RUN16(true, true, 512);
    return 0;
}
