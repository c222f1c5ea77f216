// The round-5 LDS-DMA stream probe for classify4_cls, in the guide's shape
// (MI355X_MICROARCH.md "ldsdma-fill": one loader wave
// per CU, 1 KiB per global_load_lds_dwordx4 wave-instruction, 6.4 TB/s
// default policy, 6.5-6.8 nt).  Round 4's probe moved 256-packet steps
// (five DMA pieces per 2.8 KB, three of them 256 B) through a 30-slot 84 KB
// ring and got 3.4 TB/s; that ring could not coexist with config 3's
// 125 KB LDS image.  Here:
//   - a step of P packets (1024 or 512) moves every field with 16-B/lane
//     pieces: P = 1024: src 4 x 1 KiB, dst 4 x 1 KiB, dport 2 x 1 KiB, proto
//     1 x 1 KiB (11 KiB, 11 instructions); P = 512: src 2, dst 2, dport 1 x
//     1 KiB, proto one 512-B piece (32 lanes);
//   - a ring of NS slots, at most 34 KiB (P 1024: 3 slots; P 512: 6), after a
//     125 KB reservation standing for the config-3 image (RES), or without it
//     (the ceiling of the route when nothing else needs LDS);
//   - wave 0 is the loader (keeps D steps in flight, publishes a step once
//     vmcnt says it landed), waves 1-15 consume quarter-steps of 256 packets
//     round robin (ds_read, the verdict mix, a non-temporal 4-B store per
//     lane) and release them with an LDS add.
// 256 Mi packets of random data, one 1024-thread workgroup per CU, checked.
// Every spin is bounded (an error flag instead of a hang).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream_ring.bin tools/stream_ring.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#pragma clang diagnostic ignored "-Wint-to-pointer-cast"   // 32-bit LDS addresses

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_t;
typedef __attribute__((address_space(3))) volatile uint32_t* ldsv_t;
typedef __attribute__((address_space(3))) uint32_t* ldsa_t;

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

// the classify kernel's register stream (the live floor's shape)
template <bool ST = true>
__global__ __launch_bounds__(1024) void reg_kernel(const uint4* S, const uint4* D, const uint2* DP, const uint32_t* PR,
                                                   uint32_t* V, uint32_t ngroups) {
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
        if (ST || m == 0xFFFFFFFFu) __builtin_nontemporal_store(m, V + g);   // read-only variant: never true
    }
}

constexpr uint32_t kRes = 125 * 1024;       // stands for config 3's LDS image
constexpr uint32_t kSpin = 1u << 22;

template <int N> __device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int P>
struct Shape {
    static constexpr uint32_t kSlot = 11u * P;          // src 4P, dst 4P, dport 2P, proto P
    static constexpr uint32_t kPieces = P == 1024 ? 11 : 6;
    static constexpr uint32_t kWps = P / 256;            // consumer waves per step
};

template <int P, int NS, int D, int AUX, bool RES, bool ST = true>
__global__ __launch_bounds__(1024) void ring_kernel(const uint8_t* S, const uint8_t* Dst, const uint8_t* DP,
                                                    const uint8_t* PR, uint32_t* V, uint32_t nsteps, uint32_t* err) {
    using Sh = Shape<P>;
    static_assert(D >= 1 && D < NS, "in flight");
    static_assert(Sh::kPieces * D < 64, "vmcnt");
    extern __shared__ uint4 smem[];
    const uint32_t base = RES ? kRes : 0u;                 // ring after the reservation
    const uint32_t flags = base + NS * Sh::kSlot;           // full[NS], done[NS]
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (threadIdx.x < 2 * NS) *ldsv_t(flags + 4u * threadIdx.x) = 0u;
    __syncthreads();
    const uint32_t K = nsteps > blockIdx.x ? (nsteps - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
    if (wave == 0) {
        auto issue = [&](uint32_t k) {
            const uint64_t s = blockIdx.x + uint64_t(k) * gridDim.x;
            const uint32_t sl = base + (k % NS) * Sh::kSlot;
            const uint8_t* src = S + s * 4u * P;
            const uint8_t* dst = Dst + s * 4u * P;
            const uint8_t* dp = DP + s * 2u * P;
            const uint8_t* pr = PR + s * uint64_t(P);
#pragma unroll
            for (int j = 0; j < 4 * P / 1024; ++j)
                __builtin_amdgcn_global_load_lds(src + 1024 * j + 16 * lane, (lds_t)(sl + 1024 * j), 16, 0, AUX);
#pragma unroll
            for (int j = 0; j < 4 * P / 1024; ++j)
                __builtin_amdgcn_global_load_lds(dst + 1024 * j + 16 * lane, (lds_t)(sl + 4 * P + 1024 * j), 16, 0, AUX);
#pragma unroll
            for (int j = 0; j < 2 * P / 1024; ++j)
                __builtin_amdgcn_global_load_lds(dp + 1024 * j + 16 * lane, (lds_t)(sl + 8 * P + 1024 * j), 16, 0, AUX);
            if (P == 1024 || lane < 32)                    // proto: one 1 KiB piece, or a 512-B one
                __builtin_amdgcn_global_load_lds(pr + 16 * lane, (lds_t)(sl + 10 * P), 16, 0, AUX);
        };
        auto publish = [&](uint32_t k) {
            if (lane == 0) *ldsv_t(flags + 4u * (k % NS)) = k + 1u;
        };
        for (uint32_t k = 0; k < K; ++k) {
            if (k >= uint32_t(NS)) {                        // the slot's previous step consumed?
                const uint32_t want = Sh::kWps * (k / NS);
                uint32_t n = 0;
                while (*ldsv_t(flags + 4u * (NS + k % NS)) < want && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
                if (n >= kSpin && lane == 0) atomicOr(err, 1u);
            }
            issue(k);
            if (k >= uint32_t(D)) {
                wait_vm<int(Sh::kPieces) * D>();            // step k - D has landed
                asm volatile("" ::: "memory");
                publish(k - D);
            }
        }
        wait_vm<0>();
        asm volatile("" ::: "memory");
        for (uint32_t k = K > uint32_t(D) ? K - D : 0u; k < K; ++k) publish(k);
    } else {
        const uint32_t c = wave - 1u;
        for (uint32_t idx = c; idx < K * Sh::kWps; idx += 15u) {
            const uint32_t k = idx / Sh::kWps, q = idx % Sh::kWps;
            uint32_t n = 0;
            while (*ldsv_t(flags + 4u * (k % NS)) < k + 1u && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
            if (n >= kSpin && lane == 0) atomicOr(err, 2u);
            asm volatile("" ::: "memory");
            const uint32_t sl = base + (k % NS) * Sh::kSlot;
            const uint32_t p0 = 256u * q + 4u * lane;        // this lane's four packets in the step
            const v4u s = *(const __attribute__((address_space(3))) v4u*)(sl + 4u * p0);
            const v4u d = *(const __attribute__((address_space(3))) v4u*)(sl + 4u * P + 4u * p0);
            const v2u dp = *(const __attribute__((address_space(3))) v2u*)(sl + 8u * P + 2u * p0);
            const uint32_t pr = *(const __attribute__((address_space(3))) uint32_t*)(sl + 10u * P + p0);
            const uint32_t v = mix(make_uint4(s.x, s.y, s.z, s.w), make_uint4(d.x, d.y, d.z, d.w),
                                   make_uint2(dp.x, dp.y), pr);
            // LDS reads retire in order per wave: the release follows them
            __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0)
            if (lane == 0) __hip_atomic_fetch_add(ldsa_t(flags + 4u * (NS + k % NS)), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint64_t s_glob = blockIdx.x + uint64_t(k) * gridDim.x;
            if (ST || v == 0xFFFFFFFFu) __builtin_nontemporal_store(v, V + (s_glob * P + p0) / 4u);
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
    const uint64_t N = 1ull << 28;                 // packets
    const uint32_t G = uint32_t(N / 4);            // 4-packet groups
    uint4 *src, *dst;
    uint2* dp;
    uint32_t *pr, *v, *err;
    // skewed like the engine's batches (vpp_amd/csrc/fleet.cpp)
    CK(hipMalloc(&src, N * 4)); CK(hipMalloc(&dst, N * 4)); CK(hipMalloc(&dp, N * 2));
    CK(hipMalloc(&pr, N)); CK(hipMalloc(&v, N)); CK(hipMalloc(&err, 8));
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(src), N * 4 / 8, 1);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dst), N * 4 / 8, 2);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(dp), N * 2 / 8, 3);
    fill_rand<<<1024, 256>>>(reinterpret_cast<uint64_t*>(pr), N / 8, 4);
    CK(hipMemset(err, 0, 8));
    CK(hipDeviceSynchronize());
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = 12.0 * double(N);
    auto timed = [&](const char* name, auto launch) -> int {
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
            printf("%-26s %.4f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
        }
        CK(hipMemset(v, 0, N));
        launch();
        CK(hipMemset(err + 1, 0, 4));
        check<<<1024, 256>>>(src, dst, dp, pr, v, G, err + 1);
        uint32_t h[2];
        CK(hipMemcpy(h, err, 8, hipMemcpyDeviceToHost));
        printf("%-26s check: %u wrong groups, spin flags %u\n", name, h[1], h[0]);
        fflush(stdout);
        return h[0] != 0 ? 1 : 0;                     // a spin gave up: stop here
    };
    for (int i = 0; i < 200; ++i) reg_kernel<true><<<ncu, 1024>>>(src, dst, dp, pr, v, G);
    CK(hipDeviceSynchronize());
#define RING(P, NS, Dd, A, R, ST)                                                                                 \
    {                                                                                                             \
        using Sh = Shape<P>;                                                                                      \
        const size_t lds = (R ? kRes : 0) + NS * Sh::kSlot + 8 * NS;                                              \
        auto kf = ring_kernel<P, NS, Dd, A, R, ST>;                                                               \
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,     \
                               int(lds)));                                                                        \
        char nm[64];                                                                                              \
        snprintf(nm, sizeof nm, "P%d NS%d D%d aux%d %s%s %zuB", P, NS, Dd, A, R ? "res" : "alone",                \
                 ST ? "" : " read-only", lds);                                                                    \
        if (timed(nm, [&] {                                                                                       \
                hipLaunchKernelGGL(kf, dim3(ncu), dim3(1024), lds, 0, reinterpret_cast<const uint8_t*>(src),      \
                                   reinterpret_cast<const uint8_t*>(dst), reinterpret_cast<const uint8_t*>(dp),   \
                                   reinterpret_cast<const uint8_t*>(pr), v, uint32_t(N / P), err);               \
            }))                                                                                                   \
            return 1;                                                                                             \
    }
    // read-only variants: no verdict store (the guide's ldsdma-fill figure is a read-only stream);
    // their check fails by design, so they run after the checked ones
    if (timed("R (register, classify4_cls)", [&] { reg_kernel<true><<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    RING(512, 6, 4, 2, true, true)
    RING(512, 6, 3, 2, true, true)
    RING(512, 6, 4, 0, true, true)
    RING(512, 12, 8, 2, false, true)
    RING(1024, 3, 2, 2, true, true)
    if (timed("R (register, classify4_cls)", [&] { reg_kernel<true><<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    if (timed("R read-only", [&] { reg_kernel<false><<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    RING(512, 6, 4, 2, true, false)
    RING(512, 12, 10, 2, false, false)
    RING(1024, 8, 5, 2, false, false)
    if (timed("R read-only", [&] { reg_kernel<false><<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    return 0;
}
