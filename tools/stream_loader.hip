// The decisive stream experiment for classify4_cls (round-4 verdict item 6):
// can one LDS-DMA loader wave per CU move the 12 B/packet IPv4 stream (src
// u32, dst u32, dport u16, proto u8 read; verdict u8 written) faster than the
// classify kernel's register loads?  The guide measures a read-only weight
// stream through one loader wave per CU at 6.4 TB/s (default policy) and
// 6.5-6.8 TB/s (nt) chip-wide (MI355X_MICROARCH.md, ldsdma-fill).  No
// lookups here: only the stream shapes, one 1024-thread workgroup per CU,
// 256 Mi packets of random data.
//   R   register loads exactly as classify4_cls (16-B src / dst nt, 8-B dport
//       nt, 4-B proto, 4-B nt verdict store; 4 packets per lane per step)
//   L<D,aux>  wave 0 is the loader: it DMAs each 256-packet step (src 1 KiB,
//       dst 1 KiB, dport 512 B, proto 256 B: 5 global_load_lds) into a ring
//       of 30 LDS slots and keeps D steps in flight, publishing a step once
//       its loads have landed (vmcnt); waves 1-15 consume the steps round
//       robin (ds_read, the verdict mix, nt store) and release the slot.
// Every spin is bounded (an error flag instead of a hang).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream_loader.bin tools/stream_loader.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#pragma clang diagnostic ignored "-Wint-to-pointer-cast"   // 32-bit LDS addresses

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_t;
typedef __attribute__((address_space(3))) volatile uint32_t* ldsv_t;

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
        __builtin_nontemporal_store(mix(s, d, dp, pr), V + g);
    }
}

constexpr uint32_t kSlot = 2816;             // 64 groups: src 1024, dst 1024, dport 512, proto 256
constexpr uint32_t kNS = 30;                 // ring slots (2 per consumer wave)
constexpr uint32_t kFlags = kNS * kSlot;     // full[kNS], done[kNS] after the ring
constexpr uint32_t kSpin = 1u << 22;

template <int N> __device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int kD, int kAux>
__global__ __launch_bounds__(1024) void loader_kernel(const uint4* S, const uint4* D, const uint2* DP,
                                                      const uint32_t* PR, uint32_t* V, uint32_t nsteps,
                                                      uint32_t* err) {
    extern __shared__ uint4 smem[];
    uint8_t* lds = reinterpret_cast<uint8_t*>(smem);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t flags = kFlags;           // LDS byte offset of full[] then done[]
    if (threadIdx.x < 2 * kNS) reinterpret_cast<uint32_t*>(lds + flags)[threadIdx.x] = 0u;
    __syncthreads();
    // steps of this workgroup: s_k = blockIdx.x + k gridDim.x
    const uint32_t K = nsteps > blockIdx.x ? (nsteps - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
    if (wave == 0) {
        auto issue = [&](uint32_t k) {
            const uint32_t s = blockIdx.x + k * gridDim.x;
            uint8_t* sl = lds + (k % kNS) * kSlot;
            const uint32_t* dpw = reinterpret_cast<const uint32_t*>(DP + 64u * s);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(S + 64u * s + lane), (lds_t)sl, 16, 0, kAux);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(D + 64u * s + lane), (lds_t)(sl + 1024), 16, 0, kAux);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dpw + lane), (lds_t)(sl + 2048), 4, 0, kAux);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dpw + 64 + lane), (lds_t)(sl + 2304), 4, 0, kAux);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(PR + 64u * s + lane), (lds_t)(sl + 2560), 4, 0, 0);
        };
        auto publish = [&](uint32_t k) {
            if (lane == 0) *ldsv_t(flags + 4u * (k % kNS)) = k + 1u;
        };
        for (uint32_t k = 0; k < K; ++k) {
            if (k >= kNS) {                  // the slot's previous step consumed?
                uint32_t n = 0;
                while (*ldsv_t(flags + 4u * (kNS + k % kNS)) < k - kNS + 1u && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
                if (n >= kSpin && lane == 0) atomicOr(err, 1u);
            }
            issue(k);
            if (k >= uint32_t(kD)) {
                wait_vm<5 * kD>();            // step k - D has landed
                asm volatile("" ::: "memory");
                publish(k - kD);
            }
        }
        wait_vm<0>();
        asm volatile("" ::: "memory");
        for (uint32_t k = K > uint32_t(kD) ? K - kD : 0u; k < K; ++k) publish(k);
    } else {
        const uint32_t c = wave - 1u;
        for (uint32_t k = c; k < K; k += 15u) {
            uint32_t n = 0;
            while (*ldsv_t(flags + 4u * (k % kNS)) < k + 1u && ++n < kSpin) __builtin_amdgcn_s_sleep(1);
            if (n >= kSpin && lane == 0) atomicOr(err, 2u);
            asm volatile("" ::: "memory");
            const uint8_t* sl = lds + (k % kNS) * kSlot;
            const v4u s = *reinterpret_cast<const v4u*>(sl + 16u * lane);
            const v4u d = *reinterpret_cast<const v4u*>(sl + 1024u + 16u * lane);
            const v2u dp = *reinterpret_cast<const v2u*>(sl + 2048u + 8u * lane);
            const uint32_t pr = *reinterpret_cast<const uint32_t*>(sl + 2560u + 4u * lane);
            const uint32_t v = mix(make_uint4(s.x, s.y, s.z, s.w), make_uint4(d.x, d.y, d.z, d.w), make_uint2(dp.x, dp.y), pr);
            // the reads are done before the slot is released (LDS is in order per wave)
            asm volatile("" ::: "memory");
            if (lane == 0) *ldsv_t(flags + 4u * (kNS + k % kNS)) = k + 1u;
            __builtin_nontemporal_store(v, V + 64u * (blockIdx.x + k * gridDim.x) + lane);
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
    const size_t lds = kFlags + 8 * kNS;
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
            printf("%-10s %.4f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
        }
        CK(hipMemset(v, 0, N));
        launch();
        CK(hipMemset(err + 1, 0, 4));
        check<<<1024, 256>>>(src, dst, dp, pr, v, G, err + 1);
        uint32_t h[2];
        CK(hipMemcpy(h, err, 8, hipMemcpyDeviceToHost));
        printf("%-10s check: %u wrong groups, spin flags %u\n", name, h[1], h[0]);
        return 0;
    };
    for (int i = 0; i < 200; ++i) reg_kernel<<<ncu, 1024>>>(src, dst, dp, pr, v, G);
    CK(hipDeviceSynchronize());
    const uint32_t steps = G / 64;
#define LOADER(Dd, A)                                                                                              \
    {                                                                                                              \
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(loader_kernel<Dd, A>),                                \
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));                            \
        if (timed("L" #Dd "_" #A, [&] { loader_kernel<Dd, A><<<ncu, 1024, lds>>>(src, dst, dp, pr, v, steps, err); })) \
            return 1;                                                                                              \
    }
    if (timed("R", [&] { reg_kernel<<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    LOADER(12, 2)
    LOADER(12, 0)
    LOADER(8, 2)
    LOADER(4, 2)
    if (timed("R", [&] { reg_kernel<<<ncu, 1024>>>(src, dst, dp, pr, v, G); })) return 1;
    return 0;
}
