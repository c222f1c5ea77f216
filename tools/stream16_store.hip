// Where the 16-byte layout's verdict store costs its time (round 6, VERDICT
// r05 item 2).  Config 5's stream reads 35 B and writes 1 B per packet; the
// classify kernel runs at this stream's floor, and the floor is 0.39 ms over
// the reads alone for 256 MB written (IPv4: 0.105 ms for the same bytes).
// The variants keep classify16_cls's read shape (lane l of a 256-packet wave
// step: packets base + 64k + l, 1 KiB per 16-B load instruction) and change
// only where the store sits relative to the loads it may hold up -- vmcnt
// counts loads, stores and LDS-DMA together, in issue order, so a wave that
// waits for a load also waits for every older store:
//   A    as classify16_cls: loads of step g, then its four byte stores; the
//        next step's load wait covers those stores
//   RO   A without the stores (the read ceiling)
//   D    deferred: step g's stores issued after step g + 1's loads, so a load
//        wait never covers a store issued just before it
//   D1   D with the four bytes as one 4-B store per lane (lanes exchange with
//        ds_bpermute, 256 B per instruction)
//   S4   verdicts of four steps gathered in LDS, one 16-B store per lane every
//        fourth step (after that step's loads): a quarter of the store events
//   P    the next step's loads issued before this step's stores and held in
//        registers (one step ahead)
//   W2 / W4 / W16  A with the stores of one wave step in 2 / 4 / 16 only (full
//        lines, a half / quarter / sixteenth of the bytes): does the cost
//        scale with the bytes written?
// build: hipcc -O3 --offload-arch=gfx950 -o tools/stream16_store.bin tools/stream16_store.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

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

struct Step {
    uint4 s[4], d[4];
    uint32_t dp[4], pr[4];
};

__device__ __forceinline__ void load(Step& b, const uint4* S, const uint4* D, const uint16_t* DP, const uint8_t* PR,
                                     uint32_t base, uint32_t lane) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b.s[k] = ldnt(S + base + 64u * k + lane);
        b.d[k] = ldnt(D + base + 64u * k + lane);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b.dp[k] = __builtin_nontemporal_load(DP + base + 64u * k + lane);
        b.pr[k] = __builtin_nontemporal_load(PR + base + 64u * k + lane);
    }
}

__device__ __forceinline__ void store4(uint8_t* V, uint32_t base, uint32_t lane, const uint32_t (&v)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(uint8_t(v[k]), V + base + 64u * k + lane);
}

// lane m stores packets base + 4m .. 4m + 3 as one word
__device__ __forceinline__ void store1(uint8_t* V, uint32_t base, uint32_t lane, const uint32_t (&v)[4]) {
    const uint32_t packed = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
    const uint32_t kb = 8u * (lane >> 4);
    uint32_t out = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) out |= ((bperm(packed, (4u * lane + j) & 63u) >> kb) & 0xFFu) << (8 * j);
    __builtin_nontemporal_store(out, reinterpret_cast<uint32_t*>(V + base) + lane);
}

template <int M>
__global__ __launch_bounds__(1024) void k16(const uint4* S, const uint4* D, const uint16_t* DP, const uint8_t* PR,
                                            uint8_t* V, uint32_t n, uint32_t magic) {
    extern __shared__ uint4 smem[];                         // S4: 1 KiB per wave, at LDS 1024 wave
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t nthreads = gridDim.x * blockDim.x;
    const uint32_t nsteps = n / 256u * 64u;
    const uint32_t g0 = blockIdx.x * blockDim.x + threadIdx.x;
    auto base_of = [&](uint32_t g) { return 4u * (g & ~63u); };
    if constexpr (M == 0 || M == 1 || M >= 6) {
        constexpr uint32_t Q = M == 6 ? 2u : M == 7 ? 4u : 16u;
        for (uint32_t g = g0; g < nsteps; g += nthreads) {
            Step b;
            load(b, S, D, DP, PR, base_of(g), lane);
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = mix(b.s[k], b.d[k], b.dp[k], b.pr[k]);
            if constexpr (M == 0) store4(V, base_of(g), lane, v);
            else if constexpr (M >= 6) {
                if ((g / nthreads) % Q == 0u) store4(V, base_of(g), lane, v);    // wave-uniform
                else if ((v[0] ^ v[1] ^ v[2] ^ v[3]) == magic) V[base_of(g) + lane] = 1;   // keeps the loads
            } else if ((v[0] ^ v[1] ^ v[2] ^ v[3]) == magic) V[base_of(g) + lane] = 1;   // never (magic > 3)
        }
    } else if constexpr (M == 2 || M == 3) {
        uint32_t pv[4] = {0u, 0u, 0u, 0u}, pg = 0;
        bool have = false;
        for (uint32_t g = g0; g < nsteps; g += nthreads) {
            Step b;
            load(b, S, D, DP, PR, base_of(g), lane);
            if (have) {
                if constexpr (M == 2) store4(V, base_of(pg), lane, pv);
                else store1(V, base_of(pg), lane, pv);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) pv[k] = mix(b.s[k], b.d[k], b.dp[k], b.pr[k]);
            pg = g;
            have = true;
        }
        if (have) {
            if constexpr (M == 2) store4(V, base_of(pg), lane, pv);
            else store1(V, base_of(pg), lane, pv);
        }
    } else if constexpr (M == 4) {
        // S4: step j of a group of four writes its 256 verdict bytes into the
        // wave's LDS row at 256 j; the fourth step's loads issued, one 16-B
        // store per lane moves the group (lane L: segment L / 16, bytes
        // 16 (L % 16) .. + 15 of that step)
        typedef __attribute__((address_space(3))) uint8_t* l8_t;
        const uint32_t row = 1024u * wave;
        uint32_t gs[4] = {0u, 0u, 0u, 0u};
        uint32_t j = 0;
        for (uint32_t g = g0; g < nsteps; g += nthreads) {
            Step b;
            load(b, S, D, DP, PR, base_of(g), lane);
            if (j == 0 && g != g0) {                        // the previous group, behind these loads
                const uint32_t seg = lane >> 4;
                const v4u x = *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(row + 16u * lane);
                __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(V + base_of(gs[seg]) + 16u * (lane & 15u)));
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                *(l8_t)(row + 256u * j + 64u * k + lane) = uint8_t(mix(b.s[k], b.d[k], b.dp[k], b.pr[k]));
            gs[j] = g;
            j = (j + 1u) & 3u;
        }
        // the last (possibly partial) group: bytes of the steps it holds
        const uint32_t have = j == 0 ? 4u : j;
        const uint32_t seg = lane >> 4;
        if (g0 < nsteps && seg < have) {
            const v4u x = *reinterpret_cast<const __attribute__((address_space(3))) v4u*>(row + 16u * lane);
            __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(V + base_of(gs[seg]) + 16u * (lane & 15u)));
        }
    } else {
        // P: next step's loads in registers before this step's stores
        Step a, b;
        uint32_t g = g0;
        if (g < nsteps) load(a, S, D, DP, PR, base_of(g), lane);
        while (g < nsteps) {
            const uint32_t gn = g + nthreads;
            if (gn < nsteps) load(b, S, D, DP, PR, base_of(gn), lane);
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = mix(a.s[k], a.d[k], a.dp[k], a.pr[k]);
            store4(V, base_of(g), lane, v);
            a = b;
            g = gn;
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
            printf("%-4s %.4f ms  %.2f TB/s\n", name, ms, bytes / ms / 1e9);
        }
        fflush(stdout);
        return 0;
    };
    auto check = [&](const char* name) -> int {
        CK(hipMemset(bad, 0, 4));
        diff<<<1024, 256>>>(v, v0, N, bad);
        uint32_t h = 0;
        CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
        printf("%s check against A: %u bytes differ\n", name, h);
        return 0;
    };
    const uint32_t n = uint32_t(N);
    for (int i = 0; i < 40; ++i) k16<0><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v0, n, 7);
    CK(hipDeviceSynchronize());
    for (int round = 0; round < 2; ++round) {
        timed("A", [&] { k16<0><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v0, n, 7); });
        timed("RO", [&] { k16<1><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        CK(hipMemset(v, 0, N));
        timed("D", [&] { k16<2><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0 && check("D")) return 1;
        CK(hipMemset(v, 0, N));
        timed("D1", [&] { k16<3><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0 && check("D1")) return 1;
        CK(hipMemset(v, 0, N));
        timed("S4", [&] { k16<4><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0 && check("S4")) return 1;
        CK(hipMemset(v, 0, N));
        timed("P", [&] { k16<5><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        if (round == 0 && check("P")) return 1;
        timed("W2", [&] { k16<6><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        timed("W4", [&] { k16<7><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
        timed("W16", [&] { k16<8><<<ncu, 1024, 16384>>>(src, dst, dp, pr, v, n, 7); });
    }
    return 0;
}
