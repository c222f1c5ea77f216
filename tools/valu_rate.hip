// Microbenchmark: issue cost of the VALU ops the classify kernel's inner
// stages are built from (gfx950).  8 independent chains per lane, full chip
// of 1024-thread workgroups; reports cycles per wave-instruction per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

#define CHAINS(OP)                                                     \
    _Pragma("unroll 1") for (int i = 0; i < kIters; ++i) {             \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) { OP; }          \
    }

template <int K>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed) {
    uint32_t v[8];
    uint64_t w[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        v[c] = seed ^ (threadIdx.x * 0x9E3779B1u + c);
        w[c] = (uint64_t(v[c]) << 32) | (v[c] + 7);
    }
    const uint32_t s = seed | 1u;
    // inline asm: one instruction per op, nothing folded by the compiler
    if constexpr (K == 0) CHAINS(asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s)))
    if constexpr (K == 1) CHAINS(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s)))
    if constexpr (K == 2) CHAINS(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[c]) : "s"(s)))
    if constexpr (K == 3) CHAINS(asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(w[c]) : "v"(v[c])))
    if constexpr (K == 4) CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[c]) : "v"(v[(c + 1) & 7])))
    if constexpr (K == 5) CHAINS(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[c]) : "s"(s)))
    if constexpr (K == 6) CHAINS(asm volatile("v_cmp_le_u32 vcc, %0, %1" : : "v"(v[c]), "s"(s) : "vcc"))
    if constexpr (K == 7) CHAINS(asm volatile("v_bfe_u32 %0, %0, 3, 13" : "+v"(v[c])))
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc ^= v[c] ^ uint32_t(w[c]) ^ uint32_t(w[c] >> 32);
    if (acc == 0x12345678u) out[0] = acc;
}

template <int K>
float run(uint32_t* out, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<K><<<grid, 1024>>>(out, 1);
    hipEventRecord(a);
    k<K><<<grid, 1024>>>(out, 3);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* out;
    hipMalloc(&out, 4);
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int grid = p.multiProcessorCount * 2;
    const double clk_ghz = p.clockRate / 1e6;
    const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_u32_u24", "v_lshrrev_b64",
                           "v_cndmask_b32", "v_mul_hi_u32", "v_cmp_le_u32", "v_bfe_u32"};
    float ms[8] = {run<0>(out, grid), run<1>(out, grid), run<2>(out, grid), run<3>(out, grid),
                   run<4>(out, grid), run<5>(out, grid), run<6>(out, grid), run<7>(out, grid)};
    const double waves_per_simd = double(grid) * 16 / (p.multiProcessorCount * 4);
    for (int i = 0; i < 8; ++i) {
        // cycles per wave-op (one op = one line of CHAINS for one chain)
        const double cyc = ms[i] * 1e-3 * clk_ghz * 1e9 / (waves_per_simd * kIters * 8);
        printf("%-18s %8.3f ms  %6.2f cycles/wave-op (clk %.2f GHz)\n", names[i], ms[i], cyc, clk_ghz);
    }
    return 0;
}
