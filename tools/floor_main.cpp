// Stream floor through the C ABI without PyTorch in the process (HIP runtime
// of /opt/rocm): is the in-process gap to tools/stream_bench.hip the runtime?
// build: hipcc -O2 -o tools/floor_main.bin tools/floor_main.cpp -Lvpp_amd -lcontivcls -Wl,-rpath,'$ORIGIN/../vpp_amd'
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../include/contivcls.h"

int main() {
    cls_engine* e = nullptr;
    cls_config cfg{};
    cfg.device = 0;
    if (cls_engine_create(&cfg, &e) != CLS_OK) return 1;
    const uint64_t n = 1ull << 28;
    void *s, *d, *dp, *pr, *v;
    if (hipMalloc(&s, n * 4) || hipMalloc(&d, n * 4) || hipMalloc(&dp, n * 2) || hipMalloc(&pr, n) || hipMalloc(&v, n))
        return 2;
    (void)hipMemset(s, 1, n * 4); (void)hipMemset(d, 2, n * 4); (void)hipMemset(dp, 3, n * 2);
    (void)hipMemset(pr, 1, n); (void)hipDeviceSynchronize();
    cls_pkt_soa pk{};
    pk.af = CLS_AF_V4;
    pk.src4 = static_cast<const uint32_t*>(s);
    pk.dst4 = static_cast<const uint32_t*>(d);
    pk.dport = static_cast<const uint16_t*>(dp);
    pk.proto = static_cast<const uint8_t*>(pr);
    float ms = 0;
    for (int r = 0; r < 3; ++r) {
        int rc = cls_stream_floor(e, &pk, n, static_cast<uint8_t*>(v), 10, &ms, nullptr);
        std::printf("rc %d floor %.4f ms\n", rc, ms);
    }
    cls_engine_destroy(e);
    return 0;
}
