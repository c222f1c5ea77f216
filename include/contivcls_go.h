/*
 * contivcls_go.h -- cgo shims of the C ABI (contivcls.h) for a Go host as
 * old as the reference's Go 1.9.x (/root/reference .travis.yml:7-8).
 *
 * cgo (Go >= 1.6) lets C receive a pointer to Go memory only if that memory
 * holds no Go pointers.  The ABI's packet and connection records
 * (cls_pkt_soa, cls_conn_soa) hold array pointers, so a Go value of them
 * that points at Go slices may not be passed -- Go 1.21's runtime.Pinner is
 * the newer way around that.  These shims take each slice base as a scalar
 * argument instead (a pointer to pointer-free Go memory, valid for the call)
 * and build the records on the C stack, so the Go side needs neither
 * runtime.Pinner nor unsafe.Slice.  Every shim is one ABI call; the engine
 * keeps no caller pointer after it returns (contivcls.h conventions).
 *
 * Static inline: the header is compiled into the cgo preamble (and into
 * go/shimtest/shimtest.c, which exercises exactly these functions through
 * libcontivcls.so on the GPU, tests/test_gpu_go_shims.py).
 */
#ifndef CONTIVCLS_GO_H
#define CONTIVCLS_GO_H

#include <string.h>

#include "contivcls.h"

/* cls_engine_create over devices[0 .. n) (n 1: one device, devices[0] may be
 * -1 for the current one).  Replaces NewMockACLEngine (aclengine_mock.go:124). */
static inline int clsg_engine_create(const int* devices, uint32_t n, cls_engine** out) {
    cls_config c;
    memset(&c, 0, sizeof c);
    c.device = n ? devices[0] : -1;
    if (n > 1) {
        c.n_devices = n;
        c.devices = devices;
    }
    return cls_engine_create(&c, out);
}

/* cls_classify of an IPv4 batch (host-order addresses): evalACL per packet
 * (aclengine_mock.go:473-668) and the table's hit counters. */
static inline int clsg_classify_v4(cls_engine* e, uint32_t table_id, const uint32_t* src4, const uint32_t* dst4,
                                   const uint16_t* dport, const uint8_t* proto, uint64_t n, uint8_t* verdict,
                                   uint64_t* counters, uint32_t flags) {
    cls_pkt_soa p;
    memset(&p, 0, sizeof p);
    p.af = CLS_AF_V4;
    p.src4 = src4;
    p.dst4 = dst4;
    p.dport = dport;
    p.proto = proto;
    return cls_classify(e, table_id, &p, n, verdict, counters, flags, NULL);
}

/* cls_classify of a 16-byte batch (n x 16 network-order bytes per address;
 * IPv4 as IPv4-mapped, Go's net.IP.To16). */
/* cls_classify_rules over an IPv4 batch: each packet's ACLAction and terminating rule. */
static inline int clsg_classify_rules_v4(cls_engine* e, uint32_t table_id, const uint32_t* src4, const uint32_t* dst4,
                                         const uint16_t* dport, const uint8_t* proto, uint64_t n, uint8_t* verdict,
                                         uint32_t* rules) {
    cls_pkt_soa p;
    memset(&p, 0, sizeof p);
    p.af = CLS_AF_V4;
    p.src4 = src4;
    p.dst4 = dst4;
    p.dport = dport;
    p.proto = proto;
    return cls_classify_rules(e, table_id, &p, n, verdict, rules, 0, NULL);
}

static inline int clsg_classify_v16(cls_engine* e, uint32_t table_id, const uint8_t* src16, const uint8_t* dst16,
                                    const uint16_t* dport, const uint8_t* proto, uint64_t n, uint8_t* verdict,
                                    uint64_t* counters, uint32_t flags) {
    cls_pkt_soa p;
    memset(&p, 0, sizeof p);
    p.af = CLS_AF_V16;
    p.src16 = src16;
    p.dst16 = dst16;
    p.dport = dport;
    p.proto = proto;
    return cls_classify(e, table_id, &p, n, verdict, counters, flags, NULL);
}

/* cls_connect_batch of IPv4 connections: testConnection per connection
 * (aclengine_mock.go:394-471) between interface ids (cls_if_id). */
static inline int clsg_connect_v4(cls_engine* e, const uint32_t* src_if, const uint32_t* dst_if, const uint32_t* src4,
                                  const uint32_t* dst4, const uint16_t* sport, const uint16_t* dport,
                                  const uint8_t* proto, uint64_t n, uint8_t* out, uint32_t flags) {
    cls_conn_soa c;
    memset(&c, 0, sizeof c);
    c.pkt.af = CLS_AF_V4;
    c.pkt.src4 = src4;
    c.pkt.dst4 = dst4;
    c.pkt.sport = sport;
    c.pkt.dport = dport;
    c.pkt.proto = proto;
    c.src_if = src_if;
    c.dst_if = dst_if;
    return cls_connect_batch(e, &c, n, out, flags, NULL);
}

/* cls_connect_batch of 16-byte connections. */
static inline int clsg_connect_v16(cls_engine* e, const uint32_t* src_if, const uint32_t* dst_if, const uint8_t* src16,
                                   const uint8_t* dst16, const uint16_t* sport, const uint16_t* dport,
                                   const uint8_t* proto, uint64_t n, uint8_t* out, uint32_t flags) {
    cls_conn_soa c;
    memset(&c, 0, sizeof c);
    c.pkt.af = CLS_AF_V16;
    c.pkt.src16 = src16;
    c.pkt.dst16 = dst16;
    c.pkt.sport = sport;
    c.pkt.dport = dport;
    c.pkt.proto = proto;
    c.src_if = src_if;
    c.dst_if = dst_if;
    return cls_connect_batch(e, &c, n, out, flags, NULL);
}

/* The pinned host array of a batch field (CLS_BATCH_MIRROR), NULL if none:
 * C memory, so Go may keep it as a slice (Go 1.9: (*[1 << 32]T)(p)[:n:n]). */
static inline void* clsg_batch_mirror(cls_batch* b, uint32_t field) {
    void* p = NULL;
    return cls_batch_mirror(b, field, &p) == CLS_OK ? p : NULL;
}

/* The ABI version the shims were compiled against (a Go host checks it
 * against cls_abi_version() at start-up). */
static inline int clsg_abi_version(void) { return CLS_ABI_VERSION; }

#endif /* CONTIVCLS_GO_H */
