/*
 * ORACLE -- test infrastructure only.  CPU restatement of the Contiv-VPP Go
 * ACL evaluation path, used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as bench.py's `cpu_baseline` leg.  Nothing in
 * the product (vpp_amd/) may link, import or call this file.
 *
 * Restated from (paths relative to the reference root):
 *   mock/aclengine/aclengine_mock.go:473-668  evalACL            -> orc_eval_acl
 *   mock/aclengine/aclengine_mock.go:394-471  testConnection     -> orc_test_connection
 *   Go 1.9 stdlib net (not vendored; Go 1.9.x per .travis.yml:7-8):
 *     ParseCIDR / parseIPv4 / parseIPv6 / dtoi / xtoi / IP.Mask / IP.To4 /
 *     IPNet.Contains / networkNumberAndMask    -> go_* below
 *
 * Parity pinning: the IPv4 behaviour is pinned by the 221 Connection*
 * known-answer tests of plugins/policy/renderer/acl/acl_renderer_test.go
 * (tests/golden/acl_scenarios.json, replayed by tests/test_oracle_scenarios.py).
 * IPv6 / IPv4-mapped / malformed-rule behaviour follows the Go 1.9 source
 * text and is parity-unpinned by reference tests.
 *
 * Two evaluators:
 *   orc_classify_faithful -- literal evalACL: re-parses every CIDR string of
 *     every rule for every packet (aclengine_mock.go:500,514), single thread
 *     (the Go engine serialises under its mutex, :397).  Stand-in for "the Go
 *     reference" as CPU baseline.
 *   orc_classify_fast -- rules pre-parsed once, same first-match semantics,
 *     OpenMP over host cores.  The optimised CPU port.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/contivcls.h"

/* ---------------------------------------------------------------------------
 * Go 1.9 net package restatement
 * ------------------------------------------------------------------------ */
#define GO_BIG 0xFFFFFF

typedef struct {
    int len;            /* 0 (nil), 4 or 16 */
    uint8_t b[16];
} go_ip;

typedef struct {
    go_ip ip;           /* network number (ip.Mask(m)) */
    int mlen;           /* 4 or 16 */
    uint8_t m[16];
} go_ipnet;

/* dtoi (Go 1.9 net/parse.go) */
static int go_dtoi(const char* s, int slen, int* n_out, int* i_out) {
    int n = 0, i;
    for (i = 0; i < slen && s[i] >= '0' && s[i] <= '9'; i++) {
        n = n * 10 + (s[i] - '0');
        if (n >= GO_BIG) { *n_out = GO_BIG; *i_out = i; return 0; }
    }
    if (i == 0) { *n_out = 0; *i_out = 0; return 0; }
    *n_out = n; *i_out = i; return 1;
}

/* xtoi (Go 1.9 net/parse.go) */
static int go_xtoi(const char* s, int slen, int* n_out, int* i_out) {
    int n = 0, i;
    for (i = 0; i < slen; i++) {
        char c = s[i];
        if (c >= '0' && c <= '9') { n = n * 16 + (c - '0'); }
        else if (c >= 'a' && c <= 'f') { n = n * 16 + (c - 'a') + 10; }
        else if (c >= 'A' && c <= 'F') { n = n * 16 + (c - 'A') + 10; }
        else break;
        if (n >= GO_BIG) { *n_out = 0; *i_out = i; return 0; }
    }
    if (i == 0) { *n_out = 0; *i_out = 0; return 0; }
    *n_out = n; *i_out = i; return 1;
}

static const uint8_t v4InV6Prefix[12] = {0,0,0,0,0,0,0,0,0,0,0xff,0xff};

/* parseIPv4 (Go 1.9 net/ip.go): returns a 16-byte IPv4-mapped IP */
static int go_parse_ipv4(const char* s, int slen, go_ip* out) {
    uint8_t p[4];
    for (int i = 0; i < 4; i++) {
        if (slen == 0) return 0;
        if (i > 0) {
            if (s[0] != '.') return 0;
            s++; slen--;
        }
        int n, c;
        if (!go_dtoi(s, slen, &n, &c) || n > 0xFF) return 0;
        s += c; slen -= c;
        p[i] = (uint8_t)n;
    }
    if (slen != 0) return 0;
    out->len = 16;
    memcpy(out->b, v4InV6Prefix, 12);
    memcpy(out->b + 12, p, 4);
    return 1;
}

/* parseIPv6 (Go 1.9 net/ip.go), zoneAllowed = false */
static int go_parse_ipv6(const char* s, int slen, go_ip* out) {
    uint8_t ip[16];
    memset(ip, 0, 16);
    int ellipsis = -1;
    if (slen >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        s += 2; slen -= 2;
        if (slen == 0) { out->len = 16; memcpy(out->b, ip, 16); return 1; }
    }
    int i = 0;
    while (i < 16) {
        int n, c;
        if (!go_xtoi(s, slen, &n, &c) || n > 0xFFFF) return 0;
        if (c < slen && s[c] == '.') {
            if (ellipsis < 0 && i != 16 - 4) return 0;
            if (i + 4 > 16) return 0;
            go_ip ip4;
            if (!go_parse_ipv4(s, slen, &ip4)) return 0;
            ip[i] = ip4.b[12]; ip[i + 1] = ip4.b[13];
            ip[i + 2] = ip4.b[14]; ip[i + 3] = ip4.b[15];
            slen = 0;
            i += 4;
            break;
        }
        ip[i] = (uint8_t)(n >> 8);
        ip[i + 1] = (uint8_t)n;
        i += 2;
        s += c; slen -= c;
        if (slen == 0) break;
        if (s[0] != ':' || slen == 1) return 0;
        s++; slen--;
        if (s[0] == ':') {
            if (ellipsis >= 0) return 0;
            ellipsis = i;
            s++; slen--;
            if (slen == 0) break;
        }
    }
    if (slen != 0) return 0;
    if (i < 16) {
        if (ellipsis < 0) return 0;
        int n = 16 - i;
        for (int j = i - 1; j >= ellipsis; j--) ip[j + n] = ip[j];
        for (int j = ellipsis + n - 1; j >= ellipsis; j--) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return 0;
    }
    out->len = 16;
    memcpy(out->b, ip, 16);
    return 1;
}

/* ParseIP (Go 1.9): tries IPv4 first (by scanning for '.' or ':'). */
int orc_parse_ip(const char* s, uint8_t out16[16], int* out_len) {
    int slen = (int)strlen(s);
    go_ip ip;
    ip.len = 0;
    for (int i = 0; i < slen; i++) {
        if (s[i] == '.') { if (!go_parse_ipv4(s, slen, &ip)) ip.len = 0; break; }
        if (s[i] == ':') { if (!go_parse_ipv6(s, slen, &ip)) ip.len = 0; break; }
    }
    *out_len = ip.len;
    if (ip.len) memcpy(out16, ip.b, 16);
    return ip.len != 0;
}

/* CIDRMask(ones, bits) */
static void go_cidr_mask(int ones, int bits, uint8_t* m) {
    int l = bits / 8;
    for (int i = 0; i < l; i++) {
        if (ones >= 8) { m[i] = 0xff; ones -= 8; continue; }
        m[i] = (uint8_t)~(0xff >> ones);
        ones = 0;
    }
}

static int all_ff(const uint8_t* b, int n) {
    for (int i = 0; i < n; i++) if (b[i] != 0xff) return 0;
    return 1;
}

/* IP.Mask (Go 1.9) */
static int go_ip_mask(const go_ip* ip_in, const uint8_t* mask_in, int mlen, go_ip* out) {
    const uint8_t* ip = ip_in->b;
    int iplen = ip_in->len;
    const uint8_t* mask = mask_in;
    if (mlen == 16 && iplen == 4 && all_ff(mask, 12)) { mask += 12; mlen = 4; }
    if (mlen == 4 && iplen == 16 && memcmp(ip, v4InV6Prefix, 12) == 0) { ip += 12; iplen = 4; }
    if (iplen != mlen) { out->len = 0; return 0; }
    out->len = iplen;
    for (int i = 0; i < iplen; i++) out->b[i] = ip[i] & mask[i];
    return 1;
}

/* ParseCIDR (Go 1.9 net/ip.go).  Returns 1 on success. */
static int go_parse_cidr(const char* s, go_ipnet* net) {
    int slen = (int)strlen(s);
    int slash = -1;
    for (int i = 0; i < slen; i++) if (s[i] == '/') { slash = i; break; }
    if (slash < 0) return 0;
    const char* addr = s;
    int alen = slash;
    const char* mask = s + slash + 1;
    int mlen = slen - slash - 1;
    int iplen = 4;
    go_ip ip;
    if (!go_parse_ipv4(addr, alen, &ip)) {
        iplen = 16;
        if (!go_parse_ipv6(addr, alen, &ip)) ip.len = 0;
    }
    int n, i;
    int ok = go_dtoi(mask, mlen, &n, &i);
    if (ip.len == 0 || !ok || i != mlen || n < 0 || n > 8 * iplen) return 0;
    uint8_t m[16];
    memset(m, 0, 16);
    go_cidr_mask(n, 8 * iplen, m);
    net->mlen = iplen;
    memcpy(net->m, m, 16);
    if (!go_ip_mask(&ip, m, iplen, &net->ip)) return 0;
    return 1;
}

/* IP.To4 (Go 1.9): 4-byte form or nil */
static int go_to4(const go_ip* ip, go_ip* out) {
    if (ip->len == 4) { *out = *ip; return 1; }
    if (ip->len == 16 && memcmp(ip->b, v4InV6Prefix, 12) == 0) {
        out->len = 4;
        memcpy(out->b, ip->b + 12, 4);
        return 1;
    }
    out->len = 0;
    return 0;
}

/* IPNet.Contains with networkNumberAndMask (Go 1.9 net/ip.go) */
static int go_contains(const go_ipnet* n, const go_ip* ip_in) {
    go_ip nn;
    const uint8_t* m = n->m;
    if (!go_to4(&n->ip, &nn)) {
        nn = n->ip;
        if (nn.len != 16) return 0;
    }
    switch (n->mlen) {
    case 4:
        if (nn.len != 4) return 0;
        break;
    case 16:
        if (nn.len == 4) m = n->m + 12;
        break;
    default:
        return 0;
    }
    go_ip ip = *ip_in, x;
    if (go_to4(&ip, &x)) ip = x;
    if (ip.len != nn.len) return 0;
    for (int i = 0; i < ip.len; i++)
        if ((nn.b[i] & m[i]) != (ip.b[i] & m[i])) return 0;
    return 1;
}

/* exported for tests: parse a CIDR; returns ok, network bytes and mask */
int orc_parse_cidr(const char* s, uint8_t ip_out[16], int* ip_len, uint8_t mask_out[16], int* mask_len) {
    go_ipnet n;
    if (!go_parse_cidr(s, &n)) return 0;
    memcpy(ip_out, n.ip.b, 16);
    *ip_len = n.ip.len;
    memcpy(mask_out, n.m, 16);
    *mask_len = n.mlen;
    return 1;
}

int orc_cidr_contains(const char* cidr, const uint8_t* ip, int ip_len) {
    go_ipnet n;
    if (!go_parse_cidr(cidr, &n)) return -1;
    go_ip x;
    x.len = ip_len;
    memcpy(x.b, ip, ip_len > 16 ? 16 : (ip_len < 0 ? 0 : ip_len));
    return go_contains(&n, &x);
}

/* ---------------------------------------------------------------------------
 * evalACL (aclengine_mock.go:473-668), literal form
 * ------------------------------------------------------------------------ */
#define MAX_PORT 65535u
#define MAX_ICMP_CODE 5u
#define MAX_ICMP_TYPE 16u

static int nonempty(const char* s) { return s && s[0]; }

static int action_verdict(const cls_rule* r) {
    if (!(r->flags & CLS_R_ACTIONS)) return CLS_ACL_FAILURE;              /* :646-650 */
    switch (r->acl_action) {                                              /* :655-664 */
    case CLS_ACTION_DENY: return CLS_ACL_DENY;
    case CLS_ACTION_PERMIT: return CLS_ACL_PERMIT;
    case CLS_ACTION_REFLECT: return CLS_ACL_REFLECT;
    default: return CLS_ACL_FAILURE;
    }
}

/* Returns ACLAction; *hit = index of the terminating rule, n if the default
 * DENY was reached, -1 if acl is nil.  Returns -2 if a rule would make Go
 * panic (Matches == nil). */
int orc_eval_acl(const cls_rule* rules, uint32_t n, int acl_nil,
                 const uint8_t* src, int src_len, const uint8_t* dst, int dst_len,
                 int proto, uint16_t dport, int32_t* hit) {
    if (acl_nil) { if (hit) *hit = -1; return CLS_ACL_PERMIT; }        /* :476-478 */
    go_ip sip, dip;
    sip.len = src_len; memcpy(sip.b, src, src_len);
    dip.len = dst_len; memcpy(dip.b, dst, dst_len);
    for (uint32_t k = 0; k < n; k++) {
        const cls_rule* r = &rules[k];
        if (hit) *hit = (int32_t)k;
        if (!(r->flags & CLS_R_MATCHES)) return -2;                       /* Go: nil deref */
        if (r->flags & CLS_R_MACIP) return CLS_ACL_FAILURE;              /* :481-485 */
        if (!(r->flags & CLS_R_IPRULE)) return CLS_ACL_FAILURE;          /* :486-490 */
        if ((r->flags & CLS_R_OTHER) || !(r->flags & CLS_R_IP))          /* :492-496 */
            return CLS_ACL_FAILURE;
        if (nonempty(r->src_network)) {                                   /* :499-510 */
            go_ipnet net;
            if (!go_parse_cidr(r->src_network, &net)) return CLS_ACL_FAILURE;
            if (!go_contains(&net, &sip)) continue;
        }
        if (nonempty(r->dst_network)) {                                   /* :513-524 */
            go_ipnet net;
            if (!go_parse_cidr(r->dst_network, &net)) return CLS_ACL_FAILURE;
            if (!go_contains(&net, &dip)) continue;
        }
        switch (proto) {                                                  /* :527-643 */
        case CLS_PROTO_TCP:
            if ((r->flags & CLS_R_UDP) || (r->flags & CLS_R_ICMP)) continue;
            if (!(r->flags & CLS_R_TCP)) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_TCP_SRC)) return CLS_ACL_FAILURE;
            if (r->tcp_src_lo != 0 || r->tcp_src_hi != MAX_PORT) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_TCP_DST)) return CLS_ACL_FAILURE;
            if (dport < (uint16_t)r->tcp_dst_lo || dport > (uint16_t)r->tcp_dst_hi) continue;
            break;
        case CLS_PROTO_UDP:
            if ((r->flags & CLS_R_TCP) || (r->flags & CLS_R_ICMP)) continue;
            if (!(r->flags & CLS_R_UDP)) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_UDP_SRC)) return CLS_ACL_FAILURE;
            if (r->udp_src_lo != 0 || r->udp_src_hi != MAX_PORT) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_UDP_DST)) return CLS_ACL_FAILURE;
            if (dport < (uint16_t)r->udp_dst_lo || dport > (uint16_t)r->udp_dst_hi) continue;
            break;
        case CLS_PROTO_ICMP:
            if ((r->flags & CLS_R_TCP) || (r->flags & CLS_R_UDP)) continue;
            if (!(r->flags & CLS_R_ICMP)) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_ICMP_CODE)) return CLS_ACL_FAILURE;
            if (r->icmp_code_first != 0 || r->icmp_code_last != MAX_ICMP_CODE) return CLS_ACL_FAILURE;
            if (!(r->flags & CLS_R_ICMP_TYPE)) return CLS_ACL_FAILURE;
            if (r->icmp_type_first != 0 || r->icmp_type_last != MAX_ICMP_TYPE) return CLS_ACL_FAILURE;
            if (r->flags & CLS_R_ICMPV6) return CLS_ACL_FAILURE;
            break;
        default:
            break;                                                        /* no case: fall through */
        }
        return action_verdict(r);                                         /* :645-664 */
    }
    if (hit) *hit = (int32_t)n;
    return CLS_ACL_DENY;                                                  /* :667 */
}

/* ---------------------------------------------------------------------------
 * testConnection (aclengine_mock.go:394-471).  Each ACL slot is (rules, n,
 * nil-flag).  same_if = (srcIfName == dstIfName).
 * ------------------------------------------------------------------------ */
typedef struct orc_acl_ref {
    const cls_rule* rules;
    uint32_t n;
    int nil;
} orc_acl_ref;

/* hits (may be NULL): the terminating rule of each evalACL call testConnection
 * makes, in call order -- [0] src inbound (SYN), [1] dst outbound (SYN),
 * [2] dst inbound (SYN-ACK), [3] src outbound (SYN-ACK); n of that ACL for the
 * default DENY, -1 for a call not made or made on a nil ACL.  These define
 * the connection path's per-(ACL, rule) hit counters (the reference has no
 * counters: parity unpinned, as for cls_classify's). */
int orc_test_connection_hits(const orc_acl_ref* src_in, const orc_acl_ref* src_out,
                             const orc_acl_ref* dst_in, const orc_acl_ref* dst_out, int same_if,
                             const uint8_t* src_ip, int src_len, const uint8_t* dst_ip, int dst_len,
                             int proto, uint16_t sport, uint16_t dport, int32_t* hits) {
    int src_refl = 0, dst_refl = 0, a;
    int32_t h[4] = {-1, -1, -1, -1};
#define ORC_RET(v) do { if (hits) memcpy(hits, h, sizeof h); return (v); } while (0)
    a = orc_eval_acl(src_in->rules, src_in->n, src_in->nil, src_ip, src_len, dst_ip, dst_len, proto, dport, &h[0]);
    if (a < 0) ORC_RET(a);
    if (a == CLS_ACL_FAILURE) ORC_RET(CLS_CONN_FAILURE);
    if (a == CLS_ACL_DENY) ORC_RET(CLS_CONN_DENY_SYN);
    if (a == CLS_ACL_REFLECT) { src_refl = 1; if (same_if) dst_refl = 1; }
    if (!dst_refl) {
        a = orc_eval_acl(dst_out->rules, dst_out->n, dst_out->nil, src_ip, src_len, dst_ip, dst_len, proto, dport, &h[1]);
        if (a < 0) ORC_RET(a);
        if (a == CLS_ACL_FAILURE) ORC_RET(CLS_CONN_FAILURE);
        if (a == CLS_ACL_DENY) ORC_RET(CLS_CONN_DENY_SYN);
        if (a == CLS_ACL_REFLECT) { dst_refl = 1; if (same_if) src_refl = 1; }
    }
    if (!dst_refl) {
        a = orc_eval_acl(dst_in->rules, dst_in->n, dst_in->nil, dst_ip, dst_len, src_ip, src_len, proto, sport, &h[2]);
        if (a < 0) ORC_RET(a);
        if (a == CLS_ACL_FAILURE) ORC_RET(CLS_CONN_FAILURE);
        if (a == CLS_ACL_DENY) ORC_RET(CLS_CONN_DENY_SYN_ACK);
    }
    if (!src_refl) {
        a = orc_eval_acl(src_out->rules, src_out->n, src_out->nil, dst_ip, dst_len, src_ip, src_len, proto, sport, &h[3]);
        if (a < 0) ORC_RET(a);
        if (a == CLS_ACL_FAILURE) ORC_RET(CLS_CONN_FAILURE);
        if (a == CLS_ACL_DENY) ORC_RET(CLS_CONN_DENY_SYN_ACK);
    }
    ORC_RET(CLS_CONN_ALLOW);
#undef ORC_RET
}

int orc_test_connection(const orc_acl_ref* src_in, const orc_acl_ref* src_out,
                        const orc_acl_ref* dst_in, const orc_acl_ref* dst_out, int same_if,
                        const uint8_t* src_ip, int src_len, const uint8_t* dst_ip, int dst_len,
                        int proto, uint16_t sport, uint16_t dport) {
    return orc_test_connection_hits(src_in, src_out, dst_in, dst_out, same_if, src_ip, src_len, dst_ip, dst_len,
                                    proto, sport, dport, NULL);
}

/* ---------------------------------------------------------------------------
 * Batched faithful evaluation (the "Go reference" stand-in baseline).
 * af = 4: src/dst are host-order uint32; af = 16: 16-byte network order.
 * ------------------------------------------------------------------------ */
static void load_ip(int af, const void* base, uint64_t i, uint8_t* b, int* len) {
    if (af == 4) {
        uint32_t v = ((const uint32_t*)base)[i];
        b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16);
        b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
        *len = 4;
    } else {
        memcpy(b, (const uint8_t*)base + 16 * i, 16);
        *len = 16;
    }
}

int orc_classify_faithful(const cls_rule* rules, uint32_t n_rules, int af,
                          const void* src, const void* dst, const uint16_t* dport,
                          const uint8_t* proto, uint64_t n, uint8_t* verdict,
                          uint64_t* counters /* n_rules+1 */) {
    for (uint64_t i = 0; i < n; i++) {
        uint8_t s[16], d[16];
        int sl, dl;
        int32_t hit;
        load_ip(af, src, i, s, &sl);
        load_ip(af, dst, i, d, &dl);
        int a = orc_eval_acl(rules, n_rules, 0, s, sl, d, dl, proto[i], dport[i], &hit);
        if (a < 0) return a;
        if (verdict) verdict[i] = (uint8_t)a;
        if (counters) counters[hit]++;
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * Fast CPU port: each rule pre-parsed once into a compact form, then the same
 * first-match loop, OpenMP across packets.  Semantics identical to
 * orc_eval_acl (tests check it against the faithful evaluator).
 * ------------------------------------------------------------------------ */
enum { PK_SKIP = 0, PK_TERM = 1 };
typedef struct {
    int uncond_fail;       /* steps 1-2 or src parse error: FAILURE when reached */
    int src_any, dst_any;
    int dst_fail;          /* dst parse error: FAILURE once src matched */
    go_ipnet src, dst;
    uint8_t kind[4];       /* TCP, UDP, ICMP, OTHER: PK_SKIP / PK_TERM */
    uint16_t lo[4], hi[4];
    uint8_t result[4];
} orc_crule;

struct orc_ctable {
    uint32_t n;
    orc_crule* r;
};
typedef struct orc_ctable orc_ctable;

static void crule_l4(const cls_rule* r, int proto, int res, orc_crule* c) {
    int p = proto;
    c->lo[p] = 0; c->hi[p] = 0xFFFF; c->kind[p] = PK_TERM;
    uint32_t f = r->flags;
    if (p == CLS_PROTO_TCP || p == CLS_PROTO_UDP) {
        uint32_t has = p == 0 ? CLS_R_TCP : CLS_R_UDP;
        uint32_t other1 = p == 0 ? CLS_R_UDP : CLS_R_TCP;
        uint32_t hsrc = p == 0 ? CLS_R_TCP_SRC : CLS_R_UDP_SRC;
        uint32_t hdst = p == 0 ? CLS_R_TCP_DST : CLS_R_UDP_DST;
        uint32_t slo = p == 0 ? r->tcp_src_lo : r->udp_src_lo;
        uint32_t shi = p == 0 ? r->tcp_src_hi : r->udp_src_hi;
        uint32_t dlo = p == 0 ? r->tcp_dst_lo : r->udp_dst_lo;
        uint32_t dhi = p == 0 ? r->tcp_dst_hi : r->udp_dst_hi;
        if ((f & other1) || (f & CLS_R_ICMP)) { c->kind[p] = PK_SKIP; return; }
        if (!(f & has) || !(f & hsrc) || slo != 0 || shi != MAX_PORT || !(f & hdst)) {
            c->result[p] = CLS_ACL_FAILURE; return;
        }
        uint16_t lo = (uint16_t)dlo, hi = (uint16_t)dhi;
        if (lo > hi) { c->kind[p] = PK_SKIP; return; }
        c->lo[p] = lo; c->hi[p] = hi; c->result[p] = (uint8_t)res;
    } else if (p == CLS_PROTO_ICMP) {
        if ((f & CLS_R_TCP) || (f & CLS_R_UDP)) { c->kind[p] = PK_SKIP; return; }
        if (!(f & CLS_R_ICMP) || !(f & CLS_R_ICMP_CODE) || r->icmp_code_first != 0 ||
            r->icmp_code_last != MAX_ICMP_CODE || !(f & CLS_R_ICMP_TYPE) ||
            r->icmp_type_first != 0 || r->icmp_type_last != MAX_ICMP_TYPE || (f & CLS_R_ICMPV6)) {
            c->result[p] = CLS_ACL_FAILURE; return;
        }
        c->result[p] = (uint8_t)res;
    } else {
        c->result[p] = (uint8_t)res;
    }
}

orc_ctable* orc_compile(const cls_rule* rules, uint32_t n) {
    orc_ctable* t = (orc_ctable*)calloc(1, sizeof(orc_ctable));
    t->n = n;
    t->r = (orc_crule*)calloc(n ? n : 1, sizeof(orc_crule));
    for (uint32_t k = 0; k < n; k++) {
        const cls_rule* r = &rules[k];
        orc_crule* c = &t->r[k];
        if (!(r->flags & CLS_R_MATCHES)) { free(t->r); free(t); return NULL; }
        if ((r->flags & CLS_R_MACIP) || !(r->flags & CLS_R_IPRULE) ||
            (r->flags & CLS_R_OTHER) || !(r->flags & CLS_R_IP)) { c->uncond_fail = 1; continue; }
        c->src_any = !nonempty(r->src_network);
        if (!c->src_any && !go_parse_cidr(r->src_network, &c->src)) { c->uncond_fail = 1; continue; }
        c->dst_any = !nonempty(r->dst_network);
        if (!c->dst_any && !go_parse_cidr(r->dst_network, &c->dst)) c->dst_fail = 1;
        int res = action_verdict(r);
        for (int p = 0; p < 4; p++) crule_l4(r, p, res, c);
    }
    return t;
}

void orc_ctable_free(orc_ctable* t) {
    if (!t) return;
    free(t->r);
    free(t);
}

static inline int fast_eval(const orc_ctable* t, const go_ip* s, const go_ip* d, int proto,
                            uint16_t dport, int32_t* hit) {
    int p = (proto >= 0 && proto <= 2) ? proto : 3;
    for (uint32_t k = 0; k < t->n; k++) {
        const orc_crule* c = &t->r[k];
        if (c->uncond_fail) { *hit = (int32_t)k; return CLS_ACL_FAILURE; }
        if (!c->src_any && !go_contains(&c->src, s)) continue;
        if (c->dst_fail) { *hit = (int32_t)k; return CLS_ACL_FAILURE; }
        if (!c->dst_any && !go_contains(&c->dst, d)) continue;
        if (c->kind[p] == PK_SKIP) continue;
        if (dport < c->lo[p] || dport > c->hi[p]) continue;
        *hit = (int32_t)k;
        return c->result[p];
    }
    *hit = (int32_t)t->n;
    return CLS_ACL_DENY;
}

int orc_classify_fast(const orc_ctable* t, int af, const void* src, const void* dst,
                      const uint16_t* dport, const uint8_t* proto, uint64_t n,
                      uint8_t* verdict, uint64_t* counters, int nthreads) {
    uint32_t nc = t->n + 1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
    nthreads = 1;
#endif
    uint64_t* priv = (uint64_t*)calloc((size_t)nthreads * nc, sizeof(uint64_t));
    if (!priv) return -1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        uint64_t* mine = priv + (size_t)tid * nc;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t i = 0; i < (int64_t)n; i++) {
            go_ip s, d;
            load_ip(af, src, (uint64_t)i, s.b, &s.len);
            load_ip(af, dst, (uint64_t)i, d.b, &d.len);
            int32_t hit;
            int a = fast_eval(t, &s, &d, proto[i], dport[i], &hit);
            if (verdict) verdict[i] = (uint8_t)a;
            mine[hit]++;
        }
    }
    if (counters)
        for (int th = 0; th < nthreads; th++)
            for (uint32_t k = 0; k < nc; k++) counters[k] += priv[(size_t)th * nc + k];
    free(priv);
    return 0;
}

/* Each packet's ACLAction and terminating rule index (n: the default DENY),
 * as orc_eval_acl's *hit: the checker of cls_classify_rules. */
int orc_classify_fast_hits(const orc_ctable* t, int af, const void* src, const void* dst,
                           const uint16_t* dport, const uint8_t* proto, uint64_t n,
                           uint8_t* verdict, uint32_t* hits, int nthreads) {
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#else
    (void)nthreads;
#endif
    for (int64_t i = 0; i < (int64_t)n; i++) {
        go_ip s, d;
        load_ip(af, src, (uint64_t)i, s.b, &s.len);
        load_ip(af, dst, (uint64_t)i, d.b, &d.len);
        int32_t hit;
        int a = fast_eval(t, &s, &d, proto[i], dport[i], &hit);
        if (verdict) verdict[i] = (uint8_t)a;
        hits[i] = (uint32_t)hit;
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * Fast CPU port of a batch of testConnection calls (the connection line's
 * CPU baseline): the ACLs pre-parsed (orc_compile), testConnection's order
 * and REFLECT short-cuts exactly as orc_test_connection_hits (itself
 * aclengine_mock.go:394-471), OpenMP across connections.  Interface f binds
 * table if_in[f] inbound and if_out[f] outbound (-1: no ACL, evalACL's nil
 * ACL: PERMIT); connection i enters on si[i] and leaves on di[i].
 * ------------------------------------------------------------------------ */
static inline int fast_call(const orc_ctable* const* tabs, int32_t t, const go_ip* s, const go_ip* d, int proto,
                            uint16_t port) {
    int32_t hit;
    if (t < 0) return CLS_ACL_PERMIT;
    return fast_eval(tabs[t], s, d, proto, port, &hit);
}

int orc_connect_fast(const orc_ctable* const* tabs, const int32_t* if_in, const int32_t* if_out, uint32_t n_ifs,
                     const uint32_t* si, const uint32_t* di, int af, const void* src, const void* dst,
                     const uint8_t* proto, const uint16_t* sport, const uint16_t* dport, uint64_t n,
                     uint8_t* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const uint32_t a = si[i], b = di[i];
        if (a >= n_ifs || b >= n_ifs) { out[i] = CLS_CONN_FAILURE; continue; }
        go_ip s, d;
        load_ip(af, src, (uint64_t)i, s.b, &s.len);
        load_ip(af, dst, (uint64_t)i, d.b, &d.len);
        const int same = a == b, p = proto[i];
        int src_refl = 0, dst_refl = 0, r;
        uint8_t v = CLS_CONN_ALLOW;
        r = fast_call(tabs, if_in[a], &s, &d, p, dport[i]);                     /* SYN: src inbound */
        if (r == CLS_ACL_FAILURE) { out[i] = CLS_CONN_FAILURE; continue; }
        if (r == CLS_ACL_DENY) { out[i] = CLS_CONN_DENY_SYN; continue; }
        if (r == CLS_ACL_REFLECT) { src_refl = 1; if (same) dst_refl = 1; }
        if (!dst_refl) {                                                         /* SYN: dst outbound */
            r = fast_call(tabs, if_out[b], &s, &d, p, dport[i]);
            if (r == CLS_ACL_FAILURE) { out[i] = CLS_CONN_FAILURE; continue; }
            if (r == CLS_ACL_DENY) { out[i] = CLS_CONN_DENY_SYN; continue; }
            if (r == CLS_ACL_REFLECT) { dst_refl = 1; if (same) src_refl = 1; }
        }
        if (!dst_refl) {                                                         /* SYN-ACK: dst inbound */
            r = fast_call(tabs, if_in[b], &d, &s, p, sport[i]);
            if (r == CLS_ACL_FAILURE) { out[i] = CLS_CONN_FAILURE; continue; }
            if (r == CLS_ACL_DENY) { out[i] = CLS_CONN_DENY_SYN_ACK; continue; }
        }
        if (!src_refl) {                                                         /* SYN-ACK: src outbound */
            r = fast_call(tabs, if_out[a], &d, &s, p, sport[i]);
            if (r == CLS_ACL_FAILURE) { out[i] = CLS_CONN_FAILURE; continue; }
            if (r == CLS_ACL_DENY) { out[i] = CLS_CONN_DENY_SYN_ACK; continue; }
        }
        out[i] = v;
    }
    return 0;
}

/* ---------------------------------------------------------------------------
 * Synthetic traffic generator (definition in DESIGN.md "Traffic"), identical
 * to the device generator in the product.  Used to check the device stream.
 * ------------------------------------------------------------------------ */
#define GOLDEN 0x9E3779B97F4A7C15ull
static inline uint64_t mix64(uint64_t z) {
    z += GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_gen_traffic_v4(const cls_traffic_spec* sp, uint64_t first, uint64_t n,
                        uint32_t* src4, uint32_t* dst4, uint16_t* sport, uint16_t* dport,
                        uint8_t* proto) {
    for (uint64_t k = 0; k < n; k++) {
        uint64_t i = first + k;
        uint64_t w[6];
        for (int j = 0; j < 6; j++) w[j] = mix64(sp->seed ^ ((8 * i + (uint64_t)j) * GOLDEN));
        uint32_t a0 = (uint32_t)w[0], b0 = (uint32_t)(w[0] >> 32);
        uint8_t pr;
        if (a0 % 100u < sp->pct_icmp) pr = CLS_PROTO_ICMP;
        else pr = (b0 & 1u) ? CLS_PROTO_UDP : CLS_PROTO_TCP;
        uint32_t s;
        if (sp->n_pod_ips && ((b0 >> 1) % 100u) < sp->pct_pod_src)
            s = sp->pod_ips[(uint32_t)(w[1] >> 32) % sp->n_pod_ips];
        else
            s = (uint32_t)w[1];
        uint32_t a2 = (uint32_t)w[2], b2 = (uint32_t)(w[2] >> 32);
        uint32_t d;
        if (sp->n_dst && (a2 % 100u) < sp->pct_rule_dst) {
            uint32_t j = b2 % sp->n_dst;
            uint32_t len = sp->dst_lens[j];
            uint32_t mask = len ? (0xFFFFFFFFu << (32 - len)) : 0u;
            d = (sp->dst_addrs[j] & mask) | ((uint32_t)w[3] & ~mask);
        } else {
            d = (uint32_t)w[3];
        }
        uint32_t a4 = (uint32_t)w[4], b4 = (uint32_t)(w[4] >> 32);
        uint16_t dp;
        if (sp->n_ports && (a4 % 100u) < sp->pct_table_port) dp = sp->ports[b4 % sp->n_ports];
        else dp = (uint16_t)w[5];
        uint16_t spt = (uint16_t)(1024u + ((uint32_t)(w[5] >> 32) % 64512u));
        if (src4) src4[k] = s;
        if (dst4) dst4[k] = d;
        if (sport) sport[k] = spt;
        if (dport) dport[k] = dp;
        if (proto) proto[k] = pr;
    }
}

/* The 16-byte stream (include/contivcls.h cls_traffic_spec16): addresses as
 * (hi, lo) u64 in address order, written as 16 network-order bytes. */
static void put16(uint8_t* b, uint64_t hi, uint64_t lo) {
    for (int k = 0; k < 8; k++) {
        b[k] = (uint8_t)(hi >> (56 - 8 * k));
        b[8 + k] = (uint8_t)(lo >> (56 - 8 * k));
    }
}
static void get16(const uint8_t* b, uint64_t* hi, uint64_t* lo) {
    *hi = *lo = 0;
    for (int k = 0; k < 8; k++) {
        *hi = (*hi << 8) | b[k];
        *lo = (*lo << 8) | b[8 + k];
    }
}

void orc_gen_traffic_v16(const cls_traffic_spec16* sp, uint64_t first, uint64_t n,
                         uint8_t* src16, uint8_t* dst16, uint16_t* sport, uint16_t* dport,
                         uint8_t* proto) {
    const uint64_t fd00 = 0xFD00ull << 48, mapped = 0xFFFFull << 32;
    for (uint64_t k = 0; k < n; k++) {
        uint64_t i = first + k;
        uint64_t w[8];
        for (int j = 0; j < 8; j++) w[j] = mix64(sp->seed ^ ((8 * i + (uint64_t)j) * GOLDEN));
        uint32_t a0 = (uint32_t)w[0], b0 = (uint32_t)(w[0] >> 32);
        uint8_t pr;
        if (a0 % 100u < sp->pct_icmp) pr = CLS_PROTO_ICMP;
        else pr = (b0 & 1u) ? CLS_PROTO_UDP : CLS_PROTO_TCP;
        uint64_t sh, sl;
        uint32_t b1 = (uint32_t)(w[1] >> 32);
        if (sp->n_pod_ips && ((b0 >> 1) % 100u) < sp->pct_pod_src)
            get16(sp->pod_ips + 16 * (size_t)(b1 % sp->n_pod_ips), &sh, &sl);
        else if (b1 & 1u) { sh = fd00; sl = w[6]; }
        else { sh = 0; sl = mapped | (uint32_t)w[1]; }
        uint32_t a2 = (uint32_t)w[2], b2 = (uint32_t)(w[2] >> 32);
        uint64_t dh, dl;
        if (sp->n_dst && (a2 % 100u) < sp->pct_rule_dst) {
            uint32_t j = b2 % sp->n_dst;
            uint32_t len = sp->dst_lens[j];
            uint64_t mh = len == 0 ? 0 : len >= 64 ? ~0ull : ~0ull << (64 - len);
            uint64_t ml = len <= 64 ? 0 : len >= 128 ? ~0ull : ~0ull << (128 - len);
            uint64_t ph, pl;
            get16(sp->dst_addrs + 16 * (size_t)j, &ph, &pl);
            dh = (ph & mh) | (w[3] & ~mh);
            dl = (pl & ml) | (w[7] & ~ml);
        } else if (b2 & 1u) { dh = fd00; dl = w[7]; }
        else { dh = 0; dl = mapped | (uint32_t)w[3]; }
        uint32_t a4 = (uint32_t)w[4], b4 = (uint32_t)(w[4] >> 32);
        uint16_t dp;
        if (sp->n_ports && (a4 % 100u) < sp->pct_table_port) dp = sp->ports[b4 % sp->n_ports];
        else dp = (uint16_t)w[5];
        uint16_t spt = (uint16_t)(1024u + ((uint32_t)(w[5] >> 32) % 64512u));
        if (src16) put16(src16 + 16 * k, sh, sl);
        if (dst16) put16(dst16 + 16 * k, dh, dl);
        if (sport) sport[k] = spt;
        if (dport) dport[k] = dp;
        if (proto) proto[k] = pr;
    }
}
