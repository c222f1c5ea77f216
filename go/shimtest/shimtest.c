/*
 * shimtest -- the Go binding's C shims (include/contivcls_go.h) driven the
 * way go/contivcls/contivcls.go drives them, from plain C (gcc): the image
 * has no Go toolchain, so this program stands in for the cgo calls and
 * tests/test_gpu_go_shims.py checks its outputs against the oracle.
 *
 * usage: shimtest DIR
 *   DIR/acls.txt   "acl NAME N_RULES N_IN IF... N_OUT IF..." lines, each followed
 *                  by N_RULES "rule FLAGS ACTION TSL TSH TDL TDH USL USH UDL UDH
 *                  ICF ICL ITF ITL SRC DST" lines (networks "-" for none, else "x"
 *                  and the string's bytes in hex); the first
 *                  ACL's table is the one classified
 *   DIR/ifs.txt    interface names, one per line (connection index -> name)
 *   DIR/pkt.bin    u64 n, then src4[n] dst4[n] (u32) dport[n] (u16) proto[n] (u8)
 *   DIR/conn.bin   u64 m, then si[m] di[m] (u32 indices into ifs.txt) src4[m]
 *                  dst4[m] (u32) sport[m] dport[m] (u16) proto[m] (u8)
 * writes DIR/out_*.bin: verdicts and counters of clsg_classify_v4 (and the
 * verdicts and terminating rules of clsg_classify_rules_v4), of
 * clsg_classify_v16 (the same packets IPv4-mapped), of an engine-owned batch
 * filled through its pinned mirror (clsg_batch_mirror, cls_batch_upload,
 * cls_classify_batch, cls_batch_download), the ConnectionActions of
 * clsg_connect_v4 (CLS_F_COUNT) and each ACL's connection counters.
 */
#define _POSIX_C_SOURCE 200809L   /* strdup */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "contivcls_go.h"

#define MAX_ACLS 256
#define MAX_IFS 1024

static char dir[4096];

static void die(const char* what, cls_engine* e, int rc) {
    fprintf(stderr, "shimtest: %s failed (rc %d): %s\n", what, rc, e ? cls_last_error(e) : "");
    exit(1);
}

static FILE* open_in(const char* name, const char* mode) {
    char p[4200];
    snprintf(p, sizeof p, "%s/%s", dir, name);
    FILE* f = fopen(p, mode);
    if (!f) {
        fprintf(stderr, "shimtest: cannot open %s\n", p);
        exit(1);
    }
    return f;
}

static void* read_n(FILE* f, size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p || (bytes && fread(p, 1, bytes, f) != bytes)) {
        fprintf(stderr, "shimtest: short input\n");
        exit(1);
    }
    return p;
}

static void write_out(const char* name, const void* p, size_t bytes) {
    FILE* f = open_in(name, "wb");
    if (bytes && fwrite(p, 1, bytes, f) != bytes) exit(1);
    fclose(f);
}

/* a network string: "-" (none) or "x" and its bytes in hex */
static char* dup_net(const char* s) {
    if (strcmp(s, "-") == 0) return NULL;
    const size_t n = strlen(s + 1) / 2;
    char* out = calloc(n + 1, 1);
    for (size_t i = 0; i < n; ++i) {
        unsigned v = 0;
        if (sscanf(s + 1 + 2 * i, "%2x", &v) != 1) exit(1);
        out[i] = (char)v;
    }
    return out;
}

struct acl {
    char name[128];
    uint32_t n_rules;
    cls_rule* rules;
    char* in[16];
    char* out[16];
    uint32_t n_in, n_out;
};

int main(int argc, char** argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: shimtest DIR\n");
        return 2;
    }
    snprintf(dir, sizeof dir, "%s", argv[1]);
    if (cls_abi_version() != clsg_abi_version()) {
        fprintf(stderr, "shimtest: library ABI %d, shims %d\n", cls_abi_version(), clsg_abi_version());
        return 1;
    }
    /* ---- ACLs -------------------------------------------------------------- */
    static struct acl acls[MAX_ACLS];
    uint32_t n_acls = 0;
    FILE* f = open_in("acls.txt", "r");
    char tag[16];
    while (fscanf(f, "%15s", tag) == 1) {
        if (strcmp(tag, "acl") != 0 || n_acls == MAX_ACLS) return 1;
        struct acl* a = &acls[n_acls++];
        char buf[256];
        if (fscanf(f, "%127s %u %u", a->name, &a->n_rules, &a->n_in) != 3 || a->n_in > 16) return 1;
        for (uint32_t i = 0; i < a->n_in; ++i) {
            if (fscanf(f, "%255s", buf) != 1) return 1;
            a->in[i] = strdup(buf);
        }
        if (fscanf(f, "%u", &a->n_out) != 1 || a->n_out > 16) return 1;
        for (uint32_t i = 0; i < a->n_out; ++i) {
            if (fscanf(f, "%255s", buf) != 1) return 1;
            a->out[i] = strdup(buf);
        }
        a->rules = calloc(a->n_rules ? a->n_rules : 1, sizeof(cls_rule));
        for (uint32_t k = 0; k < a->n_rules; ++k) {
            cls_rule* r = &a->rules[k];
            char src[256], dst[256];
            if (fscanf(f, "%15s %u %d %u %u %u %u %u %u %u %u %u %u %u %u %255s %255s", tag, &r->flags,
                       &r->acl_action, &r->tcp_src_lo, &r->tcp_src_hi, &r->tcp_dst_lo, &r->tcp_dst_hi, &r->udp_src_lo,
                       &r->udp_src_hi, &r->udp_dst_lo, &r->udp_dst_hi, &r->icmp_code_first, &r->icmp_code_last,
                       &r->icmp_type_first, &r->icmp_type_last, src, dst) != 17)
                return 1;
            r->src_network = dup_net(src);
            r->dst_network = dup_net(dst);
        }
    }
    fclose(f);
    if (n_acls == 0) return 1;

    int devs[1] = {0};
    cls_engine* e = NULL;
    int rc = clsg_engine_create(devs, 1, &e);
    if (rc != CLS_OK) die("clsg_engine_create", NULL, rc);
    for (uint32_t k = 0; k < n_acls; ++k) {
        struct acl* a = &acls[k];
        rc = cls_acl_put(e, a->name, a->rules, a->n_rules, (const char* const*)a->in, a->n_in,
                         (const char* const*)a->out, a->n_out);
        if (rc != CLS_OK) die("cls_acl_put", e, rc);
    }
    uint32_t tid = 0;
    if ((rc = cls_acl_table(e, acls[0].name, &tid)) != CLS_OK) die("cls_acl_table", e, rc);
    const uint32_t R = acls[0].n_rules;

    /* ---- packets: the classify shims ------------------------------------- */
    f = open_in("pkt.bin", "rb");
    uint64_t n = 0;
    if (fread(&n, 8, 1, f) != 1) return 1;
    uint32_t* src = read_n(f, n * 4);
    uint32_t* dst = read_n(f, n * 4);
    uint16_t* dport = read_n(f, n * 2);
    uint8_t* proto = read_n(f, n);
    fclose(f);
    uint8_t* verdict = malloc(n ? n : 1);
    uint64_t* ctr = calloc(R + 1, 8);
    rc = clsg_classify_v4(e, tid, src, dst, dport, proto, n, verdict, ctr, 0);
    if (rc != CLS_OK) die("clsg_classify_v4", e, rc);
    write_out("out_verdict.bin", verdict, n);
    write_out("out_counters.bin", ctr, (R + 1) * 8);
    /* each packet's terminating rule (clsg_classify_rules_v4) */
    uint32_t* rules = malloc(n ? 4 * n : 4);
    rc = clsg_classify_rules_v4(e, tid, src, dst, dport, proto, n, verdict, rules);
    if (rc != CLS_OK) die("clsg_classify_rules_v4", e, rc);
    write_out("out_rverdict.bin", verdict, n);
    write_out("out_rules.bin", rules, 4 * n);
    free(rules);

    /* the same packets as IPv4-mapped 16-byte addresses (Go's To16) */
    uint8_t* s16 = calloc(n ? n : 1, 16);
    uint8_t* d16 = calloc(n ? n : 1, 16);
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t* a = s16 + 16 * i;
        uint8_t* b = d16 + 16 * i;
        a[10] = a[11] = b[10] = b[11] = 0xFF;
        for (int j = 0; j < 4; ++j) {
            a[12 + j] = (uint8_t)(src[i] >> (24 - 8 * j));
            b[12 + j] = (uint8_t)(dst[i] >> (24 - 8 * j));
        }
    }
    memset(ctr, 0, (R + 1) * 8);
    rc = clsg_classify_v16(e, tid, s16, d16, dport, proto, n, verdict, ctr, 0);
    if (rc != CLS_OK) die("clsg_classify_v16", e, rc);
    write_out("out_verdict16.bin", verdict, n);
    write_out("out_counters16.bin", ctr, (R + 1) * 8);

    /* an engine-owned batch, filled in place through its pinned mirror */
    cls_batch* b = NULL;
    if ((rc = cls_batch_create(e, CLS_AF_V4, n, CLS_BATCH_MIRROR, &b)) != CLS_OK) die("cls_batch_create", e, rc);
    const struct {
        uint32_t field;
        const void* src;
        size_t elem;
    } fill[4] = {{CLS_BF_SRC, src, 4}, {CLS_BF_DST, dst, 4}, {CLS_BF_DPORT, dport, 2}, {CLS_BF_PROTO, proto, 1}};
    for (int k = 0; k < 4; ++k) {
        void* m = clsg_batch_mirror(b, fill[k].field);
        if (!m) die("clsg_batch_mirror", e, -1);
        memcpy(m, fill[k].src, n * fill[k].elem);
        if ((rc = cls_batch_upload(b, fill[k].field, 0, n, NULL)) != CLS_OK) die("cls_batch_upload", e, rc);
    }
    memset(ctr, 0, (R + 1) * 8);
    if ((rc = cls_classify_batch(e, tid, b, ctr, 0)) != CLS_OK) die("cls_classify_batch", e, rc);
    memset(verdict, 0xEE, n);
    if ((rc = cls_batch_download(b, CLS_BF_VERDICT, 0, n, verdict)) != CLS_OK) die("cls_batch_download", e, rc);
    write_out("out_bverdict.bin", verdict, n);
    write_out("out_bcounters.bin", ctr, (R + 1) * 8);
    cls_batch_destroy(b);

    /* ---- connections: the connect shim ------------------------------------ */
    static char* ifn[MAX_IFS];
    uint32_t n_ifs = 0;
    f = open_in("ifs.txt", "r");
    char buf[256];
    while (n_ifs < MAX_IFS && fscanf(f, "%255s", buf) == 1) ifn[n_ifs++] = strdup(buf);
    fclose(f);
    uint32_t ids[MAX_IFS];
    for (uint32_t k = 0; k < n_ifs; ++k)
        if ((rc = cls_if_id(e, ifn[k], &ids[k])) != CLS_OK) die("cls_if_id", e, rc);
    f = open_in("conn.bin", "rb");
    uint64_t m = 0;
    if (fread(&m, 8, 1, f) != 1) return 1;
    uint32_t* si = read_n(f, m * 4);
    uint32_t* di = read_n(f, m * 4);
    uint32_t* cs = read_n(f, m * 4);
    uint32_t* cd = read_n(f, m * 4);
    uint16_t* csp = read_n(f, m * 2);
    uint16_t* cdp = read_n(f, m * 2);
    uint8_t* cpr = read_n(f, m);
    fclose(f);
    for (uint64_t i = 0; i < m; ++i) {
        if (si[i] >= n_ifs || di[i] >= n_ifs) return 1;
        si[i] = ids[si[i]];
        di[i] = ids[di[i]];
    }
    uint8_t* act = malloc(m ? m : 1);
    rc = clsg_connect_v4(e, si, di, cs, cd, csp, cdp, cpr, m, act, CLS_F_COUNT);
    if (rc != CLS_OK) die("clsg_connect_v4", e, rc);
    write_out("out_conn.bin", act, m);
    for (uint32_t k = 0; k < n_acls; ++k) {
        uint32_t t = 0;
        if ((rc = cls_acl_table(e, acls[k].name, &t)) != CLS_OK) die("cls_acl_table", e, rc);
        uint64_t* cc = calloc(acls[k].n_rules + 1, 8);
        if ((rc = cls_conn_counters(e, t, cc, 0)) != CLS_OK) die("cls_conn_counters", e, rc);
        char name[200];
        snprintf(name, sizeof name, "out_conn_ctr_%u.bin", k);
        write_out(name, cc, (acls[k].n_rules + 1) * 8);
        free(cc);
    }
    cls_engine_destroy(e);
    printf("shimtest: %llu packets, %llu connections, %u ACLs\n", (unsigned long long)n, (unsigned long long)m,
           n_acls);
    return 0;
}
