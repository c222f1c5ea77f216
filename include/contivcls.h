/*
 * contivcls.h -- C ABI of the MI355X batched first-match ACL classifier.
 *
 * This is the drop-in boundary for the Contiv-VPP policy verdict backend.
 * In the reference the verdict backend is the Go test engine
 * mock/aclengine/aclengine_mock.go (MockACLEngine); in production it is VPP's
 * acl-plugin (external C binary, not in the reference tree).  Every entry
 * point below names the reference interface it replaces (file:line relative to
 * the reference root).  A Go (cgo) binding of these entry points is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *  - All functions return 0 (CLS_OK) or a negative CLS_E_* code; the detail is
 *    available from cls_last_error().  Per-packet semantic failures are
 *    VERDICTS (CLS_ACL_FAILURE / CLS_CONN_FAILURE), never error codes.
 *  - The caller owns every buffer.  The engine retains no caller pointer after
 *    a call returns (cgo rule); rule tables are deep-copied by cls_table_put.
 *  - Enum values keep the reference's numeric values.
 *  - IPv4 addresses in the 4-byte SoA are host-order uint32 (a.b.c.d =
 *    a<<24|b<<16|c<<8|d).  16-byte addresses are network-order bytes; an
 *    IPv4-mapped address (::ffff:a.b.c.d) is an IPv4 packet, exactly like Go's
 *    net.IP.To4().
 */
#ifndef CONTIVCLS_H
#define CONTIVCLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: cls_image_v4_header gained n_lctr, ctr16, swap (a destination-keyed
 *    image: the packets' src and dst must be exchanged) and off_other (a
 *    nested OTHER image); blob version 3; cls_table_info's n_lctr, ctr16,
 *    list_mode and swap; CLS_F_COUNT; CLS_AF_V16 connections;
 *    cls_acl_stats.  A v1 consumer that ignores `swap` would misread blobs. */
/* 4: cls_config's device list (multi-device engines); engine-owned batches
 *    (cls_batch_*); cls_classify_batch / cls_batch_connect; the in-library
 *    RCCL counter all-reduce (cls_comm_*); cls_shard_range. */
/* 5: cls_engine_set_option (tuning / diagnostic switches; the library no
 *    longer reads the process environment); cls_compile_v4 / v16 take an
 *    option string; entry points restore the caller's current device; over
 *    distinct devices an engine without RCCL keeps host-summed counters;
 *    cls_classify_rules (the per-packet matched-rule trace); CLS_F_DEVICE
 *    connection batches are stream-ordered. */
#define CLS_ABI_VERSION 5

/* ---- status codes ------------------------------------------------------ */
enum {
    CLS_OK = 0,
    CLS_E_INVAL = -1,    /* bad argument / malformed rule (would panic in Go) */
    CLS_E_NOMEM = -2,
    CLS_E_HIP = -3,      /* HIP runtime error */
    CLS_E_RCCL = -4,     /* RCCL (the counter all-reduce) unavailable or failed */
    CLS_E_NOTFOUND = -5, /* unknown table / ACL name */
    CLS_E_NODEV = -6     /* no usable gfx950 device */
};

/* ---- reference enums ----------------------------------------------------- */
/* vpp_acl.AclAction (acl.proto:4-8); any other int32 is carried verbatim. */
enum { CLS_ACTION_DENY = 0, CLS_ACTION_PERMIT = 1, CLS_ACTION_REFLECT = 2 };

/* ACLAction returned by evalACL (aclengine_mock.go:63-77). */
enum {
    CLS_ACL_DENY = 0,
    CLS_ACL_PERMIT = 1,
    CLS_ACL_REFLECT = 2,
    CLS_ACL_FAILURE = 3
};

/* ConnectionAction returned by Connection* (aclengine_mock.go:46-60). */
enum {
    CLS_CONN_DENY_SYN = 0,
    CLS_CONN_DENY_SYN_ACK = 1,
    CLS_CONN_ALLOW = 2,
    CLS_CONN_FAILURE = 3
};

/* ProtocolType (aclengine_mock.go:80-91).  Any other value takes evalACL's
 * `switch protocol` fall-through (no case): networks alone decide. */
enum { CLS_PROTO_TCP = 0, CLS_PROTO_UDP = 1, CLS_PROTO_ICMP = 2 };

/* ---- one ACL rule, as the vpp_acl protobuf carries it --------------------
 * Mirrors AccessLists_Acl_Rule (acl.pb.go / acl.proto:17-146).  Presence bits
 * stand for the nil-ness of each protobuf sub-message, because evalACL's
 * semantics depend on it (aclengine_mock.go:481-664).  Networks are the CIDR
 * STRINGS of the protobuf; the engine parses them with Go 1.9 net.ParseCIDR
 * semantics, so a string that fails to parse yields the same FAILURE verdicts
 * the Go engine returns.  NULL or "" means "no network" (match all).
 */
enum {
    CLS_R_MATCHES = 1u << 0,     /* rule.Matches != nil (nil would panic: rejected) */
    CLS_R_MACIP = 1u << 1,       /* Matches.MacipRule != nil */
    CLS_R_IPRULE = 1u << 2,      /* Matches.IpRule != nil */
    CLS_R_IP = 1u << 3,          /* IpRule.Ip != nil */
    CLS_R_OTHER = 1u << 4,       /* IpRule.Other != nil */
    CLS_R_TCP = 1u << 5,         /* IpRule.Tcp != nil */
    CLS_R_TCP_SRC = 1u << 6,     /* Tcp.SourcePortRange != nil */
    CLS_R_TCP_DST = 1u << 7,     /* Tcp.DestinationPortRange != nil */
    CLS_R_UDP = 1u << 8,         /* IpRule.Udp != nil */
    CLS_R_UDP_SRC = 1u << 9,
    CLS_R_UDP_DST = 1u << 10,
    CLS_R_ICMP = 1u << 11,       /* IpRule.Icmp != nil */
    CLS_R_ICMP_CODE = 1u << 12,  /* Icmp.IcmpCodeRange != nil */
    CLS_R_ICMP_TYPE = 1u << 13,  /* Icmp.IcmpTypeRange != nil */
    CLS_R_ICMPV6 = 1u << 14,     /* Icmp.Icmpv6 == true */
    CLS_R_ACTIONS = 1u << 15     /* rule.Actions != nil */
};

typedef struct cls_rule {
    uint32_t flags;             /* CLS_R_* */
    int32_t acl_action;         /* Actions.AclAction (vpp_acl.AclAction) */
    const char* src_network;    /* IpRule.Ip.SourceNetwork */
    const char* dst_network;    /* IpRule.Ip.DestinationNetwork */
    uint32_t tcp_src_lo, tcp_src_hi, tcp_dst_lo, tcp_dst_hi;
    uint32_t udp_src_lo, udp_src_hi, udp_dst_lo, udp_dst_hi;
    uint32_t icmp_code_first, icmp_code_last, icmp_type_first, icmp_type_last;
} cls_rule;

/* ---- packet batches (structure of arrays) -------------------------------- */
enum { CLS_AF_V4 = 4, CLS_AF_V16 = 16 };

typedef struct cls_pkt_soa {
    uint32_t af;               /* CLS_AF_V4: src4/dst4; CLS_AF_V16: src16/dst16 */
    const uint32_t* src4;      /* host-order IPv4 */
    const uint32_t* dst4;
    const uint8_t* src16;      /* n x 16 bytes */
    const uint8_t* dst16;
    const uint16_t* sport;     /* used by the connection path only (SYN-ACK) */
    const uint16_t* dport;
    const uint8_t* proto;      /* ProtocolType */
} cls_pkt_soa;

/* cls_classify / cls_connect_batch flags */
enum {
    CLS_F_DEVICE = 1u << 0,       /* every pointer is device memory on this engine's GPU */
    CLS_F_NO_VERDICT = 1u << 1,   /* verdict_out may be NULL (counters only) */
    CLS_F_ACCUMULATE = 1u << 2,   /* add to counters_out instead of overwriting */
    CLS_F_FORCE_LINEAR = 1u << 3, /* use the linear (ballot) kernel: GPU cross-check */
    CLS_F_TIMING = 1u << 4,       /* record HIP events around the classify kernel */
    CLS_F_CONN_CLS = 1u << 5,     /* cls_connect_batch: use the classifier images at any batch size */
    CLS_F_COUNT = 1u << 6         /* cls_connect_batch: count every evalACL call's terminating rule
                                     into the tables' connection counters (cls_conn_counters) */
};

typedef struct cls_engine cls_engine;

/* An engine over one device (n_devices = 0: `device`) or over several
 * (n_devices > 0: devices[0 .. n_devices), `device` ignored).
 * A multi-device engine keeps one ACL configuration: every table is compiled
 * once and uploaded to every device (replicated), and batches (cls_batch_*)
 * shard contiguously over the devices.  Calls that take raw packet pointers
 * (cls_classify, cls_connect_batch, cls_gen_traffic_*) run on the first
 * device.  Over distinct devices the engine creates an RCCL communicator
 * (single-process ncclCommInitAll) at creation, so batch hit counters merge
 * with an all-reduce over xGMI; a list that repeats a device (diagnostics:
 * shards on one GPU), or a host where RCCL cannot be loaded or initialised,
 * has no communicator and its counters are summed on the host when read
 * (cls_comm_info reports 0 ranks; cls_last_error keeps the RCCL reason). */
typedef struct cls_config {
    int device;                /* HIP device ordinal; -1 = current device */
    uint32_t n_devices;        /* 0: one device (`device`); else the length of `devices` */
    const int* devices;        /* HIP device ordinals (n_devices of them) */
    uint32_t reserved[4];
} cls_config;

/* ---- engine lifetime ---------------------------------------------------- */
/* Replaces NewMockACLEngine (aclengine_mock.go:124).  Destroy batches
 * (cls_batch_destroy) before their engine. */
int cls_engine_create(const cls_config* cfg, cls_engine** out);
void cls_engine_destroy(cls_engine* e);
/* Devices of the engine (1 for a single-device engine). */
int cls_engine_devices(const cls_engine* e, uint32_t* n_devices);
/* The engine of device `index` of a multi-device engine (0: `e` itself):
 * a borrowed handle for the single-device calls on that device (timing,
 * stream floors, raw device pointers of that device); configuration calls on
 * it are refused (configure through `e`). */
int cls_device_engine(cls_engine* e, uint32_t index, cls_engine** dev);
const char* cls_last_error(const cls_engine* e);
int cls_abi_version(void);
/* Diagnostics, tests and measurements: one tuning switch of the engine (and
 * of every device of a multi-device engine), `value` NULL for its default.
 * The switches force compiler choices (list_mode, list_mode_max, trie, wide,
 * orient=src|dst, lds_budget, src_search, phash_dense, v16_src_search,
 * v16_src_trie) for later cls_table_put / cls_acl_put compiles, and launch
 * plans (other_cap, wg_per_cu, conn_bitmap, conn_pair, conn_pre_rules,
 * conn_pre_narrow, pair_qcap, pair_lq, pair_other_global, conn_no_lds,
 * conn_jobs, conn_plan=32j|16j|32s|16s, conn_flush_atomic, batch_layout,
 * debug_modes, debug_conn, debug_floor) for later calls; every one keeps
 * verdicts and counters exact.  The library never reads the environment:
 * an engine runs its defaults unless told otherwise here.  CLS_E_INVAL for
 * an unknown key or a malformed value. */
int cls_engine_set_option(cls_engine* e, const char* key, const char* value);

/* ---- rule tables (one compiled, device-resident ACL) -------------------
 * cls_table_put compiles an ACL's rules (evalACL semantics,
 * aclengine_mock.go:473-668) into the engine's device layout and uploads it.
 * Replaces the per-evaluation re-parse of acl.Rules (aclengine_mock.go:480-524).
 */
int cls_table_put(cls_engine* e, const char* name, const cls_rule* rules,
                  uint32_t n_rules, uint32_t* table_id);
int cls_table_del(cls_engine* e, uint32_t table_id);

typedef struct cls_table_info {
    uint32_t n_rules;          /* R: counters_out has R+1 entries */
    uint32_t kernel;           /* 0 = linear (ballot) kernel, 1 = compiled classifier */
    uint32_t lds_bytes;        /* LDS image of the compiled classifier (v4) */
    uint32_t n_intervals;      /* elementary source intervals (v4) */
    uint32_t n_classes;        /* distinct source-prefix classes (v4) */
    uint32_t n_templates;      /* distinct (dst, port range, result) tuples (v4) */
    uint32_t n_slots;          /* flattened candidate slots (v4) */
    uint32_t lds_resident;     /* 1 if the classifier fits LDS, else global memory */
    uint32_t has_v16;          /* 1 if CLS_AF_V16 batches can be classified */
    uint32_t lds_bytes_v16;    /* LDS image of the 16-byte layout's classifier */
    uint32_t lds_resident_v16;
    uint32_t n_lctr;           /* slots counted in LDS (v4; the rest in global memory) */
    uint32_t ctr16;            /* the LDS slot counters are u16 (v4) */
    uint32_t list_mode;        /* candidate-list mode of the v4 classifier (cls_image_v4_header) */
    uint32_t swap;             /* the v4 classifier is keyed on destinations (cls_image_v4_header) */
    uint32_t reserved[1];
} cls_table_info;
int cls_table_get_info(cls_engine* e, uint32_t table_id, cls_table_info* info);

/* ---- batched first-match -------------------------------------------------
 * verdict_out[i] = evalACL(acl, pkt i) (ACLAction, aclengine_mock.go:473-668).
 * counters_out[k] (k < R) = packets whose evaluation terminated at rule k,
 * counters_out[R] = packets that fell through to the default DENY (:667).
 * `stream` is a hipStream_t (NULL: the engine's own stream).  The call is
 * synchronous with respect to the host unless CLS_F_DEVICE is set, in which
 * case work is only enqueued on `stream`.
 * Threading: any thread may call; calls are serialised while they enqueue.
 * Device work of concurrent calls on different streams may overlap, also on
 * one table: every (table, stream) pair has its own counter scratch.  A
 * table deleted (cls_table_del, cls_acl_put/del) while device work on it is
 * pending is freed only after that work finishes.
 */
int cls_classify(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pkts,
                 uint64_t n, uint8_t* verdict_out, uint64_t* counters_out,
                 uint32_t flags, void* stream);

/* The per-packet trace of evalACL's matched rule (the reference logs it at
 * Debug, aclengine_mock.go:651-654): verdict_out[i] as cls_classify (may be
 * NULL) and rule_out[i] = the index k of the rule at which packet i's
 * evaluation terminated, R for the default DENY (:667) -- the counter
 * cls_classify adds the packet to.  No counters are touched.  Flags:
 * CLS_F_DEVICE (device arrays, rule_out 4-byte aligned; stream-ordered),
 * else host arrays and the call returns with the results.  Replaces, for a
 * batch, the rule index evalACL computes and logs per call. */
int cls_classify_rules(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pkts,
                       uint64_t n, uint8_t* verdict_out, uint32_t* rule_out,
                       uint32_t flags, void* stream);

/* Milliseconds of the last classify kernel (CLS_F_TIMING), measured with HIP
 * events on the launch stream.  Blocks until that kernel has finished. */
int cls_last_kernel_ms(cls_engine* e, float* ms);
/* Every classify kernel timed (CLS_F_TIMING) since the last reset: up to `cap`
 * durations in launch order; *count = number recorded.  Recording enqueues
 * only events (no host synchronisation); reading blocks on the last one. */
int cls_kernel_times(cls_engine* e, float* ms, uint32_t cap, uint32_t* count);
/* The same kernels' start times, milliseconds after the first one's: the
 * differences are the launch-to-launch period of a stream of timed calls
 * (each kernel stamps its own start, so no event marker sits between them). */
int cls_kernel_starts(cls_engine* e, float* ms, uint32_t cap, uint32_t* count);
int cls_kernel_times_reset(cls_engine* e);

/* Measurement only (bench.py): the classify kernel's HBM stream without the
 * lookups -- the same loads and stores, order and grid -- over a device batch
 * (CLS_AF_V4: 16-B aligned addresses, 8-B dport, 4-B proto and verdict;
 * CLS_AF_V16: 16-B aligned addresses, whole 256-packet steps), `reps` timed
 * launches after one warm-up; *ms = the average launch.  Writes verdict. */
int cls_stream_floor(cls_engine* e, const cls_pkt_soa* pkts, uint64_t n, uint8_t* verdict,
                     uint32_t reps, float* ms, void* stream);
/* The same, one average per stream shape (cls_stream_floor returns their
 * minimum): shape = variant << 1 | (two 1024-thread workgroups per CU, else
 * one -- the classify kernel's own shape when its LDS image takes more than
 * half of the CU's LDS); variant 0 / 1 / 2 / 3 = loads as classify4_cls / one
 * step ahead / protocol non-temporal / both (CLS_AF_V16: variant 0 only).  Up
 * to `cap` times into ms; *count = the number of shapes. */
int cls_stream_floor_shapes(cls_engine* e, const cls_pkt_soa* pkts, uint64_t n, uint8_t* verdict,
                            uint32_t reps, float* ms, uint32_t cap, uint32_t* count, void* stream);

/* ---- ACL configuration (ACLConfig, aclengine_mock.go:110-121,671-728) --- */
/* PutACL semantics (:699-728): requires >=1 interface; re-putting a name
 * replaces it without counting an extra change; last writer wins per
 * interface direction.  A re-put whose rules equal the installed ACL's (the
 * renderer re-puts a local table whose pods changed, acl_renderer.go:186-190)
 * keeps the compiled table and only moves the interface bindings: no
 * compilation, no upload.  Either way the put installs a new ACL, so its
 * connection counters (cls_conn_counters) start from zero. */
int cls_acl_put(cls_engine* e, const char* acl_name, const cls_rule* rules,
                uint32_t n_rules, const char* const* ingress_ifs, uint32_t n_ingress,
                const char* const* egress_ifs, uint32_t n_egress);
/* DelACL semantics (:680-696). */
int cls_acl_del(cls_engine* e, const char* acl_name);
/* Table id of the installed ACL `acl_name` (GetACLByName, :228-234). */
int cls_acl_table(cls_engine* e, const char* acl_name, uint32_t* table_id);
/* GetNumOfACLs (:209), GetNumOfACLChanges (:237). */
int cls_acl_counts(cls_engine* e, uint32_t* n_acls, uint32_t* n_changes);
/* cls_acl_put calls that compiled a table / that kept the installed one. */
int cls_acl_stats(cls_engine* e, uint32_t* n_compiles, uint32_t* n_rebinds);
/* Interface id used by cls_conn_batch; ids are stable for the engine's life. */
int cls_if_id(cls_engine* e, const char* if_name, uint32_t* id);
/* Table id of the inbound/outbound ACL on an interface, -1 if none
 * (GetInboundACL / GetOutboundACL, :215-225). */
int cls_if_acls(cls_engine* e, uint32_t if_id, int32_t* in_table, int32_t* out_table);

/* ---- batched connection verdicts (testConnection, :394-471) -------------
 * For each connection i: SYN through src_if inbound then dst_if outbound
 * with (src->dst, dport); SYN-ACK through dst_if inbound then src_if outbound
 * with (dst->src, sport); REFLECT marks sides reflected exactly as the
 * reference does.  Interface->ACL bindings are snapshotted at the call.
 * Addresses: CLS_AF_V4 (src4/dst4) or CLS_AF_V16 (src16/dst16, 16-byte
 * aligned on the device; IPv4-mapped = IPv4, as Go's To4) -- Connection*
 * takes any net.IP (:243-390).  A device batch's interface id outside the
 * engine's ids gives CLS_CONN_FAILURE for that connection (a host batch is
 * rejected with CLS_E_INVAL).  At most 2^30 connections per call.
 * Large ACLs: in batches >= 65536, an ACL with a compiled classifier image
 * whose linear work would be large (host batch: connections touching it x
 * its rules >= 2048 x batch, touches estimated from a hashed sample of <= 64
 * Ki connections -- a heuristic, verdicts do not depend on it; device batch:
 * >= 2048 rules) is evaluated by the classifier kernel for both tuples of
 * every connection before the connection kernel runs; the others by a linear
 * scan of compact rules, staged in LDS when they fit.  CLS_F_CONN_CLS: every
 * imaged ACL (>= 64 rules) at any batch size; CLS_F_FORCE_LINEAR: none.
 * CLS_F_COUNT: for every evalACL call the batch makes on a non-nil ACL (only
 * the calls testConnection makes, in its order), the table's connection
 * counter of the terminating rule (R: default DENY) is incremented.
 */
typedef struct cls_conn_soa {
    cls_pkt_soa pkt;           /* src/dst/sport/dport/proto of the SYN */
    const uint32_t* src_if;    /* interface ids (cls_if_id) */
    const uint32_t* dst_if;
} cls_conn_soa;

/* The connection path's floor: the average time of a kernel that reads the
 * 22 bytes of every IPv4 connection of a device batch (src, dst, src_if,
 * dst_if, sport, dport, proto) and writes one byte, without evaluating
 * anything, over `reps` launches (whole groups of 4 connections; 16-B aligned
 * src / dst / src_if / dst_if, 8-B ports, 4-B proto and out). */
int cls_stream_floor_conn(cls_engine* e, const cls_conn_soa* conns, uint64_t n, uint8_t* out,
                          uint32_t reps, float* ms, void* stream);
int cls_connect_batch(cls_engine* e, const cls_conn_soa* conns, uint64_t n,
                      uint8_t* conn_verdict_out, uint32_t flags, void* stream);

/* Per-(ACL, rule) hit counters of the connection path: counters_out[k]
 * (k < R) = evalACL calls of cls_connect_batch (CLS_F_COUNT) on this table that
 * terminated at rule k, counters_out[R] = calls that fell through to the
 * default DENY (:667); summed over calls since the table was put or last
 * reset (reset != 0 clears them after the read).  Waits for pending device
 * work.  The reference has no counters. */
int cls_conn_counters(cls_engine* e, uint32_t table_id, uint64_t* counters_out, uint32_t reset);

/* ---- synthetic traffic (BASELINE.md / SURVEY 8(d) generator) -----------
 * Generates packets i in [first, first+n) of the counter-based splitmix64
 * stream directly into device memory (no PCIe).  Pools: pod IPs, rule
 * destination prefixes (addr, prefix length) and ports drawn from the table.
 */
typedef struct cls_traffic_spec {
    uint64_t seed;
    uint32_t pct_pod_src;      /* % of packets whose src is a pod IP (60) */
    uint32_t pct_rule_dst;     /* % whose dst lies in a rule dst prefix (50) */
    uint32_t pct_table_port;   /* % whose dport is one of the table ports (50) */
    uint32_t pct_icmp;         /* % ICMP (0 or 10); the rest split TCP/UDP evenly */
    const uint32_t* pod_ips; uint32_t n_pod_ips;
    const uint32_t* dst_addrs; const uint8_t* dst_lens; uint32_t n_dst;
    const uint16_t* ports; uint32_t n_ports;
} cls_traffic_spec;
int cls_gen_traffic_v4(cls_engine* e, const cls_traffic_spec* spec, uint64_t first,
                       uint64_t n, uint32_t* src4, uint32_t* dst4, uint16_t* sport,
                       uint16_t* dport, uint8_t* proto, void* stream);

/* The 16-byte stream (config 5, mixed families): pools of 16-byte network-
 * order addresses (IPv4 as IPv4-mapped), destination prefix lengths 0..128.
 * Packet i draws w_k = splitmix64(seed ^ ((8i + k) * golden)), k < 8, as the
 * IPv4 stream does for protocol, ports and the pool choices; an address not
 * drawn from a pool is IPv6 fd00::/64 + w_6 (src) or w_7 (dst) when bit 0 of
 * the choice word's high half is set, else IPv4-mapped ::ffff:(u32)w_1 (src)
 * or (u32)w_3 (dst); a pool prefix's host bits come from (w_3, w_7). */
typedef struct cls_traffic_spec16 {
    uint64_t seed;
    uint32_t pct_pod_src, pct_rule_dst, pct_table_port, pct_icmp;
    const uint8_t* pod_ips; uint32_t n_pod_ips;            /* n x 16 bytes */
    const uint8_t* dst_addrs; const uint8_t* dst_lens; uint32_t n_dst;
    const uint16_t* ports; uint32_t n_ports;
} cls_traffic_spec16;
int cls_gen_traffic_v16(cls_engine* e, const cls_traffic_spec16* spec, uint64_t first,
                        uint64_t n, uint8_t* src16, uint8_t* dst16, uint16_t* sport,
                        uint16_t* dport, uint8_t* proto, void* stream);

/* ---- engine-owned batches (SURVEY 8(b) ownership, 8(e) sharding) --------
 * A batch is device memory the engine owns, so a caller that must not let
 * the library keep its pointers (cgo) can still run the HBM-resident path:
 * upload once (or generate on the device), classify many times, download
 * what it needs.  Packets [0, n) shard contiguously over the engine's
 * devices (cls_shard_range): shard g = [g n / G, (g + 1) n / G) lives in
 * device g's HBM.  Fields are structure-of-arrays, each array 256-B aligned
 * per shard (the classify kernels' 16-B loads): addresses u32 (CLS_AF_V4)
 * or 16 bytes (CLS_AF_V16), ports u16, protocol and verdict u8, interface
 * ids u32 (CLS_BATCH_CONN).  With CLS_BATCH_MIRROR the batch also owns a
 * pinned host copy of every field (hipHostMalloc; cls_batch_mirror) that
 * the caller fills or reads in place: uploads and downloads with a NULL
 * host pointer move it at DMA speed.  Without it, upload / download go
 * through the engine's pinned staging buffers.
 * Work on a batch runs on its devices' engine streams; a call returns once
 * the work is enqueued unless it returns host data (counters_out,
 * downloads, cls_batch_counters, cls_batch_wait). */
typedef struct cls_batch cls_batch;
enum {
    CLS_BF_SRC = 0, CLS_BF_DST = 1, CLS_BF_SPORT = 2, CLS_BF_DPORT = 3, CLS_BF_PROTO = 4,
    CLS_BF_VERDICT = 5,        /* cls_classify_batch: ACLAction; cls_batch_connect: ConnectionAction */
    CLS_BF_SRC_IF = 6, CLS_BF_DST_IF = 7,   /* CLS_BATCH_CONN only */
    CLS_BF_COUNT = 8
};
enum {
    CLS_BATCH_CONN = 1u << 0,    /* also interface ids (connection batches) */
    CLS_BATCH_MIRROR = 1u << 1   /* a pinned host mirror of every field */
};
/* Shard g of n packets over G devices: [g n / G, (g + 1) n / G). */
int cls_shard_range(uint64_t n, uint32_t n_shards, uint32_t shard, uint64_t* first, uint64_t* count);
int cls_batch_create(cls_engine* e, uint32_t af, uint64_t n, uint32_t flags, cls_batch** out);
void cls_batch_destroy(cls_batch* b);
int cls_batch_shards(const cls_batch* b, uint32_t* n_shards);
int cls_batch_shard(const cls_batch* b, uint32_t shard, int* device, uint64_t* first, uint64_t* n);
/* Device address of a field's array in shard `shard` (for a caller's own
 * kernels, e.g. a capture path writing packets in place). */
int cls_batch_field(cls_batch* b, uint32_t shard, uint32_t field, void** dev_ptr);
/* Host address of a field's pinned mirror (whole batch, packet order). */
int cls_batch_mirror(cls_batch* b, uint32_t field, void** host_ptr);
/* Packets [first, first + n) of one field from `src` (NULL: the mirror). */
int cls_batch_upload(cls_batch* b, uint32_t field, uint64_t first, uint64_t n, const void* src);
/* ... to `dst` (NULL: the mirror).  Waits for the batch's work. */
int cls_batch_download(cls_batch* b, uint32_t field, uint64_t first, uint64_t n, void* dst);
/* The synthetic stream into the batch on the devices: packet i of the batch
 * is stream packet stream_first + i (the same stream as cls_gen_traffic_*). */
int cls_batch_gen_traffic_v4(cls_batch* b, const cls_traffic_spec* spec, uint64_t stream_first);
int cls_batch_gen_traffic_v16(cls_batch* b, const cls_traffic_spec16* spec, uint64_t stream_first);
/* evalACL over every packet of the batch (verdicts into CLS_BF_VERDICT) with
 * the table's hit counters (as cls_classify) summed over the shards: by the
 * engine's RCCL communicator when it has one (an all-reduce over the
 * devices -- and over the processes of cls_comm_init -- on a side stream, so
 * it overlaps the next call's classify; two counter buffers alternate), else
 * on the host when read.  counters_out (host, R + 1): wait and write them
 * (CLS_F_ACCUMULATE: add); NULL: only enqueue (cls_batch_counters reads the
 * last call's).  Flags: CLS_F_NO_VERDICT, CLS_F_FORCE_LINEAR, CLS_F_TIMING
 * (each device's classify kernel is timed on that device's engine:
 * cls_kernel_times of cls_device_engine), CLS_F_ACCUMULATE. */
int cls_classify_batch(cls_engine* e, uint32_t table_id, cls_batch* b, uint64_t* counters_out, uint32_t flags);
/* Counters of the batch's last cls_classify_batch (n_out >= R + 1 of that
 * table); waits for them. */
int cls_batch_counters(cls_batch* b, uint64_t* out, uint32_t n_out);
/* testConnection over a CLS_BATCH_CONN batch (as cls_connect_batch with
 * device memory; ConnectionAction into CLS_BF_VERDICT), every device its
 * shard; CLS_F_COUNT counts into each device's copy of the tables'
 * connection counters (cls_conn_counters sums them).  Returns when done. */
int cls_batch_connect(cls_engine* e, cls_batch* b, uint32_t flags);
/* Wait for every device's work on the batch. */
int cls_batch_wait(cls_batch* b);

/* ---- the hit-counter all-reduce over processes (RCCL) --------------------
 * One process per GPU (or per group of GPUs): process 0 makes an id
 * (cls_comm_unique_id), every process receives it out of band and calls
 * cls_comm_init with the same n_procs; device g of process p is rank
 * p * G + g of n_procs * G (every process's engine has G devices).  From
 * then on cls_classify_batch all-reduces its counters over all ranks.
 * n_procs = 1 with id NULL: a communicator over this engine's devices alone
 * (ncclCommInitAll; also at one device).  Replaces an earlier communicator. */
int cls_comm_unique_id(void* id128);
int cls_comm_init(cls_engine* e, uint32_t n_procs, uint32_t proc, const void* id128);
/* Ranks of the engine's communicator (0: none) and its first device's rank. */
int cls_comm_info(cls_engine* e, uint32_t* n_ranks, uint32_t* rank0);

/* ---- offline compilation (no device needed) -----------------------------
 * Compiles an ACL exactly as cls_table_put does and writes the IPv4 device
 * layouts into `blob`: a cls_image_v4_header followed by the classifier image,
 * the slot->rule map and the linear rules.  With cap too small (or blob NULL)
 * only *need is set.  Used for inspection and CPU-side verification of the
 * compiler.
 */
typedef struct cls_image_v4_header {
    uint32_t magic;            /* 0x434C5334 "CLS4" */
    uint32_t version;          /* 4 (CLS_ABI_VERSION 3) */
    uint32_t n_rules, n_lin, has_cls;
    uint32_t img_bytes, off_bounds, off_iclass, off_cells, off_lists, off_tmpl;
    uint32_t n_bounds, search_top, n_classes, n_tmpl, n_list_entries, n_ctr, lds_bytes;
    uint32_t off_image, off_ctr_rule, off_lin;   /* byte offsets inside the blob */
    uint32_t total_bytes;
    uint32_t mode;             /* source lookup: 0 interval search, 1 hash LPM, 4 trie */
    uint32_t default_class;    /* hash LPM: class when no hashed prefix matches */
    uint32_t n_hash;           /* hashed prefix lengths (ascending) */
    uint32_t hash_mask[3], hash_shift[3], hash_cap[3], off_hash[3];
    uint32_t list_mode;        /* candidate lists: 0 template scan, 1 bit vectors,
                                  2 bit vectors with global port classes,
                                  3 port-filtered sublists (radix port classes),
                                  4 port-filtered sublists (hashed port classes),
                                  5, 6: 4, 3 with wide cells in global memory (off_gcells) */
    uint32_t off_bv, bv_steps_d, bv_steps_p;
    uint32_t off_ptop;         /* list modes 2, 3: port radix at 0 (256 x u32 window address,
                                  then u8 windows of class per port) */
    uint32_t n_pclass;         /* list modes 2, 3: global port classes */
    uint32_t bv_wide;          /* some bit-vector list has more than 16 entries */
    uint32_t row_bytes;        /* a class's 4 cells (TCP, UDP, ICMP, other protocols) at
                                  off_cells + class x row_bytes */
    uint32_t default_row;      /* hash LPM: cell row of default_class (hash entries hold rows) */
    uint32_t hash_mul[3];      /* hash LPM: p = key x mul; h0 = p >> shift, h1 = next log2(cap) bits */
    uint32_t port_mul, port_mask4, port_dflt;  /* list mode 4: e = u32 at byte mulhi(port, mul) &
                                  mask4, class x 4 = (e & 0xFFFF) == port ? e >> 16 : port_dflt */
    uint32_t n_hot, off_hot;   /* per-lane counter rows of the hot slots (LDS offsets) */
    uint32_t n_lctr;           /* slots counted in LDS (the rest: global counters) */
    uint32_t ctr16;            /* LDS slot counters are u16 (else u32) */
    uint32_t swap;             /* 1: classes keyed on the DESTINATION address -- the image sees
                                  packets with src and dst exchanged */
    uint32_t off_other;        /* blob offset of the OTHER image (protocols > 2: one cell per
                                  class, interval search, template scan; magic 0x434C534F "CLSO",
                                  its slots numbered after this image's), 0 if none */
    uint32_t off_trie;         /* mode 4 (source trie): level 1 (256 u32 by src >> 24: node byte
                                  address), nodes (256 u32 by bits 16..23: leaf byte address << 4
                                  | depth), leaves (2^depth u32 {key | class << 16}) */
    uint32_t trie_depth;       /* deepest leaf of the trie */
    uint32_t off_gcells;       /* list modes 5, 6 (4, 3 with wide cells): blob offset of the
                                  cells, uint2 {pointer table byte address, counter base} per
                                  (class, protocol); n_gcells u32 words */
    uint32_t n_gcells;
} cls_image_v4_header;
int cls_compile_v4(const cls_rule* rules, uint32_t n_rules, void* blob, uint64_t cap,
                   uint64_t* need, const char* options);   /* "key=value,..." (cls_engine_set_option's compiler keys) or NULL */
/* Whether the library has a classify kernel for an image of source lookup
 * `mode` and `list_mode` (cls_image_v4_header), LDS-resident or in global
 * memory; rep16: the 16-byte core.  CLS_OK, or CLS_E_INVAL for a combination
 * no kernel implements -- cls_table_put / cls_acl_put refuse such an image
 * with CLS_E_INVAL instead of launching another variant's kernel on it. */
int cls_image_kernel(uint32_t mode, uint32_t list_mode, int lds_resident, int rep16);
/* Diagnostics (CPU verification): the bitmap form cls_connect_batch gives a
 * linear IPv4 ACL (per-ACL interval tables of source, destination and each
 * protocol's destination port, one rule bit row per interval), built from
 * `rules` and evaluated on the host for n IPv4 packets: evalACL's ACLAction
 * and the terminating rule (n_rules: default DENY) per packet. */
int cls_conn_bitmap_eval(const cls_rule* rules, uint32_t n_rules, const uint32_t* src, const uint32_t* dst,
                         const uint16_t* dport, const uint8_t* proto, uint64_t n, uint8_t* res_out,
                         uint32_t* rule_out);

/* The 16-byte layout's compiled form (what cls_classify runs for CLS_AF_V16
 * batches): both address families are mapped to 32-bit representatives by a
 * front end -- per side (0 src, 1 dst) fe_top 16-B keys at image offset
 * fe_key (interval start - 1 as u64 hi, u64 lo in address order; padding all
 * ones) and fe_n u32 representatives at fe_val -- and `core` is the IPv4
 * classifier over the rules restated on representatives (magic 0x434C3136
 * "CL16"; its linear rules are in representative space too).  Returns
 * CLS_E_INVAL when the table has no 16-byte classifier.
 */
typedef struct cls_image_v16_header {
    cls_image_v4_header core;
    uint32_t fe_key[2], fe_val[2], fe_top[2], fe_n[2];
    /* src_mode 1 (every source prefix a host route): the source side is two
     * cuckoo hashes straight to class rows -- IPv4-mapped: {key, row} 8-B
     * entries at h4 (2 x cap4), key = address bytes 12-15 as a little-endian
     * word, h = key x mul4; IPv6: 16-B keys at k6 and u32 rows at r6 (2 x
     * cap6 slots), h = (w0 x fold0 ^ w1 x fold1 ^ w2 x fold2 ^ w3) x mul6;
     * table 0 slot = h >> (32 - L), table 1 slot = (h >> (32 - 2L)) & (cap - 1).
     * The source interval table (keys, reps at src_search_val) is then not
     * in the image but at blob offset off_src_search (the protocol > 2 path). */
    uint32_t src_mode, h4, cap4, mul4, k6, r6, cap6, mul6, fold[3], dflt_row[2];
    uint32_t off_src_search, src_search_val;
    /* fe_k8[s]: side s's keys are 8 B, key8(start) - 1 with key8(x) = hi64 == 0 ?
     * min(lo64, 2^48) : 2^48 + min(hi64, 2^64 - 1 - 2^48) (exact when every
     * start has hi64 = 0 and lo64 <= 2^48, or lo64 = 0) */
    uint32_t fe_k8[2];
    /* src_mode 2 (sources not all host routes, many IPv4 intervals): an
     * IPv4-mapped source's row from the trie over its IPv4 word at the core
     * header's off_trie / trie_depth (leaf entries carry the core's class);
     * any other source's row from the side-0 search (fe_key[0] ...), whose
     * table holds only the non-IPv4 intervals and rows as values.  src_mode
     * 1 and 2: the source interval table at off_src_search has
     * src_search_top keys (8 B when src_search_k8). */
    uint32_t src_search_top, src_search_k8;
} cls_image_v16_header;
int cls_compile_v16(const cls_rule* rules, uint32_t n_rules, void* blob, uint64_t cap,
                    uint64_t* need, const char* options);

#ifdef __cplusplus
}
#endif
#endif /* CONTIVCLS_H */
