// Internal types of the engine (engine.cpp, fleet.cpp): device buffers,
// compiled tables with their device copies, the per-device engine state.
// Not part of the C ABI (include/contivcls.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/contivcls.h"
#include "compile.hpp"
#include "kernels.hpp"
#include "options.hpp"

using namespace cls;

// The caller's current device, restored when an entry point returns: the
// library sets each engine's device for its work and leaves the calling
// thread's HIP state as it found it.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        int now = -1;
        if (dev >= 0 && hipGetDevice(&now) == hipSuccess && now != dev) (void)hipSetDevice(dev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        hipError_t e = hipMalloc(&p, n < 256 ? 256 : n);
        if (e == hipSuccess) bytes = n < 256 ? 256 : n;
        return e;
    }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

// Counter scratch of one (table variant, stream): concurrent classifies of
// one table on different streams never share a counter buffer
// (include/contivcls.h, threading).  slot_val is all zero between calls: the
// remap kernel reads and clears it.
struct Scratch {
    DevBuf part;                   // per-workgroup LDS counter rows [rows][n_lctr]
    DevBuf oq;                     // OTHER queue {fill per workgroup, segments of indices}
    DevBuf slot_val;               // u64 per slot: global-tier counters, folded partials
    DevBuf out;                    // u64 rule counters when the caller gives none on device
    // (no completion event: the buffers are freed with hipFree, which
    // synchronises the device first -- a done event stamped by every call's
    // last launch cost the stream 2 us per call, config 2 0.0399 against
    // 0.0379 ms per step, profiles/r06i_finish_event_ab.txt)
};

// Slot counters of one classifier image (or of the linear kernel alone):
// slots [0, n_ctr) of the image, then R + 1 direct rule slots.
struct Counters {
    uint32_t n_slots = 0;
    uint32_t n_lctr = 0;           // slots counted in LDS (their partial rows)
    uint32_t n_image = 0;          // slots of the classifier images; the direct rule slots follow
    DevBuf d_csr;                  // uint2 {slot, rule}, grouped by rule
    DevBuf d_slot_rule;            // finish launch: u32 per slot (rule, or kHotRule | h), then the hot rules
    uint32_t n_hot = 0;
    DevBuf d_other_map;            // finish launch: compact rule index per OTHER slot, then those rules
    uint32_t n_other = 0, n_orules = 0;
    std::map<hipStream_t, std::unique_ptr<Scratch>> sc;
};

// An event shared by the tables of one counting connection batch.
struct SharedEvent {
    hipEvent_t ev = nullptr;
    SharedEvent() = default;
    SharedEvent(const SharedEvent&) = delete;
    SharedEvent& operator=(const SharedEvent&) = delete;
    ~SharedEvent() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

struct Table {
    std::string name;
    uint32_t n_rules = 0;
    std::string sig;           // the rules as given (rule_sig): a re-put of equal rules keeps this table
    // linear (ballot) table, also the protocol>2 fallback
    std::vector<LinRule4> lin4;
    DevBuf d_lin4;
    // IPv4 classifier
    bool has_cls = false;
    Cls4Image img;
    DevBuf d_img;
    Cls4Image oimg;            // protocols > 2 (compile.hpp Cls4Opts::other), read from global memory
    DevBuf d_oimg;
    // the OTHER image's source classes are img's (same interval bounds and
    // class numbering): the pair launch's queued connections carry their
    // classes (ceil(2^32 / img.row_bytes); 0: the drain searches again)
    uint32_t pair_cdiv = 0;
    // The pair launch's image (compile.hpp Cls4Opts::with_other: a fourth
    // cell per class for protocols > 2), built from sem4 at the table's
    // first connection batch that takes the pair launch: pimg_state 0 not
    // yet, 1 built and uploaded, -1 none (too large for LDS, no kernel)
    std::shared_ptr<const std::vector<SemRule>> sem4;
    int pimg_state = 0;
    Cls4Image pimg;
    DevBuf d_pimg, d_pslot_rule;
    DevBuf d_pslot16;           // the slot -> rule map as u16 (rules < 65535), 16-B padded; n16 units
    uint32_t pslot16_n16 = 0;
    int kernel = 0;            // 0 linear, 1 classifier
    bool lds_resident = false;
    // 16-byte layout (IPv6 / IPv4-mapped): classifier over 32-bit reps
    struct {
        bool ok = false;
        std::string why;           // why there is none
        Cls16Image img;
        std::vector<LinRule4> lin; // rules in rep space (FORCE_LINEAR)
        Cls4Image oimg;            // protocols > 2, rep space
        DevBuf d_img, d_lin, d_oimg;
        DevBuf d_src_search;       // src_mode 1, 2: the source interval table (global memory)
        bool lds_resident = false;
        DevBuf d_slot_rule;        // slot mode (connection batches): slot -> rule, core then OTHER image
    } p16;
    // connection path: compact linear rules (cls_connect_batch's rule pool),
    // slot -> rule of the v4 images (slot mode), and the per-rule connection
    // counters (CLS_F_COUNT; allocated on first use, R + 1 u64)
    std::vector<ConnRule4> conn4;
    std::vector<ConnRule16> conn16;
    // the bitmap form of conn4 (conn_bitmap4), built on the first connection
    // batch that wants it; empty when its tables exceed kConnBmMaxWords
    std::vector<uint32_t> conn_bm;
    bool conn_bm_built = false;
    DevBuf d_slot_rule;
    DevBuf d_conn_ctr;
    // recorded on the engine stream behind a rebind's counter clearing; a
    // counting connection batch on another stream waits for it
    hipEvent_t conn_ctr_ev = nullptr;
    // recorded behind the last counting connection batch's scatter into
    // d_conn_ctr: cls_conn_counters waits for it (not for the whole device);
    // one event per batch, shared by the batch's tables
    std::shared_ptr<SharedEvent> conn_ev;
    // bumped whenever the connection counters are cleared by a rebind (a
    // multi-device engine's peers clear their copies when it moves)
    uint64_t conn_epoch = 0;
    ~Table() {
        if (conn_ctr_ev) (void)hipEventDestroy(conn_ctr_ev);
    }
    // declared last: destroyed first, so pending device work is waited for
    // before any of the buffers above are freed
    Counters c4, c16;
};

struct AclEntry {
    uint32_t table_id = 0;
    std::vector<uint32_t> ingress, egress;
};


// The host side of a connection batch over the current bindings: one
// descriptor per bound table, (in, out) per interface, the large ACLs
// evaluated by the classifier, the rule pool with the bitmap forms.  A device
// batch's plan depends only on the bindings and the flags, so it is kept
// until they change (cls_engine::conn_gen).
struct ConnPlan {
    uint64_t key = ~0ull, gen = ~0ull;
    uint64_t id = 0;                                      // which plan s_desc / s_ifs / s_rules hold (uploaded)
    std::vector<ConnDesc> desc;
    std::vector<std::shared_ptr<Table>> dtab;             // table of each descriptor
    std::vector<IfAcls> ifs;
    std::vector<uint32_t> big;                            // descriptors of the large ACLs
    std::vector<uint8_t> pool;
    uint32_t n_ctr = 0;
    uint32_t bm_steps = 0;                                // lower-bound steps of the largest bitmap table
};

struct cls_engine {
    int device = 0;
    int n_cu = 256;
    Opts opts;                     // tuning / diagnostic switches (cls_engine_set_option)
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string err;
    std::map<uint32_t, std::shared_ptr<Table>> tables;
    uint32_t next_table = 1;
    // ACLConfig
    std::map<std::string, AclEntry> acls;
    std::unordered_map<std::string, uint32_t> if_ids;
    std::vector<std::string> if_names;
    std::vector<std::pair<int32_t, int32_t>> if_acl;   // per if id: (inbound, outbound) table id
    uint32_t changes = 0;
    uint32_t compiles = 0, rebinds = 0;   // cls_acl_put: tables compiled / puts that kept the table
    // scratch for host-pointer batches
    DevBuf s_src, s_dst, s_sport, s_dport, s_proto, s_verdict, s_if_a, s_if_b, s_desc, s_ifs;
    DevBuf s_pre;                  // connection path: classifier slot words per large ACL (8 bytes/connection)
    DevBuf s_pq;                   // connection path: the pair launch's OTHER queue
    DevBuf s_rules, s_tctr, s_cctr;  // connection path: rule pool, table counter pointers, call counters
    DevBuf s_crows;                  // ... LDS counter rows of the workgroups
    DevBuf s_rule;                   // cls_classify_rules of host arrays: the rule per packet
    bool cctr_zero = false;          // s_cctr cleared since its allocation (the scatter launch keeps it zero)
    // counting connection batches' scatter events (Table::conn_ev), reused
    // once no table holds them: one record per batch, not one per table
    std::vector<std::shared_ptr<SharedEvent>> conn_evs;
    uint64_t conn_gen = 0;           // bumped by every change of tables or interface bindings
    ConnPlan conn_plan;              // the last device batch's plan
    uint64_t plan_ids = 0, up_plan = ~0ull;   // plan ids; the plan whose tables are on the device
    // what s_desc, s_ifs, s_rules and s_tctr hold (the last upload): a
    // connection batch over unchanged bindings uploads nothing
    std::vector<uint8_t> up_desc, up_ifs, up_rules, up_tctr;
    DevBuf s_pool;
    // A device connection batch is stream-ordered (connect_locked): the stream
    // of the last one while it may still run, waited for before its scratch,
    // plan or tables change (conn_quiesce); a batch on another stream waits
    // for it on the GPU (conn_sync_ev)
    hipStream_t conn_last = nullptr;
    hipEvent_t conn_sync_ev = nullptr;
    // the 16-byte traffic generator's address pools as (hi, lo) pairs: the
    // host source of an unsynchronised upload (gen16_locked, sync = false)
    // outlives the call; gen_pending: such an upload may still be reading it
    std::vector<uint64_t> gen_pairs;
    bool gen_pending = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    // per-launch timing (CLS_F_TIMING): event pairs, recycled after a reset
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    size_t ev_used = 0;
    // Multi-device engine (cls_config n_devices > 1, fleet.cpp): this engine
    // is the primary -- the ACL configuration, table ids and the first
    // device -- and every further device has a peer engine that mirrors the
    // primary's compiled tables (uploaded, never recompiled) and interface
    // bindings (sync_peers).  Peers are reached only through cls_device_engine
    // and refuse configuration calls.
    cls_engine* primary = nullptr;           // peers: their primary
    std::vector<cls_engine*> peers;
    uint64_t synced_gen = ~0ull;             // peers: the primary's conn_gen last mirrored
    // The hit-counter all-reduce (cls_comm_init; automatic over distinct
    // devices): this device's RCCL communicator and the stream it runs on
    void* comm = nullptr;                    // ncclComm_t
    hipStream_t coll = nullptr;
    uint32_t comm_ranks = 0, comm_rank = 0;
    // engine-owned pinned staging of batch uploads / downloads (fleet.cpp)
    void* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
};

// Wait for the last stream-ordered connection batch (cls_engine::conn_last).
inline int conn_quiesce(cls_engine* e) {
    if (!e->conn_last) return CLS_OK;
    hipStream_t s = e->conn_last;
    e->conn_last = nullptr;
    if (hipStreamSynchronize(s) != hipSuccess) {
        e->err = "hipStreamSynchronize of the last connection batch failed";
        return CLS_E_HIP;
    }
    return CLS_OK;
}

// engine i of a multi-device engine (0: the primary itself)
inline cls_engine* dev_engine(cls_engine* e, size_t i) { return i == 0 ? e : e->peers[i - 1]; }
inline size_t n_dev_engines(const cls_engine* e) { return 1 + e->peers.size(); }

inline int fail(cls_engine* e, int code, const char* fmt, ...) {
    if (e) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        e->err = buf;
    }
    return code;
}

#define HIPC(e, expr)                                                                    \
    do {                                                                                 \
        hipError_t _h = (expr);                                                          \
        if (_h != hipSuccess)                                                            \
            return fail((e), CLS_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_h),  \
                        __FILE__, __LINE__);                                             \
    } while (0)

// ---- engine.cpp internals used by fleet.cpp (the caller holds e->mu) -----
int engine_open(int device, cls_engine** out);
void engine_close(cls_engine* e);
int classify_locked(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pk, uint64_t n, uint8_t* verdict_out,
                    uint64_t* counters_out, uint32_t flags, void* stream);
// sync = false: the batch's device work is only enqueued (the caller
// synchronises `stream` before it returns)
int connect_locked(cls_engine* e, const cls_conn_soa* c, uint64_t n, uint8_t* out, uint32_t flags, void* stream,
                   bool sync);
int gen4_locked(cls_engine* e, const cls_traffic_spec* sp, uint64_t first, uint64_t n, uint32_t* src4,
                uint32_t* dst4, uint16_t* sport, uint16_t* dport, uint8_t* proto, void* stream, bool sync);
int gen16_locked(cls_engine* e, const cls_traffic_spec16* sp, uint64_t first, uint64_t n, uint8_t* src16,
                 uint8_t* dst16, uint16_t* sport, uint16_t* dport, uint8_t* proto, void* stream, bool sync);
// a table's host form (rules compiled once) copied for another device, and
// its upload to an engine's device
std::shared_ptr<Table> table_clone_host(const Table& t);
int table_upload(cls_engine* e, Table& t);
// fleet.cpp: mirror the primary's tables and bindings on its peers
int sync_peers(cls_engine* e);
