// Multi-device engines, engine-owned batches and the hit-counter all-reduce
// (include/contivcls.h: cls_config's device list, cls_batch_*,
// cls_classify_batch, cls_batch_connect, cls_comm_*).
//
// packets (and connections) are independent, so a batch shards
// contiguously over the devices -- shard g = [g n / G, (g + 1) n / G) in
// device g's HBM -- and the rule table is replicated: compiled once on the
// host, uploaded to every device (the peer engines, sync_peers).  The only
// collective is the integer-sum all-reduce of the per-rule hit counters,
// ncclAllReduce(ncclUint64, ncclSum) over xGMI on a side stream of every
// device, so one call's merge overlaps the next call's classify.
// batches are engine-owned memory (device arrays, a pinned host
// mirror, pinned staging), so a cgo caller reaches the HBM-resident path
// without the library keeping any of its pointers.
// The reference has no native code; the entry points serve the evaluation
// of mock/aclengine/aclengine_mock.go:243-390 (Connection*) and :473
// (evalACL) in bulk.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "engine_int.hpp"

namespace {

// ---- RCCL, loaded on first use -------------------------------------------
// dlopen, so the library loads (and its single-device paths run) where RCCL
// is absent; an already-loaded librccl.so.1 (PyTorch's) is reused, so one
// process never holds two RCCL runtimes.
struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* d = dlerror();
            r.why = std::string("librccl.so.1 not loadable: ") + (d ? d : "?");
            return;
        }
        bool all = true;
        auto sym = [&](const char* name) {
            void* p = dlsym(h, name);
            if (!p) all = false;
            return p;
        };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(sym("ncclCommInitAll"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        r.ok = all;
        if (!all) r.why = "librccl.so.1 lacks an entry point";
    });
    return r;
}

#define RCCLC(e, expr)                                                                        \
    do {                                                                                      \
        ncclResult_t _r = (expr);                                                             \
        if (_r != ncclSuccess)                                                                \
            return fail((e), CLS_E_RCCL, "%s: %s", #expr, rccl().error_string(_r));           \
    } while (0)

// Every device engine of `e` locked (the primary's lock is the caller's):
// the order is always primary, then peers in device order.
struct PeerLocks {
    std::vector<std::unique_lock<std::mutex>> held;
    explicit PeerLocks(cls_engine* e) {
        for (cls_engine* p : e->peers) held.emplace_back(p->mu);
    }
};

// The device engine failed: its message on the engine the caller holds.
int relay(cls_engine* e, cls_engine* d, int rc) {
    if (d == e || rc == CLS_OK) return rc;
    return fail(e, rc, "device %d: %s", d->device, d->err.c_str());
}

int side_stream(cls_engine* d) {
    if (d->coll) return CLS_OK;
    HIPC(d, hipSetDevice(d->device));
    HIPC(d, hipStreamCreateWithFlags(&d->coll, hipStreamNonBlocking));
    return CLS_OK;
}

void comm_release(cls_engine* e) {
    for (size_t i = 0; i < n_dev_engines(e); ++i) {
        cls_engine* d = dev_engine(e, i);
        if (d->comm) {
            (void)hipSetDevice(d->device);
            if (d->coll) (void)hipStreamSynchronize(d->coll);
            (void)rccl().comm_destroy(static_cast<ncclComm_t>(d->comm));
            d->comm = nullptr;
        }
        d->comm_ranks = d->comm_rank = 0;
    }
}

// Communicators for the engine's devices: nranks = n_procs x G; device g of
// process proc is rank proc x G + g (id: the unique id of process 0), or
// (id NULL, n_procs 1) one ncclCommInitAll over the devices.
int comm_make(cls_engine* e, uint32_t n_procs, uint32_t proc, const void* id) {
    Rccl& r = rccl();
    if (!r.ok) return fail(e, CLS_E_RCCL, "%s", r.why.c_str());
    const size_t G = n_dev_engines(e);
    if (n_procs == 0 || proc >= n_procs || (!id && n_procs != 1))
        return fail(e, CLS_E_INVAL, "cls_comm_init: process %u of %u (an id is needed above one process)", proc,
                    n_procs);
    comm_release(e);
    std::vector<ncclComm_t> comms(G, nullptr);
    // a failed init leaves none of its communicators behind
    struct Undo {
        std::vector<ncclComm_t>& c;
        bool keep = false;
        ~Undo() {
            if (!keep)
                for (ncclComm_t x : c)
                    if (x) (void)rccl().comm_destroy(x);
        }
    } undo{comms};
    std::vector<int> devs(G);
    for (size_t g = 0; g < G; ++g) devs[g] = dev_engine(e, g)->device;
    if (!id) {
        for (size_t g = 0; g < G; ++g)
            for (size_t h = 0; h < g; ++h)
                if (devs[g] == devs[h])
                    return fail(e, CLS_E_RCCL, "device %d listed twice: RCCL needs one rank per device", devs[g]);
        RCCLC(e, r.comm_init_all(comms.data(), int(G), devs.data()));
    } else {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        RCCLC(e, r.group_start());
        for (size_t g = 0; g < G; ++g) {
            HIPC(e, hipSetDevice(devs[g]));
            const ncclResult_t rc = r.comm_init_rank(&comms[g], int(n_procs * G), uid, int(proc * G + g));
            if (rc != ncclSuccess) {
                (void)r.group_end();
                return fail(e, CLS_E_RCCL, "ncclCommInitRank (rank %zu of %zu): %s", size_t(proc) * G + g,
                            size_t(n_procs) * G, r.error_string(rc));
            }
        }
        RCCLC(e, r.group_end());
    }
    undo.keep = true;
    for (size_t g = 0; g < G; ++g) {
        cls_engine* d = dev_engine(e, g);
        d->comm = comms[g];
        d->comm_ranks = uint32_t(n_procs * G);
        d->comm_rank = uint32_t(proc * G + g);
        const int rc = side_stream(d);
        if (rc != CLS_OK) return relay(e, d, rc);
    }
    return CLS_OK;
}

// ---- batches -------------------------------------------------------------
struct BatchShard {
    cls_engine* d = nullptr;           // the device's engine
    uint64_t first = 0, n = 0;         // its packets [first, first + n) of the batch
    DevBuf mem;                        // every field's array
    size_t off[CLS_BF_COUNT] = {};     // byte offsets in mem (256-B aligned)
    DevBuf fmem[CLS_BF_COUNT];         // option batch_layout=1 (measurement): one allocation per field
    // the hit counters of the last two classify calls (u64, R + 1): a
    // buffer is written again only after its all-reduce has finished
    DevBuf ctr[2];
    hipEvent_t classified[2] = {nullptr, nullptr}, reduced[2] = {nullptr, nullptr};
    bool rec_cls[2] = {false, false}, rec_red[2] = {false, false};
    BatchShard() = default;
    BatchShard(const BatchShard&) = delete;
    BatchShard& operator=(const BatchShard&) = delete;
    // on the shard's device: its events, then (members) its buffers -- also
    // on cls_batch_create's error paths
    ~BatchShard() {
        if (d) (void)hipSetDevice(d->device);
        for (int k = 0; k < 2; ++k) {
            if (classified[k]) (void)hipEventDestroy(classified[k]);
            if (reduced[k]) (void)hipEventDestroy(reduced[k]);
        }
    }
};

size_t field_bytes(uint32_t af, uint32_t f) {
    switch (f) {
    case CLS_BF_SRC: case CLS_BF_DST: return af == CLS_AF_V16 ? 16 : 4;
    case CLS_BF_SPORT: case CLS_BF_DPORT: return 2;
    case CLS_BF_PROTO: case CLS_BF_VERDICT: return 1;
    default: return 4;                 // interface ids
    }
}

constexpr size_t kStageBytes = size_t(32) << 20;   // pinned staging buffer (two per device engine)

}  // namespace

struct cls_batch {
    cls_engine* e = nullptr;
    uint32_t af = CLS_AF_V4, flags = 0;
    uint64_t n = 0;
    std::vector<BatchShard> sh;
    uint8_t* mirror = nullptr;         // CLS_BATCH_MIRROR: pinned host copy, field-major
    size_t moff[CLS_BF_COUNT] = {};
    int cur = -1;                      // counter buffer of the last classify (-1: none)
    uint32_t n_ctr = 0;                // R + 1 of that classify
    bool reduced = false;              // ... merged by the all-reduce (else summed on the host)
    bool has(uint32_t f) const { return f < CLS_BF_SRC_IF || (flags & CLS_BATCH_CONN); }
};

namespace {

void shard_of(uint64_t n, uint32_t G, uint32_t g, uint64_t& first, uint64_t& count) {
    // [g n / G, (g + 1) n / G) without overflow for n < 2^64 / G
    const unsigned __int128 a = (unsigned __int128)n * g / G, b = (unsigned __int128)n * (g + 1) / G;
    first = uint64_t(a);
    count = uint64_t(b - a);
}

template <typename T>
T* fld(const BatchShard& s, uint32_t f) {
    if (s.fmem[f].p) return static_cast<T*>(s.fmem[f].p);
    return reinterpret_cast<T*>(static_cast<uint8_t*>(s.mem.p) + s.off[f]);
}

int staging(cls_engine* d) {
    for (int k = 0; k < 2; ++k) {
        if (!d->stage[k]) HIPC(d, hipHostMalloc(&d->stage[k], kStageBytes, hipHostMallocDefault));
        if (!d->stage_ev[k]) HIPC(d, hipEventCreateWithFlags(&d->stage_ev[k], hipEventDisableTiming));
    }
    return CLS_OK;
}

// Host <-> device of one shard's piece: straight from / to pinned memory,
// or through the device engine's two pinned staging buffers (the copy of
// one chunk overlaps the host memcpy of the next).
int move_piece(cls_engine* d, uint8_t* dev, uint8_t* host, size_t bytes, bool up, bool pinned) {
    HIPC(d, hipSetDevice(d->device));
    if (pinned) {
        HIPC(d, hipMemcpyAsync(up ? dev : host, up ? host : dev, bytes,
                               up ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, d->stream));
        return CLS_OK;
    }
    const int rc = staging(d);
    if (rc != CLS_OK) return rc;
    if (up) {
        for (size_t o = 0, c = 0; o < bytes; o += kStageBytes, ++c) {
            const int k = int(c & 1);
            const size_t m = std::min(kStageBytes, bytes - o);
            HIPC(d, hipEventSynchronize(d->stage_ev[k]));        // its previous copy has left the buffer
            std::memcpy(d->stage[k], host + o, m);
            HIPC(d, hipMemcpyAsync(dev + o, d->stage[k], m, hipMemcpyHostToDevice, d->stream));
            HIPC(d, hipEventRecord(d->stage_ev[k], d->stream));
        }
        return CLS_OK;
    }
    // down: chunk c copies while chunk c - 1 is unpacked
    size_t prev_o = 0, prev_m = 0;
    for (size_t o = 0, c = 0;; o += kStageBytes, ++c) {
        const int k = int(c & 1);
        const bool more = o < bytes;
        if (more) {
            const size_t m = std::min(kStageBytes, bytes - o);
            HIPC(d, hipMemcpyAsync(d->stage[k], dev + o, m, hipMemcpyDeviceToHost, d->stream));
            HIPC(d, hipEventRecord(d->stage_ev[k], d->stream));
        }
        if (c > 0) {
            const int j = int((c - 1) & 1);
            HIPC(d, hipEventSynchronize(d->stage_ev[j]));
            std::memcpy(host + prev_o, d->stage[j], prev_m);
        }
        if (!more) break;
        prev_o = o;
        prev_m = std::min(kStageBytes, bytes - o);
    }
    return CLS_OK;
}

int batch_move(cls_batch* b, uint32_t f, uint64_t first, uint64_t n, uint8_t* host, bool up) {
    cls_engine* e = b->e;
    if (f >= CLS_BF_COUNT || !b->has(f)) return fail(e, CLS_E_INVAL, "batch has no field %u", f);
    if (first > b->n || n > b->n - first) return fail(e, CLS_E_INVAL, "packets out of the batch");
    const bool pinned = host == nullptr;
    if (pinned && !b->mirror) return fail(e, CLS_E_INVAL, "no host pointer and no mirror (CLS_BATCH_MIRROR)");
    const size_t eb = field_bytes(b->af, f);
    for (BatchShard& s : b->sh) {
        const uint64_t lo = std::max(first, s.first), hi = std::min(first + n, s.first + s.n);
        if (lo >= hi) continue;
        uint8_t* dev = fld<uint8_t>(s, f) + (lo - s.first) * eb;
        uint8_t* h = pinned ? b->mirror + b->moff[f] + lo * eb : host + (lo - first) * eb;
        const int rc = move_piece(s.d, dev, h, (hi - lo) * eb, up, pinned);
        if (rc != CLS_OK) return relay(e, s.d, rc);
    }
    for (BatchShard& s : b->sh) HIPC(e, hipStreamSynchronize(s.d->stream));
    return CLS_OK;
}

cls_pkt_soa shard_soa(const cls_batch* b, const BatchShard& s) {
    cls_pkt_soa p;
    std::memset(&p, 0, sizeof p);
    p.af = b->af;
    if (b->af == CLS_AF_V16) {
        p.src16 = fld<uint8_t>(s, CLS_BF_SRC);
        p.dst16 = fld<uint8_t>(s, CLS_BF_DST);
    } else {
        p.src4 = fld<uint32_t>(s, CLS_BF_SRC);
        p.dst4 = fld<uint32_t>(s, CLS_BF_DST);
    }
    p.sport = fld<uint16_t>(s, CLS_BF_SPORT);
    p.dport = fld<uint16_t>(s, CLS_BF_DPORT);
    p.proto = fld<uint8_t>(s, CLS_BF_PROTO);
    return p;
}

// The last classify's counters summed over the shards (waits for them).
int read_counters(cls_batch* b, std::vector<uint64_t>& out) {
    cls_engine* e = b->e;
    if (b->cur < 0) return fail(e, CLS_E_INVAL, "no cls_classify_batch on this batch yet");
    const int k = b->cur;
    out.assign(b->n_ctr, 0);
    std::vector<uint64_t> h(b->n_ctr);
    // after an all-reduce every device holds the total: read the first
    const size_t m = b->reduced ? 1 : b->sh.size();
    for (size_t i = 0; i < m; ++i) {
        BatchShard& s = b->sh[i];
        cls_engine* d = s.d;
        HIPC(e, hipSetDevice(d->device));
        if (b->reduced) {                        // behind the all-reduce, on its stream
            int rc = side_stream(d);
            if (rc != CLS_OK) return relay(e, d, rc);
            HIPC(e, hipStreamWaitEvent(d->coll, s.reduced[k], 0));
            HIPC(e, hipMemcpyAsync(h.data(), s.ctr[k].p, size_t(b->n_ctr) * 8, hipMemcpyDeviceToHost, d->coll));
            HIPC(e, hipStreamSynchronize(d->coll));
        } else {                                 // behind the classify, on the engine stream
            HIPC(e, hipMemcpyAsync(h.data(), s.ctr[k].p, size_t(b->n_ctr) * 8, hipMemcpyDeviceToHost, d->stream));
            HIPC(e, hipStreamSynchronize(d->stream));
        }
        for (size_t r = 0; r < h.size(); ++r) out[r] += h[r];
    }
    return CLS_OK;
}

}  // namespace

// ---- peers ---------------------------------------------------------------
// Mirror the primary's tables (host form copied, uploaded to the peer's
// device; never recompiled), a rebind's counter clearing and the interface
// bindings on every peer.  Called by the configuration entry points with the
// primary's lock held.
int sync_peers(cls_engine* e) {
    for (cls_engine* p : e->peers) {
        std::lock_guard<std::mutex> g(p->mu);
        if (p->synced_gen == e->conn_gen) continue;
        HIPC(e, hipSetDevice(p->device));
        bool dropped = false;
        for (auto it = p->tables.begin(); it != p->tables.end();) {
            if (!e->tables.count(it->first)) {
                it = p->tables.erase(it);
                dropped = true;
            } else {
                ++it;
            }
        }
        if (dropped) {                  // no kept plan may hold a deleted table's buffers
            (void)conn_quiesce(p);
            p->conn_plan = ConnPlan();
            p->up_plan = ~0ull;
        }
        for (const auto& kv : e->tables) {
            auto f = p->tables.find(kv.first);
            if (f == p->tables.end()) {
                std::shared_ptr<Table> t = table_clone_host(*kv.second);
                const int rc = table_upload(p, *t);
                if (rc != CLS_OK) return relay(e, p, rc);
                p->tables[kv.first] = t;
            } else if (f->second->conn_epoch != kv.second->conn_epoch) {
                Table& pt = *f->second;          // the primary's rebind cleared its counters
                if (pt.d_conn_ctr.p) {
                    HIPC(e, hipMemsetAsync(pt.d_conn_ctr.p, 0, size_t(pt.n_rules + 1) * 8, p->stream));
                    if (!pt.conn_ctr_ev) HIPC(e, hipEventCreateWithFlags(&pt.conn_ctr_ev, hipEventDisableTiming));
                    HIPC(e, hipEventRecord(pt.conn_ctr_ev, p->stream));
                }
                pt.conn_epoch = kv.second->conn_epoch;
            }
        }
        p->if_ids = e->if_ids;
        p->if_names = e->if_names;
        p->if_acl = e->if_acl;
        p->next_table = e->next_table;
        p->conn_gen = e->conn_gen;      // its connection plans see the change
        p->synced_gen = e->conn_gen;
    }
    return CLS_OK;
}

extern "C" {

int cls_engine_create(const cls_config* cfg, cls_engine** out) {
    const DeviceGuard dg;        // the caller's device again on return
    if (!out) return CLS_E_INVAL;
    *out = nullptr;
    std::vector<int> want;
    if (cfg && cfg->n_devices) {
        if (!cfg->devices) return CLS_E_INVAL;
        want.assign(cfg->devices, cfg->devices + cfg->n_devices);
    } else {
        want.push_back(cfg ? cfg->device : -1);
    }
    cls_engine* e = nullptr;
    int rc = engine_open(want[0], &e);
    if (rc != CLS_OK) return rc;
    std::unique_ptr<cls_engine, void (*)(cls_engine*)> guard(e, cls_engine_destroy);
    bool distinct = true;
    for (size_t i = 1; i < want.size() && rc == CLS_OK; ++i) {
        cls_engine* p = nullptr;
        rc = engine_open(want[i], &p);
        if (rc != CLS_OK) break;
        p->primary = e;
        e->peers.push_back(p);
        for (size_t j = 0; j < i; ++j) distinct = distinct && dev_engine(e, j)->device != p->device;
    }
    if (rc != CLS_OK) return rc;
    // distinct devices: the counter all-reduce over xGMI from the start.
    // Without RCCL (not loadable, or its init fails) the engine still runs
    // every device and sums the counters on the host (cls_comm_info: 0
    // ranks); cls_last_error keeps the reason, and an explicit cls_comm_init
    // reports CLS_E_RCCL.
    if (want.size() > 1 && distinct && comm_make(e, 1, 0, nullptr) != CLS_OK) {
        for (size_t i = 0; i < n_dev_engines(e); ++i) {
            cls_engine* d = dev_engine(e, i);
            d->comm = nullptr;
            d->comm_ranks = d->comm_rank = 0;
        }
        e->err = "no counter all-reduce (host-summed counters): " + e->err;
    }
    *out = guard.release();
    return CLS_OK;
}

void cls_engine_destroy(cls_engine* e) {
    const DeviceGuard dg;        // the caller's device again on return
    if (!e || e->primary) return;      // a peer belongs to its primary
    bool comm = false;
    for (size_t i = 0; i < n_dev_engines(e); ++i) comm = comm || dev_engine(e, i)->comm;
    if (comm) comm_release(e);
    for (cls_engine* p : e->peers) engine_close(p);
    e->peers.clear();
    engine_close(e);
}

int cls_engine_devices(const cls_engine* e, uint32_t* n_devices) {
    if (!e || !n_devices) return CLS_E_INVAL;
    *n_devices = uint32_t(n_dev_engines(e));
    return CLS_OK;
}

int cls_device_engine(cls_engine* e, uint32_t index, cls_engine** dev) {
    if (!e || !dev) return CLS_E_INVAL;
    if (index >= n_dev_engines(e)) return fail(e, CLS_E_INVAL, "no device %u", index);
    *dev = dev_engine(e, index);
    return CLS_OK;
}

int cls_shard_range(uint64_t n, uint32_t n_shards, uint32_t shard, uint64_t* first, uint64_t* count) {
    if (!first || !count || n_shards == 0 || shard >= n_shards) return CLS_E_INVAL;
    shard_of(n, n_shards, shard, *first, *count);
    return CLS_OK;
}

int cls_comm_unique_id(void* id128) {
    if (!id128) return CLS_E_INVAL;
    Rccl& r = rccl();
    if (!r.ok) return CLS_E_RCCL;
    ncclUniqueId uid;
    if (r.get_unique_id(&uid) != ncclSuccess) return CLS_E_RCCL;
    std::memcpy(id128, &uid, sizeof uid);
    return CLS_OK;
}

int cls_comm_init(cls_engine* e, uint32_t n_procs, uint32_t proc, const void* id128) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return fail(e, CLS_E_INVAL, "cls_comm_init: use the primary engine");
    PeerLocks pl(e);
    return comm_make(e, n_procs, proc, id128);
}

int cls_comm_info(cls_engine* e, uint32_t* n_ranks, uint32_t* rank0) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (n_ranks) *n_ranks = e->comm ? e->comm_ranks : 0;
    if (rank0) *rank0 = e->comm ? e->comm_rank : 0;
    return CLS_OK;
}

int cls_batch_create(cls_engine* e, uint32_t af, uint64_t n, uint32_t flags, cls_batch** out) {
    if (!e || !out) return CLS_E_INVAL;
    *out = nullptr;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return fail(e, CLS_E_INVAL, "create batches on the primary engine");
    if (af != CLS_AF_V4 && af != CLS_AF_V16) return fail(e, CLS_E_INVAL, "af must be CLS_AF_V4 or CLS_AF_V16");
    if (flags & ~uint32_t(CLS_BATCH_CONN | CLS_BATCH_MIRROR)) return fail(e, CLS_E_INVAL, "unknown batch flags");
    PeerLocks pl(e);
    auto b = std::make_unique<cls_batch>();
    b->e = e;
    b->af = af;
    b->flags = flags;
    b->n = n;
    const uint32_t G = uint32_t(n_dev_engines(e));
    b->sh = std::vector<BatchShard>(G);
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    for (uint32_t gi = 0; gi < G; ++gi) {
        BatchShard& s = b->sh[gi];
        s.d = dev_engine(e, gi);
        shard_of(n, G, gi, s.first, s.n);
        // One allocation; array f starts a further (f + 1) x 4352 B (4 KiB +
        // 256 B) past the previous one's 256-B aligned end, so the fields'
        // streams do not walk the same HBM channels in step: config 3's
        // kernel 0.550-0.552 ms against 0.564-0.566 ms packed back to back
        // and 0.553-0.560 ms with one allocation per field
        // (profiles/r05c_batch_layout_ab.txt).
        // Option batch_layout (measurement): 0 packed, 1 per field.
        const int layout = e->opts.batch_layout;
        size_t at = 0;
        HIPC(e, hipSetDevice(s.d->device));
        for (uint32_t f = 0; f < CLS_BF_COUNT; ++f) {
            if (!b->has(f)) continue;
            const size_t bytes = al(s.n * field_bytes(af, f) + 256);   // + 256: whole 16-B groups past the end
            if (layout == 1) {
                HIPC(e, s.fmem[f].ensure(bytes));
                continue;
            }
            s.off[f] = at;
            at += bytes + (layout == 2 ? 4352 * size_t(f + 1) : 0);
        }
        if (layout != 1) HIPC(e, s.mem.ensure(at));
        for (int k = 0; k < 2; ++k) {
            HIPC(e, hipEventCreateWithFlags(&s.classified[k], hipEventDisableTiming));
            HIPC(e, hipEventCreateWithFlags(&s.reduced[k], hipEventDisableTiming));
        }
    }
    if (flags & CLS_BATCH_MIRROR) {
        size_t at = 0;
        for (uint32_t f = 0; f < CLS_BF_COUNT; ++f) {
            if (!b->has(f)) continue;
            b->moff[f] = at;
            at += al(n * field_bytes(af, f));
        }
        HIPC(e, hipHostMalloc(reinterpret_cast<void**>(&b->mirror), std::max<size_t>(at, 256),
                              hipHostMallocPortable));
    }
    *out = b.release();
    return CLS_OK;
}

void cls_batch_destroy(cls_batch* b) {
    if (!b) return;
    cls_engine* e = b->e;
    {
        std::lock_guard<std::mutex> g(e->mu);
        const DeviceGuard dg;        // the caller's device again on return
        PeerLocks pl(e);
        // the shards' last readers first; their destructors free the events
        // and buffers on each shard's device
        for (BatchShard& s : b->sh) {
            (void)hipSetDevice(s.d->device);
            (void)hipStreamSynchronize(s.d->stream);
            if (s.d->coll) (void)hipStreamSynchronize(s.d->coll);
        }
        if (b->mirror) (void)hipHostFree(b->mirror);
        b->mirror = nullptr;
        b->sh.clear();
    }
    delete b;
}

int cls_batch_shards(const cls_batch* b, uint32_t* n_shards) {
    if (!b || !n_shards) return CLS_E_INVAL;
    *n_shards = uint32_t(b->sh.size());
    return CLS_OK;
}

int cls_batch_shard(const cls_batch* b, uint32_t shard, int* device, uint64_t* first, uint64_t* n) {
    if (!b || shard >= b->sh.size()) return CLS_E_INVAL;
    if (device) *device = b->sh[shard].d->device;
    if (first) *first = b->sh[shard].first;
    if (n) *n = b->sh[shard].n;
    return CLS_OK;
}

int cls_batch_field(cls_batch* b, uint32_t shard, uint32_t field, void** dev_ptr) {
    if (!b || !dev_ptr || shard >= b->sh.size() || field >= CLS_BF_COUNT || !b->has(field)) return CLS_E_INVAL;
    *dev_ptr = fld<uint8_t>(b->sh[shard], field);
    return CLS_OK;
}

int cls_batch_mirror(cls_batch* b, uint32_t field, void** host_ptr) {
    if (!b || !host_ptr || field >= CLS_BF_COUNT || !b->has(field) || !b->mirror) return CLS_E_INVAL;
    *host_ptr = b->mirror + b->moff[field];
    return CLS_OK;
}

int cls_batch_upload(cls_batch* b, uint32_t field, uint64_t first, uint64_t n, const void* src) {
    if (!b) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(b->e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    PeerLocks pl(b->e);
    return batch_move(b, field, first, n, const_cast<uint8_t*>(static_cast<const uint8_t*>(src)), true);
}

int cls_batch_download(cls_batch* b, uint32_t field, uint64_t first, uint64_t n, void* dst) {
    if (!b) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(b->e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    PeerLocks pl(b->e);
    return batch_move(b, field, first, n, static_cast<uint8_t*>(dst), false);
}

int cls_batch_gen_traffic_v4(cls_batch* b, const cls_traffic_spec* spec, uint64_t stream_first) {
    if (!b || !spec) return CLS_E_INVAL;
    cls_engine* e = b->e;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (b->af != CLS_AF_V4) return fail(e, CLS_E_INVAL, "cls_batch_gen_traffic_v4 on a 16-byte batch");
    PeerLocks pl(e);
    for (BatchShard& s : b->sh) {
        const int rc = gen4_locked(s.d, spec, stream_first + s.first, s.n, fld<uint32_t>(s, CLS_BF_SRC),
                                   fld<uint32_t>(s, CLS_BF_DST), fld<uint16_t>(s, CLS_BF_SPORT),
                                   fld<uint16_t>(s, CLS_BF_DPORT), fld<uint8_t>(s, CLS_BF_PROTO), nullptr, false);
        if (rc != CLS_OK) return relay(e, s.d, rc);
    }
    for (BatchShard& s : b->sh) HIPC(e, hipStreamSynchronize(s.d->stream));   // the pools are engine scratch
    return CLS_OK;
}

int cls_batch_gen_traffic_v16(cls_batch* b, const cls_traffic_spec16* spec, uint64_t stream_first) {
    if (!b || !spec) return CLS_E_INVAL;
    cls_engine* e = b->e;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (b->af != CLS_AF_V16) return fail(e, CLS_E_INVAL, "cls_batch_gen_traffic_v16 on an IPv4 batch");
    PeerLocks pl(e);
    for (BatchShard& s : b->sh) {
        const int rc = gen16_locked(s.d, spec, stream_first + s.first, s.n, fld<uint8_t>(s, CLS_BF_SRC),
                                    fld<uint8_t>(s, CLS_BF_DST), fld<uint16_t>(s, CLS_BF_SPORT),
                                    fld<uint16_t>(s, CLS_BF_DPORT), fld<uint8_t>(s, CLS_BF_PROTO), nullptr, false);
        if (rc != CLS_OK) return relay(e, s.d, rc);
    }
    for (BatchShard& s : b->sh) HIPC(e, hipStreamSynchronize(s.d->stream));
    return CLS_OK;
}

int cls_classify_batch(cls_engine* e, uint32_t table_id, cls_batch* b, uint64_t* counters_out, uint32_t flags) {
    if (!e || !b) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (b->e != e) return fail(e, CLS_E_INVAL, "the batch belongs to another engine");
    auto it = e->tables.find(table_id);
    if (it == e->tables.end()) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    const uint32_t n_ctr = it->second->n_rules + 1;
    const uint32_t pass = flags & (CLS_F_NO_VERDICT | CLS_F_FORCE_LINEAR | CLS_F_TIMING);
    PeerLocks pl(e);
    const int k = b->cur < 0 ? 0 : (b->cur ^ 1);
    bool comm = true;
    for (BatchShard& s : b->sh) comm = comm && s.d->comm != nullptr;
    for (BatchShard& s : b->sh) {
        cls_engine* d = s.d;
        HIPC(e, hipSetDevice(d->device));
        if (s.ctr[k].bytes < size_t(n_ctr) * 8) {
            // a larger table: the buffer's last readers (its all-reduce) first
            if (s.rec_red[k]) HIPC(e, hipEventSynchronize(s.reduced[k]));
            if (s.rec_cls[k]) HIPC(e, hipEventSynchronize(s.classified[k]));
            HIPC(e, s.ctr[k].ensure(size_t(n_ctr) * 8));
        }
        if (s.rec_red[k]) HIPC(e, hipStreamWaitEvent(d->stream, s.reduced[k], 0));
        const cls_pkt_soa p = shard_soa(b, s);
        const int rc = classify_locked(d, table_id, &p, s.n, fld<uint8_t>(s, CLS_BF_VERDICT),
                                       s.ctr[k].as<uint64_t>(), pass | CLS_F_DEVICE, d->stream);
        if (rc != CLS_OK) return relay(e, d, rc);
        // the all-reduce's dependency (an event record costs the stream a
        // few microseconds: without a communicator the readers synchronise
        // the stream instead)
        if (comm) HIPC(e, hipEventRecord(s.classified[k], d->stream));
        s.rec_cls[k] = comm;
    }
    if (comm) {
        // every device's counters summed in place over xGMI (and over the
        // processes of cls_comm_init), on the side streams
        Rccl& r = rccl();
        for (BatchShard& s : b->sh) {
            HIPC(e, hipSetDevice(s.d->device));
            HIPC(e, hipStreamWaitEvent(s.d->coll, s.classified[k], 0));
        }
        RCCLC(e, r.group_start());
        for (BatchShard& s : b->sh) {
            const ncclResult_t rc = r.all_reduce(s.ctr[k].p, s.ctr[k].p, n_ctr, ncclUint64, ncclSum,
                                                 static_cast<ncclComm_t>(s.d->comm), s.d->coll);
            if (rc != ncclSuccess) {
                (void)r.group_end();
                return fail(e, CLS_E_RCCL, "ncclAllReduce: %s", r.error_string(rc));
            }
        }
        RCCLC(e, r.group_end());
        for (BatchShard& s : b->sh) {
            HIPC(e, hipSetDevice(s.d->device));
            HIPC(e, hipEventRecord(s.reduced[k], s.d->coll));
            s.rec_red[k] = true;
        }
    } else {
        for (BatchShard& s : b->sh) s.rec_red[k] = false;
    }
    b->cur = k;
    b->n_ctr = n_ctr;
    b->reduced = comm;
    if (!counters_out) return CLS_OK;
    std::vector<uint64_t> c;
    const int rc = read_counters(b, c);
    if (rc != CLS_OK) return rc;
    for (uint32_t i = 0; i < n_ctr; ++i)
        counters_out[i] = (flags & CLS_F_ACCUMULATE) ? counters_out[i] + c[i] : c[i];
    return CLS_OK;
}

int cls_batch_counters(cls_batch* b, uint64_t* out, uint32_t n_out) {
    if (!b || !out) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(b->e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    PeerLocks pl(b->e);
    if (b->cur >= 0 && n_out < b->n_ctr) return fail(b->e, CLS_E_INVAL, "counters need %u entries", b->n_ctr);
    std::vector<uint64_t> c;
    const int rc = read_counters(b, c);
    if (rc != CLS_OK) return rc;
    std::memcpy(out, c.data(), c.size() * 8);
    return CLS_OK;
}

int cls_batch_connect(cls_engine* e, cls_batch* b, uint32_t flags) {
    if (!e || !b) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (b->e != e) return fail(e, CLS_E_INVAL, "the batch belongs to another engine");
    if (!(b->flags & CLS_BATCH_CONN)) return fail(e, CLS_E_INVAL, "not a connection batch (CLS_BATCH_CONN)");
    PeerLocks pl(e);
    const uint32_t pass = flags & (CLS_F_FORCE_LINEAR | CLS_F_CONN_CLS | CLS_F_COUNT);
    for (BatchShard& s : b->sh) {
        cls_conn_soa c;
        c.pkt = shard_soa(b, s);
        c.src_if = fld<uint32_t>(s, CLS_BF_SRC_IF);
        c.dst_if = fld<uint32_t>(s, CLS_BF_DST_IF);
        const int rc = connect_locked(s.d, &c, s.n, fld<uint8_t>(s, CLS_BF_VERDICT), pass | CLS_F_DEVICE, s.d->stream,
                                      false);
        if (rc != CLS_OK) return relay(e, s.d, rc);
    }
    // stream-ordered on every shard's device: cls_batch_wait, cls_batch_download
    // and cls_conn_counters order behind it
    return CLS_OK;
}

int cls_batch_wait(cls_batch* b) {
    if (!b) return CLS_E_INVAL;
    cls_engine* e = b->e;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    PeerLocks pl(e);
    for (BatchShard& s : b->sh) {
        HIPC(e, hipSetDevice(s.d->device));
        HIPC(e, hipStreamSynchronize(s.d->stream));
        if (s.d->coll) HIPC(e, hipStreamSynchronize(s.d->coll));
    }
    return CLS_OK;
}

}  // extern "C"
