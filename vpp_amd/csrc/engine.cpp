// C ABI of the classifier engine (include/contivcls.h).
//
// Host side of the MI355X verdict backend: ACL configuration (the
// MockACLEngine's ACLConfig, mock/aclengine/aclengine_mock.go:110-121,
// 671-728), table compilation + upload, and the launch sequence of the
// classify / connection / traffic kernels on one gfx950 device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/contivcls.h"
#include "compile.hpp"
#include "engine_int.hpp"
#include "kernels.hpp"

using namespace cls;

// OTHER queue (protocols > 2 deferred to the finish launch): per workgroup
// room for 1/16 of its packets, at most 16 Ki entries (64 KiB per workgroup:
// the queue exists per (table, stream), and a full segment classifies in
// place, so a cap costs only speed on batches with > 6 % protocol > 2),
// split into one segment per wave (kOtherSegs): the entries per segment.
// Option other_cap (per workgroup): tests, to reach the in-place path.
static uint32_t other_cap(const cls_engine* e, uint64_t n, int grid) {
    if (e->opts.other_cap) return e->opts.other_cap / kOtherSegs;
    const uint64_t want = (n / uint64_t(std::max(grid, 1)) + 15) / 16;
    return uint32_t(std::min<uint64_t>(16384, std::max<uint64_t>(1024, want))) / kOtherSegs;
}

static int acl_put_locked(cls_engine* e, const char* acl_name, const cls_rule* rules, uint32_t n_rules,
                          const char* const* ingress_ifs, uint32_t n_ingress, const char* const* egress_ifs,
                          uint32_t n_egress);

extern "C" {

int cls_abi_version(void) { return CLS_ABI_VERSION; }

int cls_image_kernel(uint32_t mode, uint32_t list_mode, int lds_resident, int rep16) {
    return cls_kernel_exists(mode, list_mode, lds_resident != 0, rep16 != 0) ? CLS_OK : CLS_E_INVAL;
}

}  // extern "C"

// One device's engine (cls_engine_create, fleet.cpp, builds multi-device
// engines from these).  device < 0: the current device.
int engine_open(int dev, cls_engine** out) {
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CLS_E_NODEV;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return CLS_E_NODEV;
    if (dev >= ndev) return CLS_E_NODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return CLS_E_NODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CLS_E_NODEV;
    auto* e = new (std::nothrow) cls_engine();
    if (!e) return CLS_E_NOMEM;
    e->device = dev;
    e->n_cu = prop.multiProcessorCount;
    // The engine's stream (a call's stream == NULL) is a blocking stream: work
    // on the legacy default stream (torch's current stream unless the caller
    // set another) and the engine's calls stay ordered both ways.
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamDefault) != hipSuccess) {
        delete e;
        return CLS_E_HIP;
    }
    *out = e;
    return CLS_OK;
}

// Waits for the engine's device work (its streams only: other engines and
// torch streams on the device are not waited for), then frees it.
void engine_close(cls_engine* e) {
    (void)hipSetDevice(e->device);
    (void)conn_quiesce(e);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->coll) (void)hipStreamSynchronize(e->coll);
    e->conn_plan = ConnPlan();
    e->tables.clear();                 // each table's Counters wait for their streams' work
    for (auto& pr : e->ev_pool) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (int k = 0; k < 2; ++k) {
        if (e->stage_ev[k]) (void)hipEventDestroy(e->stage_ev[k]);
        if (e->stage[k]) (void)hipHostFree(e->stage[k]);
    }
    if (e->coll) (void)hipStreamDestroy(e->coll);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

extern "C" {

const char* cls_last_error(const cls_engine* e) { return e ? e->err.c_str() : "null engine"; }


// ---------------------------------------------------------------------------
// The slot -> rule map of a table variant as the remap kernel reads it: every
// slot once, grouped by rule (slot order within a rule).
// Slots: the main image's, the OTHER image's, then one per rule plus the
// default DENY (the linear kernel's).
static int counters_init(cls_engine* e, Counters& c, const Cls4Image* img, const Cls4Image* oimg,
                         uint32_t n_rules) {
    const uint32_t n_cls = img ? img->n_ctr : 0, n_oth = oimg ? oimg->n_ctr : 0;
    c.n_slots = n_cls + n_oth + n_rules + 1;
    c.n_lctr = img ? img->n_lctr : 0;
    c.n_image = n_cls + n_oth;
    std::vector<uint32_t> cnt(size_t(n_rules) + 2, 0);
    auto rule_of = [&](uint32_t i) {
        return i < n_cls ? img->ctr_rule[i] : i < n_cls + n_oth ? oimg->ctr_rule[i - n_cls] : i - n_cls - n_oth;
    };
    for (uint32_t i = 0; i < c.n_slots; ++i) cnt[rule_of(i) + 1]++;
    for (size_t r = 1; r < cnt.size(); ++r) cnt[r] += cnt[r - 1];
    std::vector<uint32_t> csr(size_t(c.n_slots) * 2);
    for (uint32_t i = 0; i < c.n_slots; ++i) {
        const uint32_t r = rule_of(i), k = cnt[r]++;
        csr[2 * size_t(k)] = i;
        csr[2 * size_t(k) + 1] = r;
    }
    HIPC(e, c.d_csr.ensure(csr.size() * 4));
    HIPC(e, hipMemcpy(c.d_csr.p, csr.data(), csr.size() * 4, hipMemcpyHostToDevice));
    // slot -> rule for the finish launch.  Rules owning many slots (default
    // DENY: one no-match slot per cell; allow-all rules: one per class) are
    // "hot": a tile sums them in LDS, so such a rule takes one atomic per
    // tile instead of one per slot.
    std::vector<std::pair<uint32_t, uint32_t>> mult;            // (slots, rule)
    for (uint32_t r = 0; r <= n_rules; ++r) {
        const uint32_t m = cnt[r] - (r ? cnt[r - 1] : 0u);      // cnt[r] is now the end of rule r's run
        if (m >= 8) mult.push_back({m, r});
    }
    std::sort(mult.begin(), mult.end(), [](const auto& a, const auto& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    if (mult.size() > kMaxHotRules) mult.resize(kMaxHotRules);
    std::vector<uint32_t> hot_of(size_t(n_rules) + 1, 0xFFFFFFFFu);
    for (uint32_t h = 0; h < mult.size(); ++h) hot_of[mult[h].second] = h;
    std::vector<uint32_t> sr(size_t(c.n_slots) + mult.size());
    for (uint32_t i = 0; i < c.n_slots; ++i) {
        const uint32_t r = rule_of(i);
        sr[i] = hot_of[r] != 0xFFFFFFFFu ? (kHotRule | hot_of[r]) : r;
    }
    for (uint32_t h = 0; h < mult.size(); ++h) sr[c.n_slots + h] = mult[h].second;
    c.n_hot = uint32_t(mult.size());
    HIPC(e, c.d_slot_rule.ensure(sr.size() * 4));
    HIPC(e, hipMemcpy(c.d_slot_rule.p, sr.data(), sr.size() * 4, hipMemcpyHostToDevice));
    // The OTHER slots' rules, numbered compactly: the finish launch counts
    // the queued OTHER packets per rule in LDS and adds one total per
    // (workgroup, rule).  (Per slot would put many slots of one rule -- a
    // TestTraffic list's sentinel -- on one counter word from every
    // workgroup.)
    c.n_other = n_oth;
    std::vector<uint32_t> om(n_oth), orules;
    std::map<uint32_t, uint32_t> cidx;
    for (uint32_t k = 0; k < n_oth; ++k) {
        const uint32_t r = rule_of(n_cls + k);
        auto it = cidx.find(r);
        if (it == cidx.end()) {
            it = cidx.emplace(r, uint32_t(orules.size())).first;
            orules.push_back(r);
        }
        om[k] = it->second;
    }
    c.n_orules = uint32_t(orules.size());
    om.insert(om.end(), orules.begin(), orules.end());
    HIPC(e, c.d_other_map.ensure(std::max<size_t>(1, om.size()) * 4));
    if (!om.empty()) HIPC(e, hipMemcpy(c.d_other_map.p, om.data(), om.size() * 4, hipMemcpyHostToDevice));
    return CLS_OK;
}

// slot -> rule of an image and its OTHER image (slot mode of the classify
// kernels: OTHER slots follow the main image's)
static int upload_slot_rule(cls_engine* e, DevBuf& d, const Cls4Image& img, const Cls4Image& oimg) {
    std::vector<uint32_t> m(img.ctr_rule.begin(), img.ctr_rule.end());
    m.insert(m.end(), oimg.ctr_rule.begin(), oimg.ctr_rule.end());
    HIPC(e, d.ensure(std::max<size_t>(1, m.size()) * 4));
    if (!m.empty()) HIPC(e, hipMemcpy(d.p, m.data(), m.size() * 4, hipMemcpyHostToDevice));
    return CLS_OK;
}

// The rules as the caller gave them, serialised (NULL network = ""): two
// puts with equal signatures compile to the same table.
static std::string rule_sig(const cls_rule* rules, uint32_t n) {
    std::string sg;
    sg.reserve(size_t(n) * 80);
    for (uint32_t k = 0; k < n; ++k) {
        const cls_rule& r = rules[k];
        const uint32_t w[14] = {r.flags, uint32_t(r.acl_action), r.tcp_src_lo, r.tcp_src_hi, r.tcp_dst_lo,
                                r.tcp_dst_hi, r.udp_src_lo, r.udp_src_hi, r.udp_dst_lo, r.udp_dst_hi,
                                r.icmp_code_first, r.icmp_code_last, r.icmp_type_first, r.icmp_type_last};
        sg.append(reinterpret_cast<const char*>(w), sizeof w);
        sg.append(r.src_network ? r.src_network : "");
        sg.push_back('\0');
        sg.append(r.dst_network ? r.dst_network : "");
        sg.push_back('\0');
    }
    return sg;
}

// The main classifier of a rule set and its OTHER image (protocols > 2), in
// the main image's orientation.
static bool build_pair(const std::vector<SemRule>& sem, uint32_t n, Cls4Image& img, Cls4Image& oimg,
                       std::string& why) {
    if (!build_cls4(sem, n, img, why)) return false;
    return build_other4(img.swap ? swap_sides(sem) : sem, n, oimg, why);
}

// The image, then (list modes 5, 6) its wide cells right after it: the
// kernel stages [0, img_bytes) into LDS and reads the cells from global memory.
static int upload(cls_engine* e, DevBuf& d, const Cls4Image& im) {
    const size_t gb = im.gcells.size() * 4;
    HIPC(e, d.ensure(im.img_bytes + gb));
    HIPC(e, hipMemcpy(d.p, im.words.data(), im.img_bytes, hipMemcpyHostToDevice));
    if (gb) HIPC(e, hipMemcpy(static_cast<uint8_t*>(d.p) + im.img_bytes, im.gcells.data(), gb, hipMemcpyHostToDevice));
    return CLS_OK;
}

// The counter scratch of (table variant, stream), created on first use.
static int scratch_of(cls_engine* e, Counters& c, uint32_t n_rules, hipStream_t s, Scratch** out);

}  // extern "C"

// A table's host form: the rules compiled once (evalACL semantics, both
// layouts, the connection path's compact rules).  No device work, so a
// multi-device engine compiles each table once and uploads it per device.
static int table_compile(cls_engine* e, const char* name, const cls_rule* rules, uint32_t n,
                         std::shared_ptr<Table>& out) {
    if (n && !rules) return fail(e, CLS_E_INVAL, "rules is NULL");
    const CompileScope scope(e->opts);      // the engine's compiler options
    auto t = std::make_shared<Table>();
    t->name = name ? name : "";
    t->n_rules = n;
    t->sig = rule_sig(rules, n);
    std::vector<SemRule> sem;
    std::string why;
    int rc = semantic_rules(rules, n, 4, sem, why);
    if (rc != CLS_OK) return fail(e, rc, "%s", why.c_str());
    t->lin4 = linear4(sem);
    t->conn4 = conn_rules4(sem);
    // classifier for anything but tiny tables
    t->kernel = 0;
    if (sem.size() > 8 && build_pair(sem, n, t->img, t->oimg, why)) {
        t->has_cls = true;
        t->kernel = 1;
        t->lds_resident = t->img.lds_ok && t->img.lds_bytes + kLdsReserved <= uint32_t(max_lds_bytes());
        if (t->img.h_bounds == t->oimg.h_bounds && t->img.h_iclass == t->oimg.h_iclass && t->img.row_bytes)
            t->pair_cdiv = uint32_t(((1ull << 32) + t->img.row_bytes - 1) / t->img.row_bytes);
        // the trie and wide cells exist only in LDS-resident images
        if (!cls_kernel_exists(t->img.mode, t->img.list_mode, t->lds_resident, false))
            return fail(e, CLS_E_INVAL, "no classify kernel for the compiled image (mode %u, list mode %u%s)",
                        t->img.mode, t->img.list_mode, t->lds_resident ? "" : ", global memory");
    }
    if (t->has_cls && t->lds_resident) t->sem4 = std::make_shared<const std::vector<SemRule>>(sem);
    // 16-byte layout: both families' reductions over one rep space
    auto& q = t->p16;
    std::vector<SemRule> s16;
    rc = semantic_rules(rules, n, 0, s16, why);
    if (rc != CLS_OK) return fail(e, rc, "%s", why.c_str());
    t->conn16 = conn_rules16(s16);
    std::string why16;
    q.ok = build_cls16(s16, n, q.img, why16) && build_other4(q.img.sem, n, q.oimg, why16);
    q.why = why16;
    if (q.ok) {
        const Cls4Image& c = q.img.core;
        q.lin = linear4(q.img.sem);
        q.lds_resident = c.lds_ok && c.lds_bytes + kLdsReserved <= uint32_t(max_lds_bytes());
        if (!cls_kernel_exists(c.mode, c.list_mode, q.lds_resident, true))
            return fail(e, CLS_E_INVAL, "no 16-byte classify kernel for the compiled image (mode %u, list mode %u%s)",
                        c.mode, c.list_mode, q.lds_resident ? "" : ", global memory");
    }
    out = std::move(t);
    return CLS_OK;
}

std::shared_ptr<Table> table_clone_host(const Table& s) {
    auto t = std::make_shared<Table>();
    t->name = s.name;
    t->n_rules = s.n_rules;
    t->sig = s.sig;
    t->lin4 = s.lin4;
    t->has_cls = s.has_cls;
    t->img = s.img;
    t->oimg = s.oimg;
    t->pair_cdiv = s.pair_cdiv;
    t->sem4 = s.sem4;                   // (the pair image is built per device, at first use)
    t->kernel = s.kernel;
    t->lds_resident = s.lds_resident;
    t->p16.ok = s.p16.ok;
    t->p16.why = s.p16.why;
    t->p16.img = s.p16.img;
    t->p16.lin = s.p16.lin;
    t->p16.oimg = s.p16.oimg;
    t->p16.lds_resident = s.p16.lds_resident;
    t->conn4 = s.conn4;
    t->conn16 = s.conn16;
    t->conn_bm = s.conn_bm;
    t->conn_bm_built = s.conn_bm_built;
    t->conn_epoch = s.conn_epoch;
    return t;
}

// The device copies of a compiled table on this engine's device.
int table_upload(cls_engine* e, Table& t) {
    HIPC(e, hipSetDevice(e->device));
    HIPC(e, t.d_lin4.ensure(std::max<size_t>(1, t.lin4.size()) * sizeof(LinRule4)));
    if (!t.lin4.empty())
        HIPC(e, hipMemcpy(t.d_lin4.p, t.lin4.data(), t.lin4.size() * sizeof(LinRule4), hipMemcpyHostToDevice));
    int rc = CLS_OK;
    if (t.has_cls) {
        rc = upload(e, t.d_img, t.img);
        if (rc == CLS_OK) rc = upload(e, t.d_oimg, t.oimg);
        if (rc == CLS_OK) rc = upload_slot_rule(e, t.d_slot_rule, t.img, t.oimg);
        if (rc != CLS_OK) return rc;
    }
    rc = counters_init(e, t.c4, t.has_cls ? &t.img : nullptr, t.has_cls ? &t.oimg : nullptr, t.n_rules);
    if (rc != CLS_OK) return rc;
    auto& q = t.p16;
    if (q.ok) {
        const Cls4Image& c = q.img.core;
        rc = upload(e, q.d_img, c);
        if (rc == CLS_OK) rc = upload(e, q.d_oimg, q.oimg);
        if (rc == CLS_OK) rc = upload_slot_rule(e, q.d_slot_rule, c, q.oimg);
        if (rc != CLS_OK) return rc;
        HIPC(e, q.d_lin.ensure(std::max<size_t>(1, q.lin.size()) * sizeof(LinRule4)));
        if (!q.lin.empty())
            HIPC(e, hipMemcpy(q.d_lin.p, q.lin.data(), q.lin.size() * sizeof(LinRule4), hipMemcpyHostToDevice));
        rc = counters_init(e, t.c16, &c, &q.oimg, t.n_rules);
        if (rc != CLS_OK) return rc;
        if (q.img.src_mode >= 1) {
            HIPC(e, q.d_src_search.ensure(q.img.src_search.size() * 4));
            HIPC(e, hipMemcpy(q.d_src_search.p, q.img.src_search.data(), q.img.src_search.size() * 4,
                              hipMemcpyHostToDevice));
        }
    }
    return CLS_OK;
}

extern "C" {

// Configuration calls are made on the primary engine; a peer (a device of a
// multi-device engine, cls_device_engine) mirrors it.
static int refuse_peer(cls_engine* e) {
    return fail(e, CLS_E_INVAL, "configure a multi-device engine through its primary engine");
}

// Diagnostics and tests: one tuning switch (options.hpp) on the engine and,
// for a multi-device engine, on every device's engine.
int cls_engine_set_option(cls_engine* e, const char* key, const char* value) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    std::string why;
    Opts o = e->opts;
    if (!opts_set(o, key, value, why)) return fail(e, CLS_E_INVAL, "%s", why.c_str());
    e->opts = o;
    for (cls_engine* p : e->peers) {
        std::lock_guard<std::mutex> gp(p->mu);
        p->opts = o;
    }
    // a kept connection plan was made under the old options
    e->conn_gen++;
    return sync_peers(e);
}

// A table (or a dropped binding) is gone: the kept connection plan must not
// hold its device buffers until the next device batch replans.
static void drop_conn_plan(cls_engine* e) {
    (void)conn_quiesce(e);          // a stream-ordered batch may still read the plan's tables
    e->conn_plan = ConnPlan();
    e->up_plan = ~0ull;
}

static int table_put_locked(cls_engine* e, const char* name, const cls_rule* rules, uint32_t n,
                            uint32_t* table_id) {
    std::shared_ptr<Table> t;
    int rc = table_compile(e, name, rules, n, t);
    if (rc == CLS_OK) rc = table_upload(e, *t);
    if (rc != CLS_OK) return rc;
    const uint32_t id = e->next_table++;
    e->tables[id] = t;
    e->conn_gen++;                  // connection plans see the change
    if (table_id) *table_id = id;
    return CLS_OK;
}

int cls_table_put(cls_engine* e, const char* name, const cls_rule* rules, uint32_t n_rules,
                  uint32_t* table_id) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    const int rc = table_put_locked(e, name, rules, n_rules, table_id);
    return rc == CLS_OK ? sync_peers(e) : rc;
}

int cls_table_del(cls_engine* e, uint32_t table_id) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    HIPC(e, hipSetDevice(e->device));
    if (!e->tables.erase(table_id)) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    e->conn_gen++;                  // connection plans see the change
    drop_conn_plan(e);
    return sync_peers(e);
}

int cls_table_get_info(cls_engine* e, uint32_t table_id, cls_table_info* info) {
    if (!e || !info) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    auto it = e->tables.find(table_id);
    if (it == e->tables.end()) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    const Table& t = *it->second;
    std::memset(info, 0, sizeof *info);
    info->n_rules = t.n_rules;
    info->kernel = uint32_t(t.kernel);
    if (t.has_cls) {
        info->lds_bytes = t.img.lds_bytes;
        info->n_intervals = t.img.n_bounds;
        info->n_classes = t.img.n_classes;
        info->n_templates = t.img.n_tmpl;
        info->n_slots = t.img.n_ctr;
        info->lds_resident = t.lds_resident ? 1 : 0;
        info->n_lctr = t.img.n_lctr;
        info->ctr16 = t.img.ctr16;
        info->list_mode = t.img.list_mode;
        info->swap = t.img.swap;
    }
    info->has_v16 = t.p16.ok ? 1u : 0u;
    if (t.p16.ok) {
        info->lds_bytes_v16 = t.p16.img.core.lds_bytes;
        info->lds_resident_v16 = t.p16.lds_resident ? 1u : 0u;
    }
    return CLS_OK;
}

// ---------------------------------------------------------------------------
constexpr uint64_t kClsChunk = 1ull << 30;   // packets per classify launch (32-bit offsets)
constexpr uint64_t kConnClsMinBatch = 1ull << 16;  // connection batches that use the classifier images
constexpr uint32_t kConnClsMinRules = 64;          // ACLs evaluated by the classifier in connection batches
constexpr uint32_t kConnClsWork = 2048;            // ... when touches x rules >= this x batch size (host batch)
constexpr uint32_t kConnClsDevRules = 2048;        // ... when it has this many rules (device batch)
constexpr uint32_t kConnBmMinRules = 8;            // linear IPv4 ACLs given the bitmap form (conn_bitmap4) ...
constexpr size_t kConnBmMaxWords = 12288;          // ... when their tables take at most 48 KiB

static bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

// The event pair of a timed call (CLS_F_TIMING): stamped by the classify
// launch itself -- start of its first chunk's kernel, end of its last one's
// (hipExtLaunchKernel, part of the dispatch: no marker packets between the
// kernels, which cost a step several microseconds each) -- or recorded around
// the call when it has no classify launch.
static int timing_pair(cls_engine* e) {
    if (e->ev_used == e->ev_pool.size()) {
        hipEvent_t a, b;
        HIPC(e, hipEventCreate(&a));
        HIPC(e, hipEventCreate(&b));
        e->ev_pool.push_back({a, b});
    }
    e->ev0 = e->ev_pool[e->ev_used].first;
    e->ev1 = e->ev_pool[e->ev_used].second;
    e->ev_used++;
    return CLS_OK;
}

static Cls4Dev cls4_dev(const Cls4Image& im, const DevBuf& d_img, const DevBuf& d_lin, uint32_t n_lin,
                        uint32_t n_rules) {
    Cls4Dev cd;
    cd.img = d_img.as<uint32_t>();
    cd.img_bytes = im.img_bytes;
    cd.off_bounds = im.off_bounds;
    cd.off_iclass = im.off_iclass;
    cd.off_cells = im.off_cells;
    cd.off_lists = im.off_lists;
    cd.off_tmpl = im.off_tmpl;
    cd.search_top = im.search_top;
    cd.n_ctr = im.n_ctr;
    cd.lds_bytes = im.lds_bytes;
    cd.lin = d_lin.as<LinRule4>();
    cd.n_lin = n_lin;
    cd.n_rules = n_rules;
    cd.mode = im.mode;
    cd.default_row = im.default_row;
    cd.row_bytes = im.row_bytes;
    cd.port_mul = im.port_mul;
    cd.port_mask4 = im.port_mask4;
    cd.port_dflt = im.port_dflt;
    cd.n_hash = im.n_hash;
    cd.list_mode = im.list_mode;
    cd.bv_steps = std::max(im.bv_steps_d, im.bv_steps_p);  // mode 2: Sd
    cd.n_hot = im.n_hot;
    cd.off_ptop = im.off_ptop;
    cd.bv_wide = im.bv_wide;
    cd.off_hot = im.off_hot;
    cd.n_lctr = im.n_lctr;
    cd.ctr16 = im.ctr16;
    cd.off_trie = im.off_trie;
    cd.trie_depth = im.trie_depth;
    cd.gcells = im.gcells.empty() ? nullptr
                                  : reinterpret_cast<const uint8_t*>(d_img.p) + im.img_bytes;   // upload()
    cd.part = nullptr;
    cd.oq = nullptr;                 // protocols > 2 classified in place unless the caller sets a queue
    cd.oq_cap = 0;
    for (uint32_t i = 0; i < kMaxHashLens; ++i) {
        cd.hash_mask[i] = im.hash_mask[i];
        cd.hash_shift[i] = im.hash_shift[i];
        cd.hash_cap[i] = im.hash_cap[i];
        cd.hash_mul[i] = im.hash_mul[i];
        cd.hash_shift1[i] = 32u - 2u * (32u - im.hash_shift[i]);
        cd.off_hash[i] = im.off_hash[i];
    }
    return cd;
}

// The v4 classifier of a table (its kernel never reads the linear rules:
// every protocol has a cell).
static Cls4Dev table_dev(const Table& t) { return cls4_dev(t.img, t.d_img, DevBuf(), 0, t.n_rules); }

// The pair launch's image of a table (Table::pimg), built and uploaded at
// its first use; false when the table has none.
static bool pair_image(cls_engine* e, Table& t) {
    if (t.pimg_state == 0) {
        t.pimg_state = -1;
        std::string why;
        const CompileScope scope(e->opts);
        if (t.sem4 && build_pair4(*t.sem4, t.n_rules, t.img.swap != 0, t.pimg, why) && t.pimg.gcells.empty() &&
            t.pimg.img_bytes + 32u <= uint32_t(max_lds_bytes()) &&
            cls_kernel_exists(t.pimg.mode, t.pimg.list_mode, true, false) &&
            upload(e, t.d_pimg, t.pimg) == CLS_OK) {
            const std::vector<uint32_t>& m = t.pimg.ctr_rule;
            if (t.d_pslot_rule.ensure(std::max<size_t>(1, m.size()) * 4) == hipSuccess &&
                (m.empty() || hipMemcpy(t.d_pslot_rule.p, m.data(), m.size() * 4, hipMemcpyHostToDevice) == hipSuccess))
                t.pimg_state = 1;
            // ... and as u16 for the launch to stage in LDS beside the image
            t.pslot16_n16 = 0;
            if (t.pimg_state > 0 && t.n_rules < 0xFFFFu && !m.empty()) {
                std::vector<uint16_t> m16((m.size() + 7) & ~size_t(7), 0);
                for (size_t i = 0; i < m.size(); ++i) m16[i] = uint16_t(m[i]);
                if (t.d_pslot16.ensure(m16.size() * 2) == hipSuccess &&
                    hipMemcpy(t.d_pslot16.p, m16.data(), m16.size() * 2, hipMemcpyHostToDevice) == hipSuccess)
                    t.pslot16_n16 = uint32_t(m16.size() / 8);
            }
        }
        if (t.pimg_state < 0) {
            t.pimg = Cls4Image();
            (void)hipGetLastError();
        }
    }
    return t.pimg_state > 0;
}

// Packets in an image's frame: src and dst exchanged for a destination-keyed one.
static Pkts4 framed(const Cls4Image& im, const Pkts4& p) {
    return im.swap ? Pkts4{p.dst, p.src, p.dport, p.proto, p.n} : p;
}

// Workgroups of a classify launch: persistent grid, as many per CU as LDS
// and threads allow, no more than the batch needs.
static int cls_grid(const cls_engine* e, bool use_cls, bool lds_resident, uint32_t lds_bytes, uint64_t n) {
    int per_cu = 2;
    if (use_cls) {
        const int by_threads = 2048 / cls_block();
        per_cu = by_threads;
        // LDS-resident images: one 1024-thread workgroup per CU, also when two
        // would fit -- half the image stagings and counter rows, and the
        // stream runs faster in that shape (config 2: 0.0363 against 0.0392
        // ms, profiles/r04d_bench_c2{_wg1,}.json; the config-3 stream floor
        // 0.519 against 0.538 ms)
        if (lds_resident) per_cu = 1;
        if (e->opts.wg_per_cu > 0)   // diagnostics
            per_cu = std::max(1, std::min(by_threads, e->opts.wg_per_cu));
    }
    const uint64_t want = (n + 4ull * 1024 - 1) / (4ull * 1024);
    return int(std::max<uint64_t>(1, std::min<uint64_t>(uint64_t(e->n_cu) * per_cu, want)));
}

static int scratch_of(cls_engine* e, Counters& c, uint32_t n_rules, hipStream_t s, Scratch** out) {
    auto& p = c.sc[s];
    if (!p) {
        auto q = std::make_unique<Scratch>();
        HIPC(e, q->slot_val.ensure(size_t(c.n_slots) * 8));
        HIPC(e, hipMemsetAsync(q->slot_val.p, 0, size_t(c.n_slots) * 8, s));
        HIPC(e, q->out.ensure(size_t(n_rules + 1) * 8));
        // rows for the largest grid (cls_grid): never reallocated under pending work
        HIPC(e, q->part.ensure(size_t(e->n_cu) * (2048 / cls_block()) * std::max<uint32_t>(1, c.n_lctr) * 4));
        p = std::move(q);
    }
    *out = p.get();
    return CLS_OK;
}

// The OTHER queue of a launch of `grid` workgroups with segments of `cap`.
static int other_queue(cls_engine* e, Scratch* sc, int grid, uint32_t cap, hipStream_t s, uint32_t** out) {
    const size_t need = (size_t(grid) * kOtherSegs * (1 + size_t(cap))) * 4;
    if (need > sc->oq.bytes) {
        HIPC(e, hipStreamSynchronize(s));       // earlier launches on this stream may still read it
        HIPC(e, sc->oq.ensure(need));
    }
    *out = sc->oq.as<uint32_t>();
    return CLS_OK;
}

// Where a call's rule counters go, and whether they start from zero.
struct CountOut {
    unsigned long long* out;       // device rule counters (the caller's or the scratch's)
    bool zero;                     // cleared by the first fold launch
};
static CountOut count_out(Scratch* sc, uint64_t* counters_out, uint32_t flags) {
    const bool dev = flags & CLS_F_DEVICE;
    if (dev && counters_out)
        return {reinterpret_cast<unsigned long long*>(counters_out), !(flags & CLS_F_ACCUMULATE)};
    return {sc->out.as<unsigned long long>(), true};   // host batches accumulate on the host
}

// The finish launch of a classify chunk (kernels.hpp FinishArgs): fold the
// workgroups' partials, and on the last chunk move every slot to its rule.
static FinishArgs finish_args(const cls_engine* e, const Counters& c, Scratch* sc, const Cls4Dev& cd,
                              const CountOut& co, bool lds_resident, uint32_t rows, bool last) {
    FinishArgs f;
    f.part = lds_resident ? sc->part.as<uint32_t>() : nullptr;
    f.rows = rows;
    f.n_lctr = c.n_lctr;
    f.slot_val = sc->slot_val.as<unsigned long long>();
    f.n_slots = c.n_slots;
    f.slot_rule = c.d_slot_rule.as<uint32_t>();
    f.n_hot = c.n_hot;
    f.out = co.out;
    f.remap = last;
    f.oq = cd.oq;
    f.oq_rows = rows;
    f.oq_cap = cd.oq_cap;
    f.other_map = c.d_other_map.as<uint32_t>();
    f.n_other = c.n_other;
    f.n_orules = c.n_orules;
    // a tile's rows over several blocks where the tiles alone leave CUs idle
    // (option fold_split=0: one block per tile)
    const uint32_t tiles = (c.n_slots + 63u) / 64u;
    if (last && f.part && tiles && e->opts.fold_split)
        f.split = std::max(1u, std::min((rows + 63u) / 64u, uint32_t(e->n_cu) / tiles));
    return f;
}

// Slot counters -> rule counters (remap, which also clears the slots);
// host batches: copy verdicts and counters back.
static int finish_counts(cls_engine* e, const Table& t, const Counters& c, Scratch* sc, const CountOut& co,
                         uint64_t n, uint8_t* verdict_out, const uint8_t* d_verdict, uint64_t* counters_out,
                         uint32_t flags, hipStream_t s, bool remapped = false) {
    const bool dev = flags & CLS_F_DEVICE;
    if (!remapped) {
        HIPC(e, launch_remap(sc->slot_val.as<unsigned long long>(), c.d_csr.as<uint2>(), c.n_slots, co.out, s));
    }
    if (!dev) {
        if (verdict_out && n) HIPC(e, hipMemcpyAsync(verdict_out, d_verdict, n, hipMemcpyDeviceToHost, s));
        std::vector<uint64_t> tmp;
        if (counters_out) {
            tmp.resize(t.n_rules + 1);
            HIPC(e, hipMemcpyAsync(tmp.data(), co.out, tmp.size() * 8, hipMemcpyDeviceToHost, s));
        }
        HIPC(e, hipStreamSynchronize(s));
        if (counters_out) {
            for (size_t i = 0; i < tmp.size(); ++i)
                counters_out[i] = (flags & CLS_F_ACCUMULATE) ? counters_out[i] + tmp[i] : tmp[i];
        }
    }
    return CLS_OK;
}

static Fe16 fe16(const Cls16Image& m, const DevBuf& d_src_search) {
    Fe16 fe;
    std::memset(&fe, 0, sizeof fe);
    for (int sd = 0; sd < 2; ++sd) {
        fe.key[sd] = m.fe_key[sd];
        fe.val[sd] = m.fe_val[sd];
        fe.top[sd] = m.fe_top[sd];
        fe.k8[sd] = m.fe_k8[sd];
    }
    fe.src_mode = m.src_mode;
    if (m.src_mode == 1) {
        const uint32_t L4 = uint32_t(__builtin_ctz(m.cap4)), L6 = uint32_t(__builtin_ctz(m.cap6));
        fe.h4 = m.h4; fe.cap4 = m.cap4; fe.mul4 = m.mul4;
        fe.s4_0 = 32u - L4; fe.s4_1 = 32u - 2u * L4; fe.L4 = L4;
        fe.k6 = m.k6; fe.r6 = m.r6; fe.cap6 = m.cap6; fe.mul6 = m.mul6;
        fe.s6_0 = 32u - L6; fe.s6_1 = 32u - 2u * L6; fe.L6 = L6;
        for (int i = 0; i < 3; ++i) fe.fold[i] = m.fold[i];
        fe.dflt4 = m.dflt_row[0];
        fe.dflt6 = m.dflt_row[1];
    }
    if (m.src_mode >= 1) {                         // protocols > 2 need the rep: the global table
        fe.gsrc = d_src_search.as<uint8_t>();
        fe.gval = m.src_search_val;
        fe.gtop = m.src_search_top;
        fe.gk8 = m.src_search_k8;
    }
    return fe;
}

// cls_classify of a 16-byte batch (CLS_AF_V16): front end to reps, then the
// classifier over the rep-space rules (compile.hpp Cls16Image).
static int classify16_locked(cls_engine* e, std::shared_ptr<Table> t, const cls_pkt_soa* pk, uint64_t n,
                             uint8_t* verdict_out, uint64_t* counters_out, uint32_t flags, void* stream) {
    auto& q = t->p16;
    if (!q.ok) return fail(e, CLS_E_INVAL, "no 16-byte classifier for this table: %s", q.why.c_str());
    if (n && (!pk->src16 || !pk->dst16 || !pk->dport || !pk->proto))
        return fail(e, CLS_E_INVAL, "missing packet arrays");
    if (!verdict_out && !(flags & CLS_F_NO_VERDICT) && n)
        return fail(e, CLS_E_INVAL, "verdict_out is NULL (set CLS_F_NO_VERDICT)");
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    const bool dev = flags & CLS_F_DEVICE;
    const uint8_t *src = pk->src16, *dst = pk->dst16, *pr = pk->proto;
    const uint16_t* dp = pk->dport;
    uint8_t* d_verdict = verdict_out;
    if (dev && n && (!aligned(src, 16) || !aligned(dst, 16)))
        return fail(e, CLS_E_INVAL, "device src16/dst16 must be 16-byte aligned");
    if (!dev && n) {
        HIPC(e, e->s_src.ensure(n * 16));
        HIPC(e, e->s_dst.ensure(n * 16));
        HIPC(e, e->s_dport.ensure(n * 2));
        HIPC(e, e->s_proto.ensure(n));
        HIPC(e, hipMemcpyAsync(e->s_src.p, src, n * 16, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dst.p, dst, n * 16, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dport.p, dp, n * 2, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_proto.p, pr, n, hipMemcpyHostToDevice, s));
        src = e->s_src.as<uint8_t>();
        dst = e->s_dst.as<uint8_t>();
        dp = e->s_dport.as<uint16_t>();
        pr = e->s_proto.as<uint8_t>();
        d_verdict = nullptr;
        if (verdict_out) {
            HIPC(e, e->s_verdict.ensure(n));
            d_verdict = e->s_verdict.as<uint8_t>();
        }
    }
    Scratch* sc = nullptr;
    {
        const int rc = scratch_of(e, t->c16, t->n_rules, s, &sc);
        if (rc != CLS_OK) return rc;
    }
    const CountOut co = count_out(sc, counters_out, flags);
    unsigned long long* slot_val = sc->slot_val.as<unsigned long long>();
    const Cls4Image& c = q.img.core;
    const bool lin = flags & CLS_F_FORCE_LINEAR;
    LaunchCfg cfg;
    cfg.stream = s;
    cfg.grid = cls_grid(e, true, q.lds_resident, c.lds_bytes, n);
    const bool timing = flags & CLS_F_TIMING;
    if (timing) {
        const int rc = timing_pair(e);
        if (rc != CLS_OK) return rc;
        if (!n) HIPC(e, hipEventRecord(e->ev0, s));
    }
    bool zeroed = false, remapped = false;
    if (n) {
        Cls4Dev cd = cls4_dev(c, q.d_img, q.d_lin, uint32_t(q.lin.size()), t->n_rules);
        cfg.other = cls4_dev(q.oimg, q.d_oimg, DevBuf(), 0, t->n_rules);
        cd.oq_cap = other_cap(e, std::min<uint64_t>(n, kClsChunk), cfg.grid);
        {
            const int rc = other_queue(e, sc, cfg.grid, cd.oq_cap, s, &cd.oq);
            if (rc != CLS_OK) return rc;
        }
        if (q.lds_resident) cd.part = sc->part.as<uint32_t>();
        Fe16 fe = fe16(q.img, q.d_src_search);
        for (uint64_t off = 0; off < n; off += kClsChunk) {
            const uint64_t m = std::min<uint64_t>(kClsChunk, n - off);
            Pkts16 pc{reinterpret_cast<const uint4*>(src + 16 * off), reinterpret_cast<const uint4*>(dst + 16 * off),
                      dp + off, pr + off, m, 0u};
            if (c.swap) std::swap(pc.src, pc.dst);          // destination-keyed image
            uint8_t* vo = d_verdict ? d_verdict + off : nullptr;
            pc.vec = aligned(pc.dport, 8) && aligned(pc.proto, 4) && (!vo || aligned(vo, 4)) ? 1u : 0u;
            cd.zero = co.zero && !zeroed ? co.out : nullptr;    // the first launch clears the call's counters
            cd.n_zero = t->n_rules + 1;
            cfg.ev_start = timing && off == 0 ? e->ev0 : nullptr;
            cfg.ev_stop = timing && off + m >= n ? e->ev1 : nullptr;
            HIPC(e, launch_classify16_cls(cd, fe, pc, vo, slot_val, q.lds_resident, lin, cfg));
            zeroed = true;
            cd.zero = nullptr;
            HIPC(e, launch_finish16(finish_args(e, t->c16, sc, cd, co, q.lds_resident, uint32_t(cfg.grid), off + m >= n),
                                    cd, cfg.other, fe, pc, vo, s));
            remapped = true;
        }
    }
    if (timing) {
        if (!n) HIPC(e, hipEventRecord(e->ev1, s));
        e->timed = true;
    }
    if (co.zero && !zeroed) HIPC(e, launch_fold(nullptr, 0, 0, slot_val, co.out, t->n_rules + 1, s));
    return finish_counts(e, *t, t->c16, sc, co, n, verdict_out, d_verdict, counters_out, flags, s, remapped);
}

// Each packet's ACLAction and terminating rule (the debug trace of
// evalACL's matched rule, aclengine_mock.go:651-654): the classify kernels'
// slot mode, then slot -> rule; tables without a classifier image run the
// linear kernel.  No counters are touched.
static int classify_rules_locked(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pk, uint64_t n,
                                 uint8_t* verdict_out, uint32_t* rule_out, uint32_t flags, void* stream) {
    auto it = e->tables.find(table_id);
    if (it == e->tables.end()) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    const std::shared_ptr<Table> t = it->second;
    const bool v16 = pk->af == CLS_AF_V16;
    if (!v16 && pk->af != CLS_AF_V4) return fail(e, CLS_E_INVAL, "af must be CLS_AF_V4 or CLS_AF_V16");
    if (n && (!pk->dport || !pk->proto || (v16 ? !pk->src16 || !pk->dst16 : !pk->src4 || !pk->dst4)))
        return fail(e, CLS_E_INVAL, "missing packet arrays");
    if (n && !rule_out) return fail(e, CLS_E_INVAL, "rule_out is NULL");
    if (n > 0xFFFFFFFFull) return fail(e, CLS_E_INVAL, "batch above 2^32 packets");
    const bool dev = flags & CLS_F_DEVICE;
    const size_t ab = v16 ? 16 : 4;
    const uint8_t* src = v16 ? pk->src16 : reinterpret_cast<const uint8_t*>(pk->src4);
    const uint8_t* dst = v16 ? pk->dst16 : reinterpret_cast<const uint8_t*>(pk->dst4);
    if (dev && n && (!aligned(rule_out, 4) || (v16 && (!aligned(src, 16) || !aligned(dst, 16))) ||
                     (!v16 && (!aligned(src, 4) || !aligned(dst, 4))) || !aligned(pk->dport, 2)))
        return fail(e, CLS_E_INVAL, "device arrays must be aligned to their element size");
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    const uint16_t* dp = pk->dport;
    const uint8_t* pr = pk->proto;
    uint8_t* d_verdict = verdict_out;
    uint32_t* d_rule = rule_out;
    if (!dev && n) {
        HIPC(e, e->s_src.ensure(n * ab));
        HIPC(e, e->s_dst.ensure(n * ab));
        HIPC(e, e->s_dport.ensure(n * 2));
        HIPC(e, e->s_proto.ensure(n));
        HIPC(e, e->s_rule.ensure(n * 4));
        HIPC(e, hipMemcpyAsync(e->s_src.p, src, n * ab, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dst.p, dst, n * ab, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dport.p, dp, n * 2, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_proto.p, pr, n, hipMemcpyHostToDevice, s));
        src = e->s_src.as<uint8_t>();
        dst = e->s_dst.as<uint8_t>();
        dp = e->s_dport.as<uint16_t>();
        pr = e->s_proto.as<uint8_t>();
        d_rule = e->s_rule.as<uint32_t>();
        d_verdict = nullptr;
        if (verdict_out) {
            HIPC(e, e->s_verdict.ensure(n));
            d_verdict = e->s_verdict.as<uint8_t>();
        }
    }
    LaunchCfg cfg;
    cfg.stream = s;
    for (uint64_t off = 0; off < n; off += kClsChunk) {        // 32-bit packet offsets in the kernels
        const uint64_t m = std::min<uint64_t>(kClsChunk, n - off);
        uint8_t* vo = d_verdict ? d_verdict + off : nullptr;
        uint32_t* ro = d_rule + off;
        if (v16) {
            const auto& q = t->p16;
            const Cls4Image& ci = q.img.core;
            const Cls4Dev cd = cls4_dev(ci, q.d_img, q.d_lin, uint32_t(q.lin.size()), t->n_rules);
            cfg.other = cls4_dev(q.oimg, q.d_oimg, DevBuf(), 0, t->n_rules);
            cfg.grid = cls_grid(e, true, q.lds_resident, ci.lds_bytes, m);
            Pkts16 pc{reinterpret_cast<const uint4*>(src + 16 * off), reinterpret_cast<const uint4*>(dst + 16 * off),
                      dp + off, pr + off, m, 0u};
            if (ci.swap) std::swap(pc.src, pc.dst);          // destination-keyed image
            HIPC(e, launch_classify16_slots(cd, fe16(q.img, q.d_src_search), pc, ro, q.lds_resident, cfg));
            HIPC(e, launch_slot_rules(ro, q.d_slot_rule.as<uint32_t>(), uint32_t(m), vo, ro, s));
        } else {
            const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src) + off;
            const uint32_t* d4 = reinterpret_cast<const uint32_t*>(dst) + off;
            const Pkts4 pc{s4, d4, dp + off, pr + off, m};
            if (t->has_cls) {
                cfg.other = cls4_dev(t->oimg, t->d_oimg, DevBuf(), 0, t->n_rules);
                cfg.grid = cls_grid(e, true, t->lds_resident, t->img.lds_bytes, m);
                HIPC(e, launch_classify4_slots(table_dev(*t), framed(t->img, pc), ro, t->lds_resident, cfg));
                HIPC(e, launch_slot_rules(ro, t->d_slot_rule.as<uint32_t>(), uint32_t(m), vo, ro, s));
            } else {
                cfg.grid = cls_grid(e, false, false, 0, m);
                HIPC(e, launch_classify4_linear(t->d_lin4.as<LinRule4>(), uint32_t(t->lin4.size()), t->n_rules, pc,
                                                vo, nullptr, cfg, ro));
            }
        }
    }
    if (!dev && n) {
        if (verdict_out) HIPC(e, hipMemcpyAsync(verdict_out, d_verdict, n, hipMemcpyDeviceToHost, s));
        HIPC(e, hipMemcpyAsync(rule_out, d_rule, n * 4, hipMemcpyDeviceToHost, s));
        HIPC(e, hipStreamSynchronize(s));
    }
    return CLS_OK;
}

int cls_classify_rules(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pk, uint64_t n, uint8_t* verdict_out,
                       uint32_t* rule_out, uint32_t flags, void* stream) {
    if (!e || !pk) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    return classify_rules_locked(e, table_id, pk, n, verdict_out, rule_out, flags, stream);
}

int cls_classify(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pk, uint64_t n,
                 uint8_t* verdict_out, uint64_t* counters_out, uint32_t flags, void* stream) {
    if (!e || !pk) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    return classify_locked(e, table_id, pk, n, verdict_out, counters_out, flags, stream);
}

}  // extern "C"

int classify_locked(cls_engine* e, uint32_t table_id, const cls_pkt_soa* pk, uint64_t n,
                    uint8_t* verdict_out, uint64_t* counters_out, uint32_t flags, void* stream) {
    auto it = e->tables.find(table_id);
    if (it == e->tables.end()) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    std::shared_ptr<Table> t = it->second;
    if (pk->af == CLS_AF_V16) return classify16_locked(e, t, pk, n, verdict_out, counters_out, flags, stream);
    if (pk->af != CLS_AF_V4) return fail(e, CLS_E_INVAL, "af must be CLS_AF_V4 or CLS_AF_V16");
    if (n && (!pk->src4 || !pk->dst4 || !pk->dport || !pk->proto))
        return fail(e, CLS_E_INVAL, "missing packet arrays");
    if (!verdict_out && !(flags & CLS_F_NO_VERDICT) && n)
        return fail(e, CLS_E_INVAL, "verdict_out is NULL (set CLS_F_NO_VERDICT)");
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    const bool dev = flags & CLS_F_DEVICE;

    Pkts4 p{pk->src4, pk->dst4, pk->dport, pk->proto, n};
    uint8_t* d_verdict = verdict_out;
    if (!dev && n) {
        HIPC(e, e->s_src.ensure(n * 4));
        HIPC(e, e->s_dst.ensure(n * 4));
        HIPC(e, e->s_dport.ensure(n * 2));
        HIPC(e, e->s_proto.ensure(n));
        HIPC(e, hipMemcpyAsync(e->s_src.p, pk->src4, n * 4, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dst.p, pk->dst4, n * 4, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dport.p, pk->dport, n * 2, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_proto.p, pk->proto, n, hipMemcpyHostToDevice, s));
        p = Pkts4{e->s_src.as<uint32_t>(), e->s_dst.as<uint32_t>(), e->s_dport.as<uint16_t>(),
                  e->s_proto.as<uint8_t>(), n};
        d_verdict = nullptr;
        if (verdict_out) {
            HIPC(e, e->s_verdict.ensure(n));
            d_verdict = e->s_verdict.as<uint8_t>();
        }
    }
    Scratch* sc = nullptr;
    {
        const int rc = scratch_of(e, t->c4, t->n_rules, s, &sc);
        if (rc != CLS_OK) return rc;
    }
    const CountOut co = count_out(sc, counters_out, flags);
    unsigned long long* slot_val = sc->slot_val.as<unsigned long long>();

    const bool vec = aligned(p.src, 16) && aligned(p.dst, 16) && aligned(p.dport, 8) &&
                     aligned(p.proto, 4) && (!d_verdict || aligned(d_verdict, 4));
    LaunchCfg cfg;
    cfg.stream = s;
    const bool use_cls = t->has_cls && !(flags & CLS_F_FORCE_LINEAR);
    cfg.grid = cls_grid(e, use_cls, t->lds_resident, t->img.lds_bytes, n);

    const bool timing = flags & CLS_F_TIMING;
    if (timing) {
        const int rc = timing_pair(e);
        if (rc != CLS_OK) return rc;
        if (!(n && use_cls)) HIPC(e, hipEventRecord(e->ev0, s));
    }
    bool zeroed = false, remapped = false;
    if (n) {
        if (use_cls) {
            Cls4Dev cd = table_dev(*t);
            cfg.other = cls4_dev(t->oimg, t->d_oimg, DevBuf(), 0, t->n_rules);
            cd.oq_cap = other_cap(e, std::min<uint64_t>(n, kClsChunk), cfg.grid);
            {
                const int rc = other_queue(e, sc, cfg.grid, cd.oq_cap, s, &cd.oq);
                if (rc != CLS_OK) return rc;
            }
            if (t->lds_resident) cd.part = sc->part.as<uint32_t>();
            // the kernel indexes packets with 32-bit offsets: chunks of 2^30
            for (uint64_t off = 0; off < n; off += kClsChunk) {
                const uint64_t m = std::min<uint64_t>(kClsChunk, n - off);
                const Pkts4 pc = framed(t->img, Pkts4{p.src + off, p.dst + off, p.dport + off, p.proto + off, m});
                uint8_t* vo = d_verdict ? d_verdict + off : nullptr;
                cd.zero = co.zero && !zeroed ? co.out : nullptr;   // the first launch clears the call's counters
                cd.n_zero = t->n_rules + 1;
                cfg.ev_start = timing && off == 0 ? e->ev0 : nullptr;
                cfg.ev_stop = timing && off + m >= n ? e->ev1 : nullptr;
                HIPC(e, launch_classify4_cls(cd, pc, vo, slot_val, t->lds_resident, vec, cfg));
                zeroed = true;
                cd.zero = nullptr;
                FinishArgs fa = finish_args(e, t->c4, sc, cd, co, t->lds_resident, uint32_t(cfg.grid), off + m >= n);
                fa.qmask = 1u;                      // the IPv4 launch's queue entries (run_n kMaskQ)
                HIPC(e, launch_finish4(fa, cfg.other, pc, vo, s));
                remapped = true;
            }
        } else {
            const uint32_t base = t->c4.n_image;
            HIPC(e, launch_classify4_linear(t->d_lin4.as<LinRule4>(), uint32_t(t->lin4.size()), t->n_rules, p,
                                            d_verdict, slot_val + base, cfg));
        }
    }
    if (timing) {
        // ev0 / ev1: the classify kernel's own start and end (stamped by its
        // launch, before the fold of the workgroup partials)
        if (!(n && use_cls)) HIPC(e, hipEventRecord(e->ev1, s));
        e->timed = true;
    }
    if (co.zero && !zeroed) HIPC(e, launch_fold(nullptr, 0, 0, slot_val, co.out, t->n_rules + 1, s));
    return finish_counts(e, *t, t->c4, sc, co, n, verdict_out, d_verdict, counters_out, flags, s, remapped);
}

extern "C" {

// Each stream shape's time (cls_stream_floor_shapes): shape = variant << 1 |
// (two workgroups per CU), 8 shapes for the IPv4 layout, 2 for the 16-byte one.
static int stream_shapes(cls_engine* e, const cls_pkt_soa* pk, uint64_t n, uint8_t* verdict, uint32_t reps,
                         std::vector<float>& out, void* stream) {
    if (!e || !pk || !verdict || n == 0 || n > kClsChunk) return CLS_E_INVAL;
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    Pkts4 p4{pk->src4, pk->dst4, pk->dport, pk->proto, n};
    Pkts16 p16{reinterpret_cast<const uint4*>(pk->src16), reinterpret_cast<const uint4*>(pk->dst16), pk->dport,
               pk->proto, n, 1u};
    const bool v4 = pk->af == CLS_AF_V4;
    if (v4 ? !(aligned(pk->src4, 16) && aligned(pk->dst4, 16) && aligned(pk->dport, 8) && aligned(pk->proto, 4) &&
               aligned(verdict, 4))
           : !(pk->af == CLS_AF_V16 && aligned(pk->src16, 16) && aligned(pk->dst16, 16)))
        return fail(e, CLS_E_INVAL, "stream floor: device arrays of the classify kernel's alignment");
    // the floor is the fastest of the stream shapes: one or two 1024-thread
    // workgroups per CU (the classify kernel runs one when its LDS image
    // takes more than half the CU's LDS), loads one step ahead or not, the
    // protocol stream non-temporal or cached
    hipEvent_t a, b;
    HIPC(e, hipEventCreate(&a));
    HIPC(e, hipEventCreate(&b));
    int rc = CLS_OK;
    const uint32_t k = std::max<uint32_t>(1, reps);
    const bool dbg = e->opts.debug_floor;
    out.clear();
    for (int shape = 0; shape < (v4 ? 8 : 2) && rc == CLS_OK; ++shape) {
        const int grid = e->n_cu * (1 + (shape & 1)), variant = shape >> 1;
        for (uint32_t i = 0; i <= k && rc == CLS_OK; ++i) {   // launch 0: warm-up
            if (i == 1 && hipEventRecord(a, s) != hipSuccess) rc = CLS_E_HIP;
            if (rc == CLS_OK &&
                launch_stream(v4 ? &p4 : nullptr, v4 ? nullptr : &p16, verdict, grid, variant, s) != hipSuccess)
                rc = fail(e, CLS_E_HIP, "stream floor launch failed");
        }
        float t = 0.0f;
        if (rc == CLS_OK && hipEventRecord(b, s) == hipSuccess && hipEventSynchronize(b) == hipSuccess &&
            hipEventElapsedTime(&t, a, b) == hipSuccess) {
            t /= float(k);
            if (dbg) std::fprintf(stderr, "stream floor: grid %d variant %d: %.4f ms\n", grid, variant, t);
            out.push_back(t);
        } else if (rc == CLS_OK) {
            rc = fail(e, CLS_E_HIP, "stream floor timing failed");
        }
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return rc;
}

int cls_stream_floor(cls_engine* e, const cls_pkt_soa* pk, uint64_t n, uint8_t* verdict, uint32_t reps,
                     float* ms, void* stream) {
    if (!e || !ms) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    std::vector<float> t;
    const int rc = stream_shapes(e, pk, n, verdict, reps, t, stream);
    if (rc != CLS_OK) return rc;
    *ms = *std::min_element(t.begin(), t.end());
    return CLS_OK;
}

int cls_stream_floor_shapes(cls_engine* e, const cls_pkt_soa* pk, uint64_t n, uint8_t* verdict, uint32_t reps,
                            float* ms, uint32_t cap, uint32_t* count, void* stream) {
    if (!e || !count || (cap && !ms)) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    std::vector<float> t;
    const int rc = stream_shapes(e, pk, n, verdict, reps, t, stream);
    if (rc != CLS_OK) return rc;
    *count = uint32_t(t.size());
    std::copy(t.begin(), t.begin() + std::min<size_t>(cap, t.size()), ms);
    return CLS_OK;
}

int cls_last_kernel_ms(cls_engine* e, float* ms) {
    if (!e || !ms) return CLS_E_INVAL;
    if (!e->timed) return fail(e, CLS_E_INVAL, "no timed classify recorded");
    HIPC(e, hipEventSynchronize(e->ev1));
    HIPC(e, hipEventElapsedTime(ms, e->ev0, e->ev1));
    return CLS_OK;
}

int cls_kernel_times(cls_engine* e, float* ms, uint32_t cap, uint32_t* count) {
    if (!e || !count) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    *count = uint32_t(e->ev_used);
    if (e->ev_used == 0) return CLS_OK;
    HIPC(e, hipEventSynchronize(e->ev_pool[e->ev_used - 1].second));
    for (size_t i = 0; i < e->ev_used && i < cap && ms; ++i)
        HIPC(e, hipEventElapsedTime(&ms[i], e->ev_pool[i].first, e->ev_pool[i].second));
    return CLS_OK;
}

int cls_kernel_starts(cls_engine* e, float* ms, uint32_t cap, uint32_t* count) {
    if (!e || !count) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    *count = uint32_t(e->ev_used);
    if (e->ev_used == 0) return CLS_OK;
    HIPC(e, hipEventSynchronize(e->ev_pool[e->ev_used - 1].second));
    for (size_t i = 0; i < e->ev_used && i < cap && ms; ++i)
        HIPC(e, hipEventElapsedTime(&ms[i], e->ev_pool[0].first, e->ev_pool[i].first));
    return CLS_OK;
}

int cls_kernel_times_reset(cls_engine* e) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (e->ev_used) HIPC(e, hipEventSynchronize(e->ev_pool[e->ev_used - 1].second));
    e->ev_used = 0;
    return CLS_OK;
}

// ---------------------------------------------------------------------------
// ACLConfig
static uint32_t if_id_locked(cls_engine* e, const std::string& name) {
    auto it = e->if_ids.find(name);
    if (it != e->if_ids.end()) return it->second;
    const uint32_t id = uint32_t(e->if_names.size());
    e->if_ids[name] = id;
    e->if_names.push_back(name);
    e->if_acl.push_back({-1, -1});
    e->conn_gen++;                  // connection plans see the change
    return id;
}

static int acl_del_locked(cls_engine* e, const std::string& name) {
    auto it = e->acls.find(name);
    if (it == e->acls.end()) return fail(e, CLS_E_NOTFOUND, "cannot find ACL: %s", name.c_str());
    const int32_t tid = int32_t(it->second.table_id);
    (void)hipSetDevice(e->device);
    for (auto& b : e->if_acl) {
        if (b.first == tid) b.first = -1;
        if (b.second == tid) b.second = -1;
    }
    e->tables.erase(it->second.table_id);
    e->conn_gen++;                  // connection plans see the change
    drop_conn_plan(e);
    e->acls.erase(it);
    e->changes++;
    return CLS_OK;
}

int cls_acl_put(cls_engine* e, const char* acl_name, const cls_rule* rules, uint32_t n_rules,
                const char* const* ingress_ifs, uint32_t n_ingress, const char* const* egress_ifs,
                uint32_t n_egress) {
    if (!e || !acl_name) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    const int rc = acl_put_locked(e, acl_name, rules, n_rules, ingress_ifs, n_ingress, egress_ifs, n_egress);
    return rc == CLS_OK ? sync_peers(e) : rc;
}

}  // extern "C"

static int acl_put_locked(cls_engine* e, const char* acl_name, const cls_rule* rules, uint32_t n_rules,
                          const char* const* ingress_ifs, uint32_t n_ingress, const char* const* egress_ifs,
                          uint32_t n_egress) {
    if (n_ingress + n_egress == 0) return fail(e, CLS_E_INVAL, "ACL with empty interfaces");
    if (n_rules && !rules) return fail(e, CLS_E_INVAL, "rules is NULL");
    const std::string name(acl_name);
    uint32_t tid;
    auto old = e->acls.find(name);
    auto same = old == e->acls.end() ? e->tables.end() : e->tables.find(old->second.table_id);
    if (same != e->tables.end() && same->second->sig == rule_sig(rules, n_rules)) {
        // Equal rules (the renderer re-puts a table whose pods changed,
        // acl_renderer.go:186-190): keep the compiled table, move the bindings.
        // A put installs a new ACL (PutACL replaces the message,
        // aclengine_mock.go:707-713), so its connection counters start from
        // zero either way.  Every connection batch has finished its work on
        // them (cls_connect_batch synchronises its stream before it returns,
        // under this mutex), so the clearing is queued on the engine stream
        // without waiting; a later counting batch on another stream waits for
        // the event recorded behind it.
        tid = old->second.table_id;
        Table& kt = *same->second;
        if (kt.d_conn_ctr.p) {
            const int qrc = conn_quiesce(e);           // a counting batch on another stream may still add
            if (qrc != CLS_OK) return qrc;
            (void)hipSetDevice(e->device);
            HIPC(e, hipMemsetAsync(kt.d_conn_ctr.p, 0, size_t(kt.n_rules + 1) * 8, e->stream));
            if (!kt.conn_ctr_ev) HIPC(e, hipEventCreateWithFlags(&kt.conn_ctr_ev, hipEventDisableTiming));
            HIPC(e, hipEventRecord(kt.conn_ctr_ev, e->stream));
        }
        kt.conn_epoch++;                // a multi-device engine's peers clear their copies
        for (auto& b : e->if_acl) {
            if (b.first == int32_t(tid)) b.first = -1;
            if (b.second == int32_t(tid)) b.second = -1;
        }
        e->acls.erase(old);
        e->rebinds++;
    } else {
        int rc = table_put_locked(e, acl_name, rules, n_rules, &tid);
        if (rc != CLS_OK) return rc;
        if (old != e->acls.end()) {         // PutACL: delete the original first, not a change
            acl_del_locked(e, name);
            e->changes--;
        }
        e->compiles++;
    }
    AclEntry a;
    a.table_id = tid;
    for (uint32_t i = 0; i < n_ingress; ++i) {
        const uint32_t id = if_id_locked(e, ingress_ifs[i]);
        a.ingress.push_back(id);
        e->if_acl[id].first = int32_t(tid);
        e->conn_gen++;                  // connection plans see the change
    }
    for (uint32_t i = 0; i < n_egress; ++i) {
        const uint32_t id = if_id_locked(e, egress_ifs[i]);
        a.egress.push_back(id);
        e->if_acl[id].second = int32_t(tid);
        e->conn_gen++;                  // connection plans see the change
    }
    e->acls[name] = a;
    e->changes++;
    return CLS_OK;
}

extern "C" {

int cls_acl_stats(cls_engine* e, uint32_t* n_compiles, uint32_t* n_rebinds) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (n_compiles) *n_compiles = e->compiles;
    if (n_rebinds) *n_rebinds = e->rebinds;
    return CLS_OK;
}

int cls_acl_del(cls_engine* e, const char* acl_name) {
    if (!e || !acl_name) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    const int rc = acl_del_locked(e, acl_name);
    return rc == CLS_OK ? sync_peers(e) : rc;
}

int cls_acl_table(cls_engine* e, const char* acl_name, uint32_t* table_id) {
    if (!e || !acl_name || !table_id) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    auto it = e->acls.find(acl_name);
    if (it == e->acls.end()) return fail(e, CLS_E_NOTFOUND, "cannot find ACL: %s", acl_name);
    *table_id = it->second.table_id;
    return CLS_OK;
}

int cls_acl_counts(cls_engine* e, uint32_t* n_acls, uint32_t* n_changes) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (n_acls) *n_acls = uint32_t(e->acls.size());
    if (n_changes) *n_changes = e->changes;
    return CLS_OK;
}

int cls_if_id(cls_engine* e, const char* if_name, uint32_t* id) {
    if (!e || !if_name || !id) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    if (e->primary) return refuse_peer(e);
    *id = if_id_locked(e, if_name);
    return sync_peers(e);
}

int cls_if_acls(cls_engine* e, uint32_t if_id, int32_t* in_table, int32_t* out_table) {
    if (!e) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (if_id >= e->if_acl.size()) return fail(e, CLS_E_NOTFOUND, "no interface %u", if_id);
    if (in_table) *in_table = e->if_acl[if_id].first;
    if (out_table) *out_table = e->if_acl[if_id].second;
    return CLS_OK;
}

// The bitmap form of a linear IPv4 ACL (kernels.hpp kConnBmHeader): for the
// source, the destination and each protocol's destination port, the
// elementary intervals of the rules' prefixes (port ranges) and, per
// interval, the bit row of the rules whose term holds there -- each
// predicate evaluated exactly as the scan does (conn_match, the meta TERM bit,
// port_in) at the interval's first value, which is exact because prefixes
// and ranges only change membership at the interval starts.  Appends the
// words (16-B multiple) to `out`; false (nothing appended) when the tables
// would exceed `cap_words`.
static bool conn_bitmap4(const std::vector<ConnRule4>& r, uint32_t n_rules, size_t cap_words,
                         std::vector<uint32_t>& out) {
    const uint32_t R = uint32_t(r.size()), W = std::max<uint32_t>(1, (R + 31) / 32);
    (void)n_rules;
    auto port_in = [](uint32_t port, uint32_t pw) { return ((port - (pw & 0xFFFFu)) & 0xFFFFu) <= (pw >> 16); };
    struct Tab {
        std::vector<uint32_t> keys, rows;
    };
    // the interval starts of the six tables first (sorting 2R values each):
    // the size check needs only their counts, so a table over the cap never
    // builds its keys x R predicate rows
    auto addr_keys = [&](bool dst) {
        std::vector<uint64_t> b{0};
        for (const ConnRule4& x : r) {
            const uint32_t a = dst ? x.dst_addr : x.src_addr, m = dst ? x.dst_mask : x.src_mask;
            if (!m) continue;
            b.push_back(a);
            b.push_back(uint64_t(a) + uint64_t(~m) + 1);        // one past the prefix
        }
        std::sort(b.begin(), b.end());
        b.erase(std::unique(b.begin(), b.end()), b.end());
        while (!b.empty() && b.back() > 0xFFFFFFFFull) b.pop_back();
        return std::vector<uint32_t>(b.begin(), b.end());
    };
    auto port_keys = [&](uint32_t p) {
        std::vector<uint32_t> b{0};
        if (p < 2)
            for (const ConnRule4& x : r) {
                if (!((x.meta >> (8 * p)) & 0x80u)) continue;
                const uint32_t lo = x.port[p] & 0xFFFFu, end = lo + (x.port[p] >> 16) + 1;   // one past hi
                b.push_back(lo);
                b.push_back(end & 0xFFFFu);                      // wraps to 0 past 65535
            }
        std::sort(b.begin(), b.end());
        b.erase(std::unique(b.begin(), b.end()), b.end());
        return b;
    };
    // size (the rows are R x intervals bits); interval counts fit the
    // descriptor's 16-bit fields
    size_t words = kConnBmHeader / 4 + 2 * size_t(R);
    if (words > cap_words) return false;
    std::vector<Tab> tabs(6);
    for (int k = 0; k < 6; ++k) {
        tabs[k].keys = k < 2 ? addr_keys(k == 1) : port_keys(uint32_t(k - 2));
        words += tabs[k].keys.size() * (1 + size_t(W));
        if (words > cap_words || tabs[k].keys.size() > 0xFFFFu) return false;
    }
    // then the rows: bit i of an interval's row set when rule i's term holds
    // at the interval's first value
    for (int k = 0; k < 6; ++k) {
        Tab& t = tabs[k];
        t.rows.assign(t.keys.size() * W, 0u);
        for (size_t j = 0; j < t.keys.size(); ++j) {
            const uint32_t x = t.keys[j];
            uint32_t* row = t.rows.data() + j * W;
            for (uint32_t i = 0; i < R; ++i) {
                bool hit;
                if (k < 2) {
                    const uint32_t a = k ? r[i].dst_addr : r[i].src_addr, m = k ? r[i].dst_mask : r[i].src_mask;
                    hit = ((x ^ a) & m) == 0;
                } else {
                    const uint32_t p = uint32_t(k - 2);
                    const uint32_t pw = p == 0 ? r[i].port[0] : p == 1 ? r[i].port[1] : 0xFFFF0000u;
                    hit = ((r[i].meta >> (8 * p)) & 0x80u) && port_in(x, pw);
                }
                if (hit) row[i / 32] |= 1u << (i % 32);
            }
        }
    }
    const size_t at = out.size();
    out.insert(out.end(), {W, uint32_t(tabs[0].keys.size()), uint32_t(tabs[1].keys.size()), R,
                           uint32_t(tabs[2].keys.size()), uint32_t(tabs[3].keys.size()),
                           uint32_t(tabs[4].keys.size()), uint32_t(tabs[5].keys.size())});
    for (const Tab& t : tabs) {
        out.insert(out.end(), t.keys.begin(), t.keys.end());
        out.insert(out.end(), t.rows.begin(), t.rows.end());
    }
    for (const ConnRule4& x : r) {
        out.push_back(x.meta);
        out.push_back(x.index);
    }
    out.resize(at + ((out.size() - at + 3) & ~size_t(3)), 0u);
    return true;
}

int cls_connect_batch(cls_engine* e, const cls_conn_soa* c, uint64_t n, uint8_t* out,
                      uint32_t flags, void* stream) {
    if (!e || !c || (n && !out)) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    // host arrays: returns with the verdicts; CLS_F_DEVICE: stream-ordered
    return connect_locked(e, c, n, out, flags, stream, false);
}

}  // extern "C"

// The OTHER queue of a pair launch: a fixed segment per workgroup (its
// overflow is classified in place), so the buffer does not grow with the
// batch: the entries of a pair-launch workgroup (option pair_qcap: per
// wave, tests, to reach the in-place path).
static uint32_t pair_qcap(const cls_engine* e, uint64_t n, int grid) {
    if (e->opts.pair_qcap_set) return e->opts.pair_qcap * (kPairBlock / 64);
    return uint32_t(std::min<uint64_t>(pair_queue_words(n, grid), 16384));
}

int connect_locked(cls_engine* e, const cls_conn_soa* c, uint64_t n, uint8_t* out, uint32_t flags, void* stream,
                   bool sync) {
    const cls_pkt_soa& pk = c->pkt;
    const bool k16 = pk.af == CLS_AF_V16;
    if (!k16 && pk.af != CLS_AF_V4) return fail(e, CLS_E_INVAL, "af must be CLS_AF_V4 or CLS_AF_V16");
    const void *src = k16 ? static_cast<const void*>(pk.src16) : pk.src4,
               *dst = k16 ? static_cast<const void*>(pk.dst16) : pk.dst4;
    if (n && (!src || !dst || !pk.sport || !pk.dport || !pk.proto || !c->src_if || !c->dst_if))
        return fail(e, CLS_E_INVAL, "missing connection arrays");
    const bool dev = flags & CLS_F_DEVICE, count = flags & CLS_F_COUNT;
    const size_t ab = k16 ? 16 : 4;                       // address bytes
    // the kernels index connections with 32-bit offsets
    if (n > kClsChunk) return fail(e, CLS_E_INVAL, "connection batch above 2^30 connections");
    if (dev && k16 && n && (!aligned(src, 16) || !aligned(dst, 16)))
        return fail(e, CLS_E_INVAL, "device src16/dst16 must be 16-byte aligned");
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    // Device batches are stream-ordered (the call returns once its launches
    // are queued, like cls_classify with CLS_F_DEVICE) and share the engine's
    // connection scratch: the last batch's stream, if another, is waited for
    // on the GPU (an event recorded on it now); a scratch buffer grows, and
    // the plan or its uploads change, only once that batch has finished.
    if (e->conn_last && e->conn_last != s) {
        if (!e->conn_sync_ev) HIPC(e, hipEventCreateWithFlags(&e->conn_sync_ev, hipEventDisableTiming));
        HIPC(e, hipEventRecord(e->conn_sync_ev, e->conn_last));
        HIPC(e, hipStreamWaitEvent(s, e->conn_sync_ev, 0));
    }
    auto grow = [&](DevBuf& d, size_t bytes) -> hipError_t {
        if (bytes > d.bytes && conn_quiesce(e) != CLS_OK) return hipErrorUnknown;
        return d.ensure(bytes);
    };
    const uint32_t n_ifs = uint32_t(e->if_acl.size());
    if (!dev)
        for (uint64_t i = 0; i < n; ++i)
            if (c->src_if[i] >= n_ifs || c->dst_if[i] >= n_ifs)
                return fail(e, CLS_E_INVAL, "connection %llu: unknown interface id", (unsigned long long)i);
    const uint32_t *sif = c->src_if, *dif = c->dst_if;
    const uint16_t *sp = pk.sport, *dp = pk.dport;
    const uint8_t* pr = pk.proto;
    uint8_t* o = out;
    if (!dev && n) {
        HIPC(e, grow(e->s_src, n * ab)); HIPC(e, grow(e->s_dst, n * ab));
        HIPC(e, grow(e->s_if_a, n * 4)); HIPC(e, grow(e->s_if_b, n * 4));
        HIPC(e, grow(e->s_sport, n * 2)); HIPC(e, grow(e->s_dport, n * 2));
        HIPC(e, grow(e->s_proto, n)); HIPC(e, grow(e->s_verdict, n));
        HIPC(e, hipMemcpyAsync(e->s_src.p, src, n * ab, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dst.p, dst, n * ab, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_if_a.p, sif, n * 4, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_if_b.p, dif, n * 4, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_sport.p, sp, n * 2, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_dport.p, dp, n * 2, hipMemcpyHostToDevice, s));
        HIPC(e, hipMemcpyAsync(e->s_proto.p, pr, n, hipMemcpyHostToDevice, s));
        src = e->s_src.p; dst = e->s_dst.p;
        sif = e->s_if_a.as<uint32_t>(); dif = e->s_if_b.as<uint32_t>();
        sp = e->s_sport.as<uint16_t>(); dp = e->s_dport.as<uint16_t>();
        pr = e->s_proto.as<uint8_t>(); o = e->s_verdict.as<uint8_t>();
    }
    // The plan (ConnPlan): a device batch reuses the last one while the
    // bindings and the flags are the same; a host batch picks its large ACLs
    // from a sample of its connections, so it plans every time.
    const bool use_big = n && !(flags & CLS_F_FORCE_LINEAR) && (n >= kConnClsMinBatch || (flags & CLS_F_CONN_CLS));
    const bool use_bm = !k16 && n && !(flags & CLS_F_FORCE_LINEAR) && e->opts.conn_bitmap;
    const uint64_t key = uint64_t(k16) | uint64_t(count) << 1 | uint64_t(use_big) << 2 |
                         uint64_t((flags & CLS_F_CONN_CLS) != 0) << 3 | uint64_t(use_bm) << 4;
    ConnPlan fresh;
    ConnPlan& P = dev ? e->conn_plan : fresh;
    const bool planned = dev && P.gen == e->conn_gen && P.key == key;
    if (!planned) {
        if (dev) {
            const int qrc = conn_quiesce(e);        // the kept plan's tables may be in use
            if (qrc != CLS_OK) return qrc;
        }
        P = ConnPlan();
        // Snapshot the bindings: one descriptor per bound table, (in, out) per
        // interface.  Linear ACLs' compact rules go to the call's rule pool.
        std::unordered_map<int32_t, int32_t> slot;
        auto desc_of = [&](int32_t tid) -> int32_t {
            if (tid < 0) return -1;
            auto f = slot.find(tid);
            if (f != slot.end()) return f->second;
            auto t = e->tables.find(uint32_t(tid));
            if (t == e->tables.end()) return -1;
            const Table& T = *t->second;
            ConnDesc d{};
            d.pre_blk = -1;
            d.bm_off = 0xFFFFFFFFu;
            d.n = uint32_t(k16 ? T.conn16.size() : T.conn4.size());
            d.n_rules = T.n_rules;
            d.ctr_off = P.n_ctr;
            P.n_ctr += T.n_rules + 1;
            P.desc.push_back(d);
            P.dtab.push_back(t->second);
            slot[tid] = int32_t(P.desc.size() - 1);
            return int32_t(P.desc.size() - 1);
        };
        P.ifs.resize(std::max<size_t>(1, e->if_acl.size()));
        for (size_t i = 0; i < e->if_acl.size(); ++i)
            P.ifs[i] = IfAcls{desc_of(e->if_acl[i].first), desc_of(e->if_acl[i].second), -1, -1};
        // Large ACLs: the classifier evaluates the SYN tuple (src, dst, dport)
        // and the SYN-ACK tuple (dst, src, sport) of every connection in slot
        // mode (res | slot << 2 per connection); the connection kernel then
        // reads those words instead of scanning the ACL, and maps the slot to
        // its rule only for the calls testConnection makes.  Whole-batch
        // evaluation keeps the classify launches dense (no compaction).
        // Which ACLs: with a host batch, those whose linear work would be
        // large -- connections touching the ACL x its rule count >=
        // kConnClsWork x batch (touches estimated per interface binding from
        // <= 64 Ki sampled connections, at hashed positions); with a device
        // batch, the ACLs of >= kConnClsDevRules rules.  CLS_F_CONN_CLS: every
        // imaged ACL.
        if (use_big) {
            std::vector<uint64_t> touch(P.dtab.size(), 0);
            if (!dev && !(flags & CLS_F_CONN_CLS)) {
                const uint64_t m = std::min<uint64_t>(n, 65536);
                std::vector<uint64_t> per_if(P.ifs.size(), 0);
                for (uint64_t k = 0; k < m; ++k) {
                    // sample k: a splitmix-scrambled position in stratum k (no stride aliasing)
                    uint64_t z = (k + 1) * 0x9E3779B97F4A7C15ull;
                    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                    z ^= z >> 31;
                    const uint64_t lo = k * n / m, hi = (k + 1) * n / m;
                    const uint64_t i = lo + z % (hi - lo);
                    per_if[c->src_if[i]] += 1;
                    if (c->dst_if[i] != c->src_if[i]) per_if[c->dst_if[i]] += 1;
                }
                for (size_t f = 0; f < n_ifs; ++f) {
                    const uint64_t t = per_if[f] * n / m;
                    if (P.ifs[f].in >= 0) touch[P.ifs[f].in] += t;
                    if (P.ifs[f].out >= 0 && P.ifs[f].out != P.ifs[f].in) touch[P.ifs[f].out] += t;
                }
            }
            for (uint32_t j = 0; j < P.dtab.size(); ++j) {
                const Table& t = *P.dtab[j];
                const bool imaged = k16 ? t.p16.ok : t.has_cls;
                if (!imaged || t.n_rules < kConnClsMinRules) continue;
                const bool want = (flags & CLS_F_CONN_CLS) ||
                                  (dev ? t.n_rules >= kConnClsDevRules
                                       : double(touch[j]) * t.n_rules >= double(kConnClsWork) * double(n));
                if (want) P.big.push_back(j);
            }
        }
        // the large ACLs' result-word blocks: block b = the ACL big[b], also
        // per interface (the connection kernel loads a connection's words
        // before its descriptors)
        for (size_t b = 0; b < P.big.size(); ++b) {
            ConnDesc& d = P.desc[P.big[b]];
            const Table& t = *P.dtab[P.big[b]];
            d.pre_blk = int32_t(b);
            d.n = 0;
            d.slot_rule = k16 ? t.p16.d_slot_rule.as<uint32_t>() : t.d_slot_rule.as<uint32_t>();
            for (IfAcls& f : P.ifs) {
                if (f.in == int32_t(P.big[b])) f.in_pre = int32_t(b);
                if (f.out == int32_t(P.big[b])) f.out_pre = int32_t(b);
            }
        }
        // the rule pool of the linear ACLs
        const size_t rb = k16 ? sizeof(ConnRule16) : sizeof(ConnRule4);
        for (size_t j = 0; j < P.desc.size(); ++j) {
            if (P.desc[j].pre_blk >= 0) continue;
            P.desc[j].rule_off = uint32_t(P.pool.size() / rb);
            const uint8_t* r = k16 ? reinterpret_cast<const uint8_t*>(P.dtab[j]->conn16.data())
                                   : reinterpret_cast<const uint8_t*>(P.dtab[j]->conn4.data());
            P.pool.insert(P.pool.end(), r, r + size_t(P.desc[j].n) * rb);
        }
        // IPv4: the bitmap form of the longer linear ACLs, longest first, while
        // the pool (and the LDS counters when counting) still fit LDS -- a wave
        // then pays a fixed number of reads per evaluation instead of its
        // longest lane's scan (option conn_bitmap=0: scans only).
        if (use_bm) {
            const size_t lds_max0 = size_t(max_lds_bytes());
            // the LDS counters take their share only when they can be LDS counters
            // at all (otherwise they are global, cmode 2); no subtraction wraps
            const size_t ctr_b = count ? size_t(conn_lds_ctr_bytes(P.n_ctr)) : 0, reserve = std::min<size_t>(lds_max0 / 8, 8192);
            const size_t ctr_lds = ctr_b + reserve <= lds_max0 ? ctr_b : 0;
            const size_t cap = lds_max0 - reserve - ctr_lds;
            std::vector<size_t> order;
            for (size_t j = 0; j < P.desc.size(); ++j)
                if (P.desc[j].pre_blk < 0 && P.desc[j].n >= kConnBmMinRules) order.push_back(j);
            std::stable_sort(order.begin(), order.end(),
                             [&](size_t a, size_t b) { return P.desc[a].n > P.desc[b].n; });
            std::vector<uint32_t> words;
            for (size_t j : order) {
                Table& t = *P.dtab[j];
                if (!t.conn_bm_built) {                         // once per table: rules are immutable
                    if (!conn_bitmap4(t.conn4, t.n_rules, kConnBmMaxWords, t.conn_bm)) t.conn_bm.clear();
                    t.conn_bm_built = true;
                }
                const size_t used = P.pool.size() + words.size() * 4;
                if (t.conn_bm.empty() || used + t.conn_bm.size() * 4 > cap) continue;
                P.desc[j].bm_off = uint32_t(used);              // the pool is a multiple of 32 B, blobs of 16 B
                const std::vector<uint32_t>& h = t.conn_bm;     // header {W, ns, nd, nr, n0, n1, n2, n3}
                P.desc[j].bm_sd = h[1] | (h[2] << 16);
                P.desc[j].bm_tu = h[4] | (h[5] << 16);
                P.desc[j].bm_w = h[0];
                for (uint32_t len : {h[1], h[2], h[4], h[5]})   // ceil(log2(len)) steps take a table to one key
                    while ((1u << P.bm_steps) < len) ++P.bm_steps;
                words.insert(words.end(), t.conn_bm.begin(), t.conn_bm.end());
            }
            const uint8_t* wb = reinterpret_cast<const uint8_t*>(words.data());
            P.pool.insert(P.pool.end(), wb, wb + words.size() * 4);
        }
        P.id = ++e->plan_ids;
        if (dev) {
            P.key = key;
            P.gen = e->conn_gen;
        }
    }
    std::vector<ConnDesc>& desc = P.desc;
    std::vector<std::shared_ptr<Table>>& dtab = P.dtab;
    std::vector<IfAcls>& ifs = P.ifs;
    const std::vector<uint8_t>& pool = P.pool;
    const std::vector<uint32_t>& big = P.big;
    const uint32_t n_ctr = P.n_ctr;
    // The result words: block b (the ACL big[b]) at pre + 2 b stride, the SYN
    // tuple's words first, the SYN-ACK tuple's at + stride (a multiple of 4,
    // so both halves stay 16-B aligned for the pair launch's stores).  In
    // byte mode (pre_res8 below) block b is stride bytes at pre + b stride.
    const uint64_t stride = (n + 3) & ~uint64_t(3);
    // Both tuples of a large ACL in one launch (classify4_pair) when the image
    // is LDS-resident and the arrays allow its 16-B loads.  When every large
    // ACL takes that launch and the batch counts, the launch writes each
    // word's counter index (descriptor counter base + the slot's rule)
    // instead of its slot: the connection kernel then counts a large-ACL call
    // without a descriptor read and a dependent slot -> rule gather.
    auto pair_ok = [&](const Table& t) {
        const uint32_t *s4 = static_cast<const uint32_t*>(src), *d4 = static_cast<const uint32_t*>(dst);
        return !k16 && t.lds_resident && aligned(s4, 16) && aligned(d4, 16) && aligned(dp, 8) && aligned(sp, 8) &&
               aligned(pr, 4) && e->opts.conn_pair;
    };
    bool all_pair = !big.empty();
    for (uint32_t b : big) all_pair = all_pair && pair_ok(*dtab[b]);
    const bool pre_rules = count && all_pair && e->opts.conn_pre_rules;
    // ... and a batch that does not count needs only the ACLActions: one byte
    // per connection for both tuples (the words would be 8 B)
    const bool pre_res8 = !count && all_pair && e->opts.conn_pre_narrow;
    // ... and a counting one u16 words when every counter index fits 14 bits
    const uint32_t pre_bytes = pre_res8 ? 1u : pre_rules && P.n_ctr <= (1u << 14) &&
                                                       e->opts.conn_pre_narrow ? 2u : 4u;
    if (!big.empty()) {
        if (n > kClsChunk) return fail(e, CLS_E_INVAL, "connection batch above 2^30 with classifier ACLs");
        HIPC(e, grow(e->s_pre, big.size() * (pre_res8 ? stride : 2 * stride * pre_bytes)));
        for (size_t b = 0; b < big.size(); ++b) {
            Table& t = *dtab[big[b]];
            uint32_t* pre = reinterpret_cast<uint32_t*>(e->s_pre.as<uint8_t>() +
                                                        b * (pre_res8 ? stride : 2 * stride * pre_bytes));
            LaunchCfg cfg;
            cfg.stream = s;
            if (!k16) {
                Cls4Dev cd = table_dev(t);
                const uint32_t *s4 = static_cast<const uint32_t*>(src), *d4 = static_cast<const uint32_t*>(dst);
                const Pkts4 syn = framed(t.img, Pkts4{s4, d4, dp, pr, n}), ack = framed(t.img, Pkts4{d4, s4, sp, pr, n});
                // Both tuples in one launch when the image is LDS-resident and
                // the arrays allow 16-B loads; the OTHER image beside the main
                // one when both fit (no slot counters in this mode)
                if (pair_ok(t) && e->opts.pair_o4 && (!count || pre_rules) && pair_image(e, t)) {
                    // the pair image: protocols > 2 in the main loop with the
                    // others -- no OTHER queue, drain or second image (its
                    // slots are its own: counting takes the counter-index
                    // words; option pair_o4=0: the OTHER queue below)
                    const Cls4Dev pd = cls4_dev(t.pimg, t.d_pimg, DevBuf(), 0, t.n_rules);
                    // counting: the slot -> rule map in LDS after the image when
                    // it fits (else each word's rule is a global gather)
                    PairMap sm;
                    sm.srl = (t.pimg.img_bytes + 15u) & ~15u;
                    if (pre_rules && t.pslot16_n16 && e->opts.pair_map_lds &&
                        sm.srl + 16u * t.pslot16_n16 + 32u <= uint32_t(max_lds_bytes())) {
                        sm.map = t.d_pslot16.as<uint16_t>();
                        sm.n16 = t.pslot16_n16;
                    } else {
                        sm.srl = 0;
                    }
                    cfg.grid = cls_grid(e, true, true, sm.srl ? sm.srl + 16u * sm.n16 : t.pimg.img_bytes, n);
                    if (e->opts.debug_conn)
                        std::fprintf(stderr, "pair: pimg %u mode %u list mode %u map %u (img %u oimg %u)\n",
                                     t.pimg.img_bytes, t.pimg.mode, t.pimg.list_mode, 16u * sm.n16, t.img.img_bytes,
                                     t.oimg.img_bytes);
                    HIPC(e, launch_classify4_pair(pd, pd, 0, framed(t.pimg, Pkts4{s4, d4, dp, pr, n}), sp, pre, stride,
                                                  nullptr, 0, pre_rules ? t.d_pslot_rule.as<uint32_t>() : nullptr,
                                                  desc[big[b]].ctr_off, pre_bytes, 0, false, 0u, true, sm, cfg));
                } else if (pair_ok(t)) {
                    uint32_t o_at = (t.img.img_bytes + 15u) & ~15u;
                    // (+ 32: the queue fill word after the images)
                    if (o_at + t.oimg.img_bytes + 32u > uint32_t(max_lds_bytes())) o_at = 0;
                    if (e->opts.pair_other_global || e->opts.pair_other_late == 2) o_at = 0;   // tests
                    // else, when the OTHER image does not fit beside the main
                    // one, staged over it for the drain (option
                    // pair_other_late=0: read from global memory there)
                    const bool o_late = !o_at && !e->opts.pair_other_global && e->opts.pair_other_late > 0 &&
                                        t.oimg.img_bytes + 32u <= uint32_t(max_lds_bytes());
                    Cls4Dev od = cls4_dev(t.oimg, t.d_oimg, DevBuf(), 0, t.n_rules);
                    if (o_at) {
                        od.off_bounds += o_at; od.off_iclass += o_at; od.off_cells += o_at;
                        od.off_lists += o_at; od.off_tmpl += o_at;
                    }
                    cfg.grid = cls_grid(e, true, true, pair_queue_lds(t.img.img_bytes, o_at, t.oimg.img_bytes, o_late), n);
                    // the OTHER queue, one segment per wave: its first entries
                    // in the LDS left after the images (one workgroup per CU
                    // either way), the rest in global memory
                    // (options pair_qcap / pair_lq: entries per
                    // wave in all / in LDS, tests)
                    const uint32_t nwv = kPairBlock / 64;
                    const uint32_t qw = (pair_qcap(e, n, cfg.grid) + nwv - 1) / nwv;
                    const uint32_t q_lds = pair_queue_lds(t.img.img_bytes, o_at, t.oimg.img_bytes, o_late);
                    uint32_t lq_cap = std::min<uint32_t>(qw, (uint32_t(max_lds_bytes()) - q_lds) / 16u / nwv);
                    if (e->opts.pair_lq >= 0) lq_cap = std::min<uint32_t>(lq_cap, uint32_t(e->opts.pair_lq));
                    const uint32_t gq = qw - lq_cap;
                    HIPC(e, grow(e->s_pq, size_t(cfg.grid) * nwv * std::max<uint32_t>(1, gq) * 16));
                    if (e->opts.debug_conn)      // diagnostics: where the OTHER image and queue live
                        std::fprintf(stderr, "pair: img %u oimg %u o_at %u o_late %d lq %u gq %u cdiv %u\n",
                                     t.img.img_bytes, t.oimg.img_bytes, o_at, int(o_late), lq_cap, gq,
                                     e->opts.pair_class ? t.pair_cdiv : 0u);
                    HIPC(e, launch_classify4_pair(cd, od, o_at, syn, sp, pre, stride, e->s_pq.as<uint32_t>(), gq,
                                                  pre_rules ? t.d_slot_rule.as<uint32_t>() : nullptr,
                                                  desc[big[b]].ctr_off, pre_bytes, lq_cap, o_late,
                                                  e->opts.pair_class ? t.pair_cdiv : 0u, false, PairMap{}, cfg));
                } else {
                    cfg.other = cls4_dev(t.oimg, t.d_oimg, DevBuf(), 0, t.n_rules);
                    cfg.grid = cls_grid(e, true, t.lds_resident, t.img.lds_bytes, n);
                    HIPC(e, launch_classify4_slots(cd, syn, pre, t.lds_resident, cfg));
                    HIPC(e, launch_classify4_slots(cd, ack, pre + stride, t.lds_resident, cfg));
                }
            } else {
                auto& q = t.p16;
                const Cls4Image& ci = q.img.core;
                Cls4Dev cd = cls4_dev(ci, q.d_img, q.d_lin, uint32_t(q.lin.size()), t.n_rules);
                cfg.other = cls4_dev(q.oimg, q.d_oimg, DevBuf(), 0, t.n_rules);
                cfg.grid = cls_grid(e, true, q.lds_resident, ci.lds_bytes, n);
                const Fe16 fe = fe16(q.img, q.d_src_search);
                const uint4 *s16 = static_cast<const uint4*>(src), *d16 = static_cast<const uint4*>(dst);
                Pkts16 syn{s16, d16, dp, pr, n, 0u}, ack{d16, s16, sp, pr, n, 0u};
                if (ci.swap) {                               // destination-keyed image
                    std::swap(syn.src, syn.dst);
                    std::swap(ack.src, ack.dst);
                }
                HIPC(e, launch_classify16_slots(cd, fe, syn, pre, q.lds_resident, cfg));
                HIPC(e, launch_classify16_slots(cd, fe, ack, pre + stride, q.lds_resident, cfg));
            }
        }
    }
    ConnArgs a{};
    a.n_ifs = n_ifs;
    a.rules_bytes = uint32_t(pool.size());
    a.n_ctr = count ? n_ctr : 0;
    a.src_if = sif; a.dst_if = dif; a.src = src; a.dst = dst;
    a.sport = sp; a.dport = dp; a.proto = pr; a.n = n; a.out = o;
    // LDS: the rule pool first (every evaluation step reads it), then the u32
    // counters if they fit beside it; otherwise global-memory variants
    // (option conn_no_lds, tests: bit 0 rules from global memory, bit 1
    // global counters, bit 2 descriptor / interface tables from global memory)
    const int no_lds = e->opts.conn_no_lds;
    const size_t lds_max = size_t(max_lds_bytes());
    const bool lds_rules = n && !pool.empty() && pool.size() + 16 + kConnStateEntries <= lds_max && !(no_lds & 1);
    // the pool at LDS 0, then the state machine's table, then the rest
    const size_t sm_at = lds_rules ? (pool.size() + 15) & ~size_t(15) : 0;
    const size_t lds_used = sm_at + kConnStateEntries;
    a.sm_lds = uint32_t(sm_at);
    int cmode = 0;
    if (count && n_ctr) cmode = lds_used + conn_lds_ctr_bytes(n_ctr) <= lds_max && !(no_lds & 2) ? 1 : 2;
    a.ctr_lds = uint32_t(lds_used);
    // the call's tables, uploaded only when they differ from the last upload
    // (same bindings, same batch kind: nothing to copy)
    auto upload = [&](DevBuf& d, std::vector<uint8_t>& last, const void* src, size_t bytes, size_t min_bytes) -> int {
        const void* was = d.p;
        HIPC(e, grow(d, std::max(bytes, min_bytes)));
        const uint8_t* b = static_cast<const uint8_t*>(src);
        if (d.p == was && last.size() == bytes && (bytes == 0 || std::memcmp(last.data(), b, bytes) == 0))
            return CLS_OK;
        const int qrc = conn_quiesce(e);                 // an earlier copy may still read `last`
        if (qrc != CLS_OK) return qrc;
        last.assign(b, b + bytes);
        // from the engine's copy: it outlives the call (an unsynchronised
        // batch, sync = false, may still be copying when this returns)
        if (bytes) HIPC(e, hipMemcpyAsync(d.p, last.data(), bytes, hipMemcpyHostToDevice, s));
        return CLS_OK;
    };
    if (e->up_plan != P.id) {                             // a kept plan's tables are on the device already
        int rc = upload(e->s_desc, e->up_desc, desc.data(), desc.size() * sizeof(ConnDesc), sizeof(ConnDesc));
        if (rc == CLS_OK) rc = upload(e->s_ifs, e->up_ifs, ifs.data(), ifs.size() * sizeof(IfAcls), sizeof(IfAcls));
        if (rc == CLS_OK) rc = upload(e->s_rules, e->up_rules, pool.data(), pool.size(), 16);
        if (rc != CLS_OK) return rc;
        e->up_plan = dev ? P.id : ~0ull;
    }
    a.desc = e->s_desc.as<ConnDesc>();
    a.pre = big.empty() ? nullptr : e->s_pre.as<uint32_t>();
    a.pre_stride = stride;
    a.pre_rules = pre_rules ? 1u : 0u;
    a.pre_bytes = pre_bytes;
    a.n_big = uint32_t(big.size());
    a.bm_steps = P.bm_steps;
    a.ifs = e->s_ifs.as<IfAcls>();
    a.rules = e->s_rules.p;
    std::vector<unsigned long long*> tctr;
    if (cmode) {
        // the call counters are zero between calls (the scatter launch clears
        // what it moves); cleared here only when (re)allocated
        const size_t had = e->s_cctr.bytes;
        HIPC(e, grow(e->s_cctr, size_t(n_ctr) * 8 * kConnCtrCopies));
        if (e->s_cctr.bytes != had || !e->cctr_zero)
            HIPC(e, hipMemsetAsync(e->s_cctr.p, 0, e->s_cctr.bytes, s));
        // zero again only once the scatter launch (which clears what it
        // moves) is queued: an early return below forces the memset next time
        e->cctr_zero = false;
        a.ctr = e->s_cctr.as<unsigned long long>();
        for (size_t j = 0; j < dtab.size(); ++j) {
            Table& t = *dtab[j];
            if (!t.d_conn_ctr.p) {
                HIPC(e, t.d_conn_ctr.ensure(size_t(t.n_rules + 1) * 8));
                HIPC(e, hipMemsetAsync(t.d_conn_ctr.p, 0, size_t(t.n_rules + 1) * 8, s));
            }
            if (t.conn_ctr_ev && s != e->stream) HIPC(e, hipStreamWaitEvent(s, t.conn_ctr_ev, 0));
            tctr.push_back(t.d_conn_ctr.as<unsigned long long>());
        }
        const int rc = upload(e->s_tctr, e->up_tctr, tctr.data(), tctr.size() * sizeof(void*), sizeof(void*));
        if (rc != CLS_OK) return rc;
    }
    // The descriptor and interface tables go to LDS after the pool and the
    // counters when they fit (else the kernel reads them from global memory).
    // Persistent grid: as many 512-thread workgroups per CU as the LDS
    // allows, at most three (the kernel's registers allow 24 waves per CU);
    // else two of 768 threads, two of 512 or one of 1024 (plan_of below).
    a.n_desc = uint32_t(desc.size());
    const size_t meta = desc.size() * sizeof(ConnDesc) + ifs.size() * sizeof(IfAcls);
    // The launch's LDS plan for counters of ctr_b bytes: the descriptor and
    // interface tables after the pool and counters unless they would cost a
    // workgroup per CU, then (IPv4, `jobs`) the waves' job lists (512 B per
    // wave) on the same terms -- else the kernel's owner search and shuffles
    // (option conn_jobs=0: tests).  Counting with LDS counters and 16-byte
    // addresses, the kernel holds up to 96 VGPRs (kernels.hip connect_kernel):
    // at most two workgroups per CU.
    struct LdsPlan {
        size_t lds;
        uint32_t meta_lds, job_lds;
        int per_cu, block;
    };
    // Where three 512-thread workgroups do not fit but two 768-thread ones
    // do (the shared part -- pool, counters, tables -- is paid per
    // workgroup, the job lists per wave), the 768-thread shape keeps 24 waves
    // per CU instead of 16 (option conn_wg768=0: the 512 / 1024 shapes only).
    auto plan_of = [&](size_t ctr_b, bool jobs) {
        jobs = jobs && !k16 && e->opts.conn_jobs;
        const int cu_cap = std::min(cmode == 1 && k16 ? 2 : 3, e->opts.conn_wg_per_cu > 0 ? e->opts.conn_wg_per_cu : 3);
        auto shape = [&](int cap, int block) {
            auto per_cu_of = [&](size_t b) { return b ? std::max(1, std::min(cap, int(lds_max / b))) : cap; };
            LdsPlan q{lds_used + ctr_b, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
            const size_t meta_at = (q.lds + 15) & ~size_t(15);
            if (meta_at + meta <= lds_max && per_cu_of(meta_at + meta) == per_cu_of(q.lds) && !(no_lds & 4)) {
                q.meta_lds = uint32_t(meta_at);
                q.lds = meta_at + meta;
            }
            q.per_cu = per_cu_of(q.lds);
            q.block = block ? block : q.per_cu >= 2 ? 512 : 1024;
            const size_t job_at = (q.lds + 15) & ~size_t(15), job_b = size_t(q.block / 64) * 512;
            if (jobs && job_at + job_b <= lds_max && (q.per_cu == 1 || per_cu_of(job_at + job_b) == q.per_cu)) {
                q.job_lds = uint32_t(job_at);
                q.lds = job_at + job_b;
            }
            return q;
        };
        // (job lists first, then waves per CU)
        auto rank = [](const LdsPlan& p) { return (p.job_lds != 0xFFFFFFFFu ? 64 : 0) + p.per_cu * p.block / 64; };
        const LdsPlan q = shape(cu_cap, 0);
        if (cu_cap == 3 && e->opts.conn_wg768) {
            const LdsPlan r = shape(2, 768);
            if (r.per_cu == 2 && rank(r) > rank(q)) return r;
        }
        return q;
    };
    LdsPlan plan = plan_of(0, true);
    a.ctr16 = 0u;
    if (cmode == 1) {
        // LDS counters: u32, or u16 pairs (half the LDS, a bound on a
        // workgroup's connections); with job lists (at most two workgroups
        // per CU) or without (three where the LDS allows).  Option conn_plan
        // = 32j / 16j / 32s / 16s forces one (tests, measurements).
        const size_t b32 = size_t(n_ctr) * 4, b16 = conn_lds_ctr_bytes(n_ctr);
        const LdsPlan c[4] = {plan_of(b32, true), plan_of(b16, true), plan_of(b32, false), plan_of(b16, false)};
        int pick = -1;
        if (e->opts.conn_plan >= 0) {
            pick = e->opts.conn_plan;
            if (c[pick].lds > lds_max) pick = -1;
        }
        if (pick < 0) {
            // the job lists first, then waves per CU, then u16 (12 local
            // ACLs, ms per counted batch: 16j 0.1367, 32j 0.1379, 32s 0.1468, 16s
            // 0.1571; 64: 16j 0.2289, 32 (no room for job lists) 0.2367, 16s
            // 0.2449 -- profiles/r05zh_conn_counted_plans.txt)
            auto score = [&](int k) {
                return c[k].lds > lds_max ? -1 : (c[k].job_lds != 0xFFFFFFFFu ? 8 : 0) + c[k].per_cu * c[k].block / 256 +
                                            (k % 2 == 1);
            };
            pick = 0;
            for (int k = 1; k < 4; ++k)
                if (score(k) > score(pick)) pick = k;
        }
        plan = c[pick];
        a.ctr16 = pick % 2 ? 1u : 0u;
    }
    size_t lds = plan.lds;
    a.meta_lds = plan.meta_lds;
    a.job_lds = plan.job_lds;
    const int per_cu = plan.per_cu, block = plan.block;
    // Persistent grid: as many 512-thread workgroups per CU as the LDS
    // allows, at most three (the kernel's registers allow 24 waves per CU);
    // where it allows only one, one 1024-thread workgroup.  u16 counters: at
    // most kConnWgConns connections per workgroup -- a larger batch runs k
    // full rounds of the resident grid (equal workgroups, no partial round)
    const uint64_t resident = uint64_t(e->n_cu) * per_cu;
    uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(resident, (n + block - 1) / block));
    if (a.ctr16) {
        const uint64_t per_wg = uint64_t(kConnWgConns / block) * block;
        if (n > grid * per_wg) grid = resident * ((n + resident * per_wg - 1) / (resident * per_wg));
    }
    if (e->opts.debug_conn) {              // diagnostics: the launch's LDS plan
        size_t nbm = 0;
        for (const ConnDesc& d : desc) nbm += d.bm_off != 0xFFFFFFFFu;
        std::fprintf(stderr, "connect: n %llu desc %zu big %zu bitmaps %zu pool %zu lds_rules %d ctr %u cmode %d "
                     "meta %s jobs %s lds %zu ctr16 %u per_cu %d block %d grid %llu bm_steps %u\n", (unsigned long long)n,
                     desc.size(), big.size(), nbm, pool.size(), int(lds_rules), n_ctr, cmode,
                     a.meta_lds != 0xFFFFFFFFu ? "lds" : "global", a.job_lds != 0xFFFFFFFFu ? "lds" : "shuffle",
                     lds,
                     a.ctr16, per_cu, block, (unsigned long long)grid, P.bm_steps);
    }
    // LDS counters leave the launch as one row per workgroup, summed into the
    // tables' counters by the rows launch (option conn_flush_atomic: device
    // atomics into the copies of the call counters and the scatter launch,
    // tests)
    const uint32_t nw = a.ctr16 ? (n_ctr + 1u) / 2u : n_ctr;
    a.ctr_rows = nullptr;
    if (cmode == 1 && n && !e->opts.conn_flush_atomic) {
        HIPC(e, grow(e->s_crows, size_t(grid) * nw * 4));
        a.ctr_rows = e->s_crows.as<uint32_t>();
    }
    HIPC(e, launch_connect(a, k16, lds_rules, cmode, int(grid), block, lds, s));
    if (cmode && n) {
        uint32_t max_rules = 0;
        for (const ConnDesc& d : desc) max_rules = std::max(max_rules, d.n_rules);
        if (a.ctr_rows) {
            HIPC(e, launch_conn_rows(a.ctr_rows, uint32_t(grid), nw, a.ctr16 != 0, n_ctr, a.desc,
                                     uint32_t(desc.size()), e->s_tctr.as<unsigned long long* const>(), s));
        } else {
            HIPC(e, launch_conn_scatter(a.desc, e->s_tctr.as<unsigned long long* const>(), uint32_t(desc.size()),
                                        max_rules, e->s_cctr.as<unsigned long long>(), kConnCtrCopies, true, n_ctr,
                                        s));
        }
        e->cctr_zero = true;
        // cls_conn_counters waits for this batch's scatter, not the device:
        // it reads on the engine's stream, so a batch on that stream needs no
        // event (and every earlier batch is ordered before it, conn_last);
        // one on another stream records one (an event per batch cost the
        // stream ~5 us, profiles/r06u_conn_default_12_batches.txt)
        std::shared_ptr<SharedEvent> ev;
        if (s != e->stream) {
            for (auto& x : e->conn_evs)
                if (x.use_count() == 1) {
                    ev = x;
                    break;
                }
            if (!ev) {
                ev = std::make_shared<SharedEvent>();
                HIPC(e, hipEventCreateWithFlags(&ev->ev, hipEventDisableTiming));
                e->conn_evs.push_back(ev);
            }
            HIPC(e, hipEventRecord(ev->ev, s));
        }
        for (size_t j = 0; j < dtab.size(); ++j) dtab[j]->conn_ev = ev;
    } else if (cmode) {
        e->cctr_zero = true;            // n == 0: nothing was counted
    }
    if (!dev && n) HIPC(e, hipMemcpyAsync(out, o, n, hipMemcpyDeviceToHost, s));
    // a host batch returns with its verdicts; a device batch is
    // stream-ordered (conn_last: its scratch is reused only behind it)
    if (sync || !dev) {
        HIPC(e, hipStreamSynchronize(s));
        e->conn_last = nullptr;
    } else if (n) {
        e->conn_last = s;
    }
    return CLS_OK;
}

extern "C" {

int cls_stream_floor_conn(cls_engine* e, const cls_conn_soa* c, uint64_t n, uint8_t* out, uint32_t reps,
                          float* ms, void* stream) {
    if (!e || !c || !out || !ms || c->pkt.af != CLS_AF_V4 || n < 4 || n > kClsChunk) return CLS_E_INVAL;
    const cls_pkt_soa& pk = c->pkt;
    if (!aligned(pk.src4, 16) || !aligned(pk.dst4, 16) || !aligned(c->src_if, 16) || !aligned(c->dst_if, 16) ||
        !aligned(pk.sport, 8) || !aligned(pk.dport, 8) || !aligned(pk.proto, 4) || !aligned(out, 4))
        return fail(e, CLS_E_INVAL, "cls_stream_floor_conn: device arrays must be 16/8/4-byte aligned");
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    ConnArgs a{};
    a.src = pk.src4; a.dst = pk.dst4; a.src_if = c->src_if; a.dst_if = c->dst_if;
    a.sport = pk.sport; a.dport = pk.dport; a.proto = pk.proto; a.out = out; a.n = n;
    const int grid = int(std::min<uint64_t>(uint64_t(e->n_cu) * 2, (n / 4 + 1023) / 1024));
    hipEvent_t t0, t1;
    HIPC(e, hipEventCreate(&t0));
    HIPC(e, hipEventCreate(&t1));
    HIPC(e, launch_stream_conn(a, grid, s));          // warm
    HIPC(e, hipEventRecord(t0, s));
    for (uint32_t r = 0; r < std::max(1u, reps); ++r) HIPC(e, launch_stream_conn(a, grid, s));
    HIPC(e, hipEventRecord(t1, s));
    HIPC(e, hipEventSynchronize(t1));
    float t = 0.f;
    HIPC(e, hipEventElapsedTime(&t, t0, t1));
    *ms = t / float(std::max(1u, reps));
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    return CLS_OK;
}

// One device's connection counters of a table, added to `acc`: waits for
// the last counting batch's scatter and a rebind's clearing (events), not
// for other work on the device.
static int conn_counters_dev(cls_engine* d, uint32_t table_id, std::vector<uint64_t>& acc, uint32_t reset) {
    auto it = d->tables.find(table_id);
    if (it == d->tables.end()) return fail(d, CLS_E_NOTFOUND, "no table %u", table_id);
    Table& t = *it->second;
    if (!t.d_conn_ctr.p) return CLS_OK;
    HIPC(d, hipSetDevice(d->device));
    const size_t bytes = size_t(t.n_rules + 1) * 8;
    std::vector<uint64_t> h(t.n_rules + 1);
    if (t.conn_ev) HIPC(d, hipStreamWaitEvent(d->stream, t.conn_ev->ev, 0));
    if (t.conn_ctr_ev) HIPC(d, hipStreamWaitEvent(d->stream, t.conn_ctr_ev, 0));
    HIPC(d, hipMemcpyAsync(h.data(), t.d_conn_ctr.p, bytes, hipMemcpyDeviceToHost, d->stream));
    if (reset) HIPC(d, hipMemsetAsync(t.d_conn_ctr.p, 0, bytes, d->stream));
    HIPC(d, hipStreamSynchronize(d->stream));
    for (size_t i = 0; i < h.size(); ++i) acc[i] += h[i];
    return CLS_OK;
}

int cls_conn_counters(cls_engine* e, uint32_t table_id, uint64_t* counters_out, uint32_t reset) {
    if (!e || !counters_out) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    auto it = e->tables.find(table_id);
    if (it == e->tables.end()) return fail(e, CLS_E_NOTFOUND, "no table %u", table_id);
    std::vector<uint64_t> acc(size_t(it->second->n_rules) + 1, 0);
    // a multi-device engine: the sum over its devices (each counts its own
    // shard of every connection batch)
    for (size_t i = 0; i < n_dev_engines(e); ++i) {
        cls_engine* d = dev_engine(e, i);
        std::unique_lock<std::mutex> lk(d->mu, std::defer_lock);
        if (d != e) lk.lock();
        const int rc = conn_counters_dev(d, table_id, acc, reset);
        if (rc != CLS_OK) return d == e ? rc : fail(e, rc, "device %d: %s", d->device, d->err.c_str());
    }
    std::memcpy(counters_out, acc.data(), acc.size() * 8);
    return CLS_OK;
}

// ---------------------------------------------------------------------------
int cls_gen_traffic_v4(cls_engine* e, const cls_traffic_spec* sp, uint64_t first, uint64_t n,
                       uint32_t* src4, uint32_t* dst4, uint16_t* sport, uint16_t* dport,
                       uint8_t* proto, void* stream) {
    if (!e || !sp) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    return gen4_locked(e, sp, first, n, src4, dst4, sport, dport, proto, stream, true);
}

}  // extern "C"

int gen4_locked(cls_engine* e, const cls_traffic_spec* sp, uint64_t first, uint64_t n, uint32_t* src4,
                uint32_t* dst4, uint16_t* sport, uint16_t* dport, uint8_t* proto, void* stream, bool sync) {
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    const size_t bp = size_t(sp->n_pod_ips) * 4, bd = size_t(sp->n_dst) * 4, bl = sp->n_dst,
                 bq = size_t(sp->n_ports) * 2;
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    HIPC(e, e->s_pool.ensure(al(bp) + al(bd) + al(bl) + al(bq) + 16));
    uint8_t* base = e->s_pool.as<uint8_t>();
    TrafficDev t;
    t.seed = sp->seed;
    t.pct_pod = sp->pct_pod_src; t.pct_dst = sp->pct_rule_dst;
    t.pct_port = sp->pct_table_port; t.pct_icmp = sp->pct_icmp;
    t.pods = reinterpret_cast<const uint32_t*>(base); t.n_pods = sp->n_pod_ips;
    t.dst_addrs = reinterpret_cast<const uint32_t*>(base + al(bp));
    t.dst_lens = base + al(bp) + al(bd); t.n_dst = sp->n_dst;
    t.ports = reinterpret_cast<const uint16_t*>(base + al(bp) + al(bd) + al(bl)); t.n_ports = sp->n_ports;
    if (bp) HIPC(e, hipMemcpyAsync(base, sp->pod_ips, bp, hipMemcpyHostToDevice, s));
    if (bd) HIPC(e, hipMemcpyAsync(base + al(bp), sp->dst_addrs, bd, hipMemcpyHostToDevice, s));
    if (bl) HIPC(e, hipMemcpyAsync(base + al(bp) + al(bd), sp->dst_lens, bl, hipMemcpyHostToDevice, s));
    if (bq) HIPC(e, hipMemcpyAsync(base + al(bp) + al(bd) + al(bl), sp->ports, bq, hipMemcpyHostToDevice, s));
    HIPC(e, launch_gen4(t, first, n, src4, dst4, sport, dport, proto, s));
    // the pools are engine scratch (sync = false: the caller synchronises
    // before the next use)
    if (sync) HIPC(e, hipStreamSynchronize(s));
    return CLS_OK;
}

extern "C" {

// Blob of cls_compile_v4 / cls_compile_v16: header (v4 header, then `extra`
// bytes of a larger header), image, slot -> rule map, linear rules.
static int write_blob(const Cls4Image* img, const std::vector<LinRule4>& lin, uint32_t n, uint32_t magic,
                      const void* extra, size_t extra_bytes, void* blob, uint64_t cap, uint64_t* need,
                      const std::vector<uint32_t>* trailer = nullptr, size_t trailer_field = 0,
                      const Cls4Image* other = nullptr) {
    cls_image_v4_header h;
    std::memset(&h, 0, sizeof h);
    h.magic = magic;
    h.version = 4;
    h.n_rules = n;
    h.n_lin = uint32_t(lin.size());
    h.has_cls = img ? 1u : 0u;
    if (img) {
        const Cls4Image& im = *img;
        h.img_bytes = im.img_bytes; h.off_bounds = im.off_bounds; h.off_iclass = im.off_iclass;
        h.off_cells = im.off_cells; h.off_lists = im.off_lists; h.off_tmpl = im.off_tmpl;
        h.n_bounds = im.n_bounds; h.search_top = im.search_top; h.n_classes = im.n_classes;
        h.n_tmpl = im.n_tmpl; h.n_list_entries = im.n_list_entries; h.n_ctr = im.n_ctr;
        h.lds_bytes = im.lds_bytes;
        h.mode = im.mode;
        h.default_class = im.default_class;
        h.n_hash = im.n_hash;
        h.list_mode = im.list_mode;
        h.off_bv = im.off_bv;
        h.bv_steps_d = im.bv_steps_d;
        h.bv_steps_p = im.bv_steps_p;
        h.off_ptop = im.off_ptop;
        h.n_pclass = im.n_pclass;
        h.bv_wide = im.bv_wide;
        h.row_bytes = im.row_bytes;
        h.port_mul = im.port_mul;
        h.port_mask4 = im.port_mask4;
        h.port_dflt = im.port_dflt;
        h.default_row = im.default_row;
        h.n_hot = im.n_hot;
        h.off_hot = im.off_hot;
        h.n_lctr = im.n_lctr;
        h.ctr16 = im.ctr16;
        h.swap = im.swap;
        h.off_trie = im.off_trie;
        h.trie_depth = im.trie_depth;
        h.n_gcells = uint32_t(im.gcells.size());
        for (uint32_t i = 0; i < kMaxHashLens; ++i) {
            h.hash_mask[i] = im.hash_mask[i];
            h.hash_shift[i] = im.hash_shift[i];
            h.hash_cap[i] = im.hash_cap[i];
            h.hash_mul[i] = im.hash_mul[i];
            h.off_hash[i] = im.off_hash[i];
        }
    }
    auto al = [](uint64_t x) { return (x + 15) & ~uint64_t(15); };
    h.off_image = uint32_t(al(sizeof h + extra_bytes));
    h.off_ctr_rule = uint32_t(al(h.off_image + h.img_bytes));
    h.off_lin = uint32_t(al(h.off_ctr_rule + uint64_t(h.n_ctr) * 4));
    h.total_bytes = uint32_t(h.off_lin + lin.size() * sizeof(LinRule4));
    if (h.n_gcells) {
        h.off_gcells = uint32_t(al(h.total_bytes));
        h.total_bytes = h.off_gcells + h.n_gcells * 4u;
    }
    const uint32_t off_trailer = uint32_t(al(h.total_bytes));
    if (trailer) h.total_bytes = off_trailer + uint32_t(trailer->size() * 4);
    uint64_t need_o = 0;                      // the OTHER image: a nested blob (magic "CLSO")
    if (other) {
        write_blob(other, {}, n, 0x434C534Fu, nullptr, 0, nullptr, 0, &need_o);
        h.off_other = uint32_t(al(h.total_bytes));
        h.total_bytes = h.off_other + uint32_t(need_o);
    }
    *need = h.total_bytes;
    if (!blob || cap < h.total_bytes) return CLS_OK;
    uint8_t* b = static_cast<uint8_t*>(blob);
    std::memset(b, 0, h.total_bytes);
    std::memcpy(b, &h, sizeof h);
    if (extra_bytes) std::memcpy(b + sizeof h, extra, extra_bytes);
    if (trailer) {
        std::memcpy(b + sizeof h + trailer_field, &off_trailer, 4);   // extra header field: trailer offset
        std::memcpy(b + off_trailer, trailer->data(), trailer->size() * 4);
    }
    if (img) {
        std::memcpy(b + h.off_image, img->words.data(), img->img_bytes);
        std::memcpy(b + h.off_ctr_rule, img->ctr_rule.data(), size_t(h.n_ctr) * 4);
        if (h.n_gcells) std::memcpy(b + h.off_gcells, img->gcells.data(), size_t(h.n_gcells) * 4);
    }
    if (!lin.empty()) std::memcpy(b + h.off_lin, lin.data(), lin.size() * sizeof(LinRule4));
    if (other) write_blob(other, {}, n, 0x434C534Fu, nullptr, 0, b + h.off_other, need_o, &need_o);
    return CLS_OK;
}

int cls_gen_traffic_v16(cls_engine* e, const cls_traffic_spec16* sp, uint64_t first, uint64_t n,
                        uint8_t* src16, uint8_t* dst16, uint16_t* sport, uint16_t* dport, uint8_t* proto,
                        void* stream) {
    if (!e || !sp) return CLS_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const DeviceGuard dg;        // the caller's device again on return
    return gen16_locked(e, sp, first, n, src16, dst16, sport, dport, proto, stream, true);
}

}  // extern "C"

int gen16_locked(cls_engine* e, const cls_traffic_spec16* sp, uint64_t first, uint64_t n, uint8_t* src16,
                 uint8_t* dst16, uint16_t* sport, uint16_t* dport, uint8_t* proto, void* stream, bool sync) {
    if ((src16 && !aligned(src16, 16)) || (dst16 && !aligned(dst16, 16)))
        return fail(e, CLS_E_INVAL, "src16/dst16 must be 16-byte aligned");
    HIPC(e, hipSetDevice(e->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
    // pools as (hi, lo) u64 pairs in address order
    auto pairs = [](const uint8_t* b, uint32_t m) {
        std::vector<uint64_t> v(size_t(m) * 2, 0);
        for (uint32_t j = 0; j < m; ++j)
            for (int k = 0; k < 16; ++k) v[2 * j + k / 8] = (v[2 * j + k / 8] << 8) | b[16 * size_t(j) + k];
        return v;
    };
    // the pairs live in the engine (an unsynchronised upload still reads
    // them after the call returns); an earlier such upload finishes first
    if (e->gen_pending) HIPC(e, hipStreamSynchronize(s));
    e->gen_pending = false;
    const std::vector<uint64_t> pods = pairs(sp->pod_ips, sp->n_pod_ips), dsta = pairs(sp->dst_addrs, sp->n_dst);
    std::vector<uint64_t>& hp = e->gen_pairs;
    hp.assign(pods.begin(), pods.end());
    hp.insert(hp.end(), dsta.begin(), dsta.end());
    const size_t bp = pods.size() * 8, bd = dsta.size() * 8, bl = sp->n_dst, bq = size_t(sp->n_ports) * 2;
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    HIPC(e, e->s_pool.ensure(al(bp) + al(bd) + al(bl) + al(bq) + 16));
    uint8_t* base = e->s_pool.as<uint8_t>();
    TrafficDev16 t;
    t.seed = sp->seed;
    t.pct_pod = sp->pct_pod_src; t.pct_dst = sp->pct_rule_dst;
    t.pct_port = sp->pct_table_port; t.pct_icmp = sp->pct_icmp;
    t.pods = reinterpret_cast<const uint64_t*>(base); t.n_pods = sp->n_pod_ips;
    t.dst_addrs = reinterpret_cast<const uint64_t*>(base + al(bp));
    t.dst_lens = base + al(bp) + al(bd); t.n_dst = sp->n_dst;
    t.ports = reinterpret_cast<const uint16_t*>(base + al(bp) + al(bd) + al(bl)); t.n_ports = sp->n_ports;
    if (bp) HIPC(e, hipMemcpyAsync(base, hp.data(), bp, hipMemcpyHostToDevice, s));
    if (bd) HIPC(e, hipMemcpyAsync(base + al(bp), hp.data() + pods.size(), bd, hipMemcpyHostToDevice, s));
    if (bl) HIPC(e, hipMemcpyAsync(base + al(bp) + al(bd), sp->dst_lens, bl, hipMemcpyHostToDevice, s));
    if (bq) HIPC(e, hipMemcpyAsync(base + al(bp) + al(bd) + al(bl), sp->ports, bq, hipMemcpyHostToDevice, s));
    e->gen_pending = !sync;
    HIPC(e, launch_gen16(t, first, n, reinterpret_cast<uint4*>(src16), reinterpret_cast<uint4*>(dst16), sport, dport,
                         proto, s));
    if (sync) HIPC(e, hipStreamSynchronize(s));   // the pools are engine scratch
    return CLS_OK;
}

extern "C" {

int cls_compile_v4(const cls_rule* rules, uint32_t n, void* blob, uint64_t cap, uint64_t* need,
                   const char* options) {
    if ((n && !rules) || !need) return CLS_E_INVAL;
    std::vector<SemRule> sem;
    std::string why;
    Opts o;
    if (!opts_parse(o, options, why)) return CLS_E_INVAL;
    const CompileScope scope(o);
    int rc = semantic_rules(rules, n, 4, sem, why);
    if (rc != CLS_OK) return rc;
    std::vector<LinRule4> lin = linear4(sem);
    Cls4Image img, oimg;
    const bool has = sem.size() > 8 && build_pair(sem, n, img, oimg, why);
    if (has && o.pair4) {
        // (option pair4: the connection pair launch's four-cell image, in the
        // main image's orientation, instead -- CPU tests of that compile)
        Cls4Image pimg;
        if (!build_pair4(sem, n, img.swap != 0, pimg, why)) return CLS_E_INVAL;
        return write_blob(&pimg, lin, n, 0x434C5334u, nullptr, 0, blob, cap, need, nullptr, 0, nullptr);
    }
    return write_blob(has ? &img : nullptr, lin, n, 0x434C5334u, nullptr, 0, blob, cap, need, nullptr, 0,
                      has ? &oimg : nullptr);
}

// Diagnostics (CPU tests): the connection path's bitmap form of an ACL
// (conn_bitmap4) evaluated on the host, exactly as conn_bm reads it.
int cls_conn_bitmap_eval(const cls_rule* rules, uint32_t n_rules, const uint32_t* src, const uint32_t* dst,
                         const uint16_t* dport, const uint8_t* proto, uint64_t n, uint8_t* res_out,
                         uint32_t* rule_out) {
    if ((n_rules && !rules) || (n && (!src || !dst || !dport || !proto || !res_out || !rule_out)))
        return CLS_E_INVAL;
    std::vector<SemRule> sem;
    std::string why;
    const int rc = semantic_rules(rules, n_rules, 4, sem, why);
    if (rc != CLS_OK) return rc;
    std::vector<uint32_t> w;
    if (!conn_bitmap4(conn_rules4(sem), n_rules, size_t(1) << 26, w)) return CLS_E_NOMEM;
    const uint32_t W = w[0], ns = w[1], nd = w[2], np[4] = {w[4], w[5], w[6], w[7]};
    const uint32_t os = kConnBmHeader / 4, od = os + ns * (1 + W), t0 = od + nd * (1 + W);
    const uint32_t t1 = t0 + np[0] * (1 + W), t2 = t1 + np[1] * (1 + W), t3 = t2 + np[2] * (1 + W);
    const uint32_t orl = t3 + np[3] * (1 + W);
    auto row = [&](uint32_t o, uint32_t cnt, uint32_t x) {       // last key <= x (key 0 first)
        uint32_t pos = 0;
        for (uint32_t i = 1; i < cnt; ++i)
            if (w[o + i] <= x) pos = i;
        return o + cnt + W * pos;
    };
    for (uint64_t k = 0; k < n; ++k) {
        const uint32_t p = proto[k] <= 2 ? proto[k] : 3u;
        const uint32_t tp[4] = {t0, t1, t2, t3};
        const uint32_t sr = row(os, ns, src[k]), dr = row(od, nd, dst[k]), pr = row(tp[p], np[p], dport[k]);
        res_out[k] = 0;
        rule_out[k] = n_rules;
        for (uint32_t j = 0; j < W; ++j) {
            const uint32_t m = w[sr + j] & w[dr + j] & w[pr + j];
            if (m) {
                const uint32_t i = 32 * j + uint32_t(__builtin_ctz(m));
                res_out[k] = uint8_t((w[orl + 2 * i] >> (8 * p)) & 3u);
                rule_out[k] = w[orl + 2 * i + 1];
                break;
            }
        }
    }
    return CLS_OK;
}

int cls_compile_v16(const cls_rule* rules, uint32_t n, void* blob, uint64_t cap, uint64_t* need,
                    const char* options) {
    if ((n && !rules) || !need) return CLS_E_INVAL;
    std::vector<SemRule> sem;
    std::string why;
    Opts o;
    if (!opts_parse(o, options, why)) return CLS_E_INVAL;
    const CompileScope scope(o);
    int rc = semantic_rules(rules, n, 0, sem, why);
    if (rc != CLS_OK) return rc;
    Cls16Image img;
    Cls4Image oimg;
    if (!build_cls16(sem, n, img, why) || !build_other4(img.sem, n, oimg, why)) return CLS_E_INVAL;
    cls_image_v16_header h16;
    std::memset(&h16, 0, sizeof h16);
    for (int sd = 0; sd < 2; ++sd) {
        h16.fe_key[sd] = img.fe_key[sd];
        h16.fe_val[sd] = img.fe_val[sd];
        h16.fe_top[sd] = img.fe_top[sd];
        h16.fe_n[sd] = img.fe_n[sd];
        h16.fe_k8[sd] = img.fe_k8[sd];
    }
    h16.src_mode = img.src_mode;
    h16.h4 = img.h4; h16.cap4 = img.cap4; h16.mul4 = img.mul4;
    h16.k6 = img.k6; h16.r6 = img.r6; h16.cap6 = img.cap6; h16.mul6 = img.mul6;
    for (int i = 0; i < 3; ++i) h16.fold[i] = img.fold[i];
    h16.dflt_row[0] = img.dflt_row[0];
    h16.dflt_row[1] = img.dflt_row[1];
    h16.src_search_val = img.src_search_val;
    h16.src_search_top = img.src_search_top;
    h16.src_search_k8 = img.src_search_k8;
    const size_t extra = sizeof h16 - sizeof h16.core;
    return write_blob(&img.core, linear4(img.sem), n, 0x434C3136u, reinterpret_cast<const uint8_t*>(&h16) + sizeof h16.core,
                      extra, blob, cap, need, img.src_mode >= 1 ? &img.src_search : nullptr,
                      offsetof(cls_image_v16_header, off_src_search) - sizeof h16.core, &oimg);
}

}  // extern "C"
