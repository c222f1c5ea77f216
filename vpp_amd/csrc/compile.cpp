// Rule-set compiler (see compile.hpp for the design).
#include "compile.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <unordered_map>

namespace cls {

namespace {

constexpr uint32_t kMaxPort = 65535u;

bool nonempty(const char* s) { return s != nullptr && s[0] != '\0'; }

uint8_t action_result(const cls_rule& r) {
    if (!(r.flags & CLS_R_ACTIONS)) return RES_FAIL;          // aclengine_mock.go:646-650
    switch (r.acl_action) {                                  // :655-664
    case CLS_ACTION_DENY: return RES_DENY;
    case CLS_ACTION_PERMIT: return RES_PERMIT;
    case CLS_ACTION_REFLECT: return RES_REFLECT;
    default: return RES_FAIL;
    }
}

Term fail_term() {
    Term t;
    t.term = true;
    t.lo = 0; t.hi = 0xFFFF;
    t.res = RES_FAIL;
    return t;
}

// TCP/UDP section of evalACL's protocol switch (:528-598)
Term l4_term(const cls_rule& r, int p, uint8_t res) {
    const bool tcp = p == P_TCP;
    const uint32_t has = tcp ? CLS_R_TCP : CLS_R_UDP;
    const uint32_t sibling = tcp ? CLS_R_UDP : CLS_R_TCP;
    const uint32_t hsrc = tcp ? CLS_R_TCP_SRC : CLS_R_UDP_SRC;
    const uint32_t hdst = tcp ? CLS_R_TCP_DST : CLS_R_UDP_DST;
    const uint32_t slo = tcp ? r.tcp_src_lo : r.udp_src_lo;
    const uint32_t shi = tcp ? r.tcp_src_hi : r.udp_src_hi;
    const uint32_t dlo = tcp ? r.tcp_dst_lo : r.udp_dst_lo;
    const uint32_t dhi = tcp ? r.tcp_dst_hi : r.udp_dst_hi;
    Term t;
    if ((r.flags & sibling) || (r.flags & CLS_R_ICMP)) return t;        // continue
    if (!(r.flags & has)) return fail_term();
    if (!(r.flags & hsrc) || slo != 0 || shi != kMaxPort) return fail_term();
    if (!(r.flags & hdst)) return fail_term();
    const uint16_t lo = static_cast<uint16_t>(dlo), hi = static_cast<uint16_t>(dhi);  // uint16() casts, :559
    if (lo > hi) return t;                                              // never inside [lo, hi]
    t.term = true; t.lo = lo; t.hi = hi; t.res = res;
    return t;
}

// ICMP case (:600-642)
Term icmp_term(const cls_rule& r, uint8_t res) {
    Term t;
    if ((r.flags & CLS_R_TCP) || (r.flags & CLS_R_UDP)) return t;
    if (!(r.flags & CLS_R_ICMP)) return fail_term();
    if (!(r.flags & CLS_R_ICMP_CODE) || r.icmp_code_first != 0 || r.icmp_code_last != 5)
        return fail_term();
    if (!(r.flags & CLS_R_ICMP_TYPE) || r.icmp_type_first != 0 || r.icmp_type_last != 16)
        return fail_term();
    if (r.flags & CLS_R_ICMPV6) return fail_term();
    t.term = true; t.lo = 0; t.hi = 0xFFFF; t.res = res;   // ICMP ignores the port
    return t;
}

SemRule terminator(uint32_t k) {
    SemRule s;
    s.index = k;
    for (auto& t : s.t) t = fail_term();
    return s;
}

bool matches_everything(const SemRule& s) {
    if (!s.src_any || !s.dst_any) return false;
    for (const auto& t : s.t)
        if (!t.term || t.lo != 0 || t.hi != 0xFFFF) return false;
    return true;
}

inline uint32_t v4_word(const uint8_t* a) {
    return (uint32_t(a[0]) << 24) | (uint32_t(a[1]) << 16) | (uint32_t(a[2]) << 8) | a[3];
}
inline uint32_t v4_mask(int len) { return len ? (0xFFFFFFFFu << (32 - len)) : 0u; }

}  // namespace

int semantic_rules(const cls_rule* rules, uint32_t n, int fam, std::vector<SemRule>& out,
                   std::string& err) {
    out.clear();
    for (uint32_t k = 0; k < n; ++k) {
        const cls_rule& r = rules[k];
        if (!(r.flags & CLS_R_MATCHES)) {
            err = "rule " + std::to_string(k) + ": Matches is nil (evalACL would panic)";
            return CLS_E_INVAL;
        }
    }
    for (uint32_t k = 0; k < n; ++k) {
        const cls_rule& r = rules[k];
        // :481-496 unconditional failures
        if ((r.flags & CLS_R_MACIP) || !(r.flags & CLS_R_IPRULE) || (r.flags & CLS_R_OTHER) ||
            !(r.flags & CLS_R_IP)) {
            out.push_back(terminator(k));
            return CLS_OK;
        }
        SemRule s;
        s.index = k;
        if (nonempty(r.src_network)) {                       // :499-510
            s.src = parse_cidr(r.src_network);
            if (s.src.fam == 0) { out.push_back(terminator(k)); return CLS_OK; }
            if (s.src.fam != fam) continue;                  // never Contains() this family
            s.src_any = false;
        }
        bool dst_fail = false;
        if (nonempty(r.dst_network)) {                       // :513-524
            s.dst = parse_cidr(r.dst_network);
            if (s.dst.fam == 0) dst_fail = true;
            else if (s.dst.fam != fam) continue;
            else s.dst_any = false;
        }
        if (dst_fail) {
            s.dst_any = true;
            for (auto& t : s.t) t = fail_term();
        } else {
            const uint8_t res = action_result(r);
            s.t[P_TCP] = l4_term(r, P_TCP, res);
            s.t[P_UDP] = l4_term(r, P_UDP, res);
            s.t[P_ICMP] = icmp_term(r, res);
            s.t[P_OTHER].term = true;                        // no case: networks alone
            s.t[P_OTHER].res = res;
        }
        bool any_term = false;
        for (const auto& t : s.t) any_term |= t.term;
        if (!any_term) continue;
        out.push_back(s);
        if (matches_everything(s)) return CLS_OK;            // later rules unreachable
    }
    return CLS_OK;
}

static uint32_t pack_port(const Term& t) { return uint32_t(t.lo) | (uint32_t(t.hi - t.lo) << 16); }

static uint32_t pack_meta(const SemRule& s) {
    uint32_t m = 0;
    for (int p = 0; p < NPROTO; ++p)
        m |= uint32_t((s.t[p].term ? 0x80u : 0u) | s.t[p].res) << (8 * p);
    return m;
}

std::vector<LinRule4> linear4(const std::vector<SemRule>& sem) {
    std::vector<LinRule4> v(sem.size());
    for (size_t i = 0; i < sem.size(); ++i) {
        const SemRule& s = sem[i];
        LinRule4& l = v[i];
        std::memset(&l, 0, sizeof l);
        if (!s.src_any) { l.src_mask = v4_mask(s.src.len); l.src_addr = v4_word(s.src.addr) & l.src_mask; }
        if (!s.dst_any) { l.dst_mask = v4_mask(s.dst.len); l.dst_addr = v4_word(s.dst.addr) & l.dst_mask; }
        for (int p = 0; p < NPROTO; ++p) l.port[p] = pack_port(s.t[p]);
        l.meta = pack_meta(s);
        l.index = s.index;
    }
    return v;
}

std::vector<LinRule16> linear16(const std::vector<SemRule>& sem) {
    std::vector<LinRule16> v(sem.size());
    for (size_t i = 0; i < sem.size(); ++i) {
        const SemRule& s = sem[i];
        LinRule16& l = v[i];
        std::memset(&l, 0, sizeof l);
        l.src_any = s.src_any; l.dst_any = s.dst_any;
        if (!s.src_any) { std::memcpy(l.src_addr, s.src.addr, 16); l.src_len = uint8_t(s.src.len); }
        if (!s.dst_any) { std::memcpy(l.dst_addr, s.dst.addr, 16); l.dst_len = uint8_t(s.dst.len); }
        for (int p = 0; p < NPROTO; ++p) l.port[p] = pack_port(s.t[p]);
        l.meta = pack_meta(s);
        l.index = s.index;
    }
    return v;
}

// ---------------------------------------------------------------------------
// IPv4 classifier image
// ---------------------------------------------------------------------------
namespace {

struct Pfx {
    uint32_t addr;  // masked
    int len;
    uint64_t lo() const { return addr; }
    uint64_t hi() const { return uint64_t(addr) + ((uint64_t(1) << (32 - len)) - 1); }
    bool operator<(const Pfx& o) const { return addr != o.addr ? addr < o.addr : len < o.len; }
    bool operator==(const Pfx& o) const { return addr == o.addr && len == o.len; }
};

struct VecHash {
    size_t operator()(const std::vector<uint16_t>& v) const {
        uint64_t h = 1469598103934665603ull;
        for (uint16_t x : v) { h ^= x; h *= 1099511628211ull; }
        return size_t(h);
    }
};

struct TmplKey {
    uint32_t a, m, pw, res;
    bool operator==(const TmplKey& o) const { return a == o.a && m == o.m && pw == o.pw && res == o.res; }
};
struct TmplHash {
    size_t operator()(const TmplKey& k) const {
        uint64_t h = k.a * 0x9E3779B97F4A7C15ull ^ (uint64_t(k.m) << 32 | k.pw) * 0xC2B2AE3D27D4EB4Full ^ k.res;
        return size_t(h ^ (h >> 29));
    }
};

uint32_t align4(uint32_t w) { return (w + 3u) & ~3u; }

}  // namespace

bool build_cls4(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img,
                std::string& why) {
    img = Cls4Image();
    // distinct source prefixes
    std::vector<Pfx> pfx;
    for (const auto& s : sem)
        if (!s.src_any) pfx.push_back({v4_word(s.src.addr) & v4_mask(s.src.len), s.src.len});
    std::sort(pfx.begin(), pfx.end());
    pfx.erase(std::unique(pfx.begin(), pfx.end()), pfx.end());
    std::map<std::pair<uint32_t, int>, int> pfx_id;
    for (size_t i = 0; i < pfx.size(); ++i) pfx_id[{pfx[i].addr, pfx[i].len}] = int(i);

    // elementary interval boundaries
    std::vector<uint32_t> bounds{0u};
    for (const auto& p : pfx) {
        bounds.push_back(p.addr);
        if (p.hi() < 0xFFFFFFFFull) bounds.push_back(uint32_t(p.hi() + 1));
    }
    std::sort(bounds.begin(), bounds.end());
    bounds.erase(std::unique(bounds.begin(), bounds.end()), bounds.end());

    // sweep: longest covering prefix of each interval (prefixes are laminar)
    std::vector<int> lpm(bounds.size(), -1);
    {
        std::vector<int> stack;
        size_t next = 0;  // pfx sorted by (addr, len): containers before contained
        for (size_t k = 0; k < bounds.size(); ++k) {
            const uint64_t x = bounds[k];
            while (!stack.empty() && pfx[stack.back()].hi() < x) stack.pop_back();
            while (next < pfx.size() && pfx[next].lo() == x) stack.push_back(int(next++));
            lpm[k] = stack.empty() ? -1 : stack.back();
        }
    }
    // parent (next shorter covering prefix) of every prefix, for chains
    std::vector<int> parent(pfx.size(), -1);
    {
        std::vector<int> stack;
        for (size_t i = 0; i < pfx.size(); ++i) {
            while (!stack.empty() && pfx[stack.back()].hi() < pfx[i].lo()) stack.pop_back();
            parent[i] = stack.empty() ? -1 : stack.back();
            stack.push_back(int(i));
        }
    }
    // rules (positions in sem) by exact source prefix; ANY-source rules apart
    std::vector<std::vector<uint32_t>> by_pfx(pfx.size());
    std::vector<uint32_t> any_src;
    for (uint32_t i = 0; i < sem.size(); ++i) {
        const auto& s = sem[i];
        if (s.src_any) any_src.push_back(i);
        else by_pfx[pfx_id[{v4_word(s.src.addr) & v4_mask(s.src.len), s.src.len}]].push_back(i);
    }
    // classes = distinct LPM results (+ "no prefix")
    std::vector<int> class_of_pfx(pfx.size() + 1, -1);  // index 0 = none
    std::vector<int> class_pfx;
    std::vector<uint16_t> iclass(bounds.size());
    for (size_t k = 0; k < bounds.size(); ++k) {
        int key = lpm[k] + 1;
        if (class_of_pfx[key] < 0) {
            class_of_pfx[key] = int(class_pfx.size());
            class_pfx.push_back(lpm[k]);
        }
        if (class_of_pfx[key] > 0xFFFF) { why = "more than 65536 source classes"; return false; }
        iclass[k] = uint16_t(class_of_pfx[key]);
    }
    const uint32_t n_classes = uint32_t(class_pfx.size());
    const uint32_t n_real_bounds = uint32_t(bounds.size());
    // pad to 2*top entries so the branch-free search never needs a bound check:
    // sentinel 0xFFFFFFFF keeps the class of the last interval (which holds it)
    uint32_t top = 1;
    while (top * 2 <= n_real_bounds) top *= 2;
    bounds.resize(size_t(top) * 2, 0xFFFFFFFFu);
    iclass.resize(size_t(top) * 2, iclass[n_real_bounds - 1]);

    // templates, lists and cells
    std::unordered_map<TmplKey, uint32_t, TmplHash> tmpl_id;
    std::vector<TmplKey> tmpls;
    std::unordered_map<std::vector<uint16_t>, uint32_t, VecHash> list_id;
    std::vector<uint16_t> lists;
    std::vector<uint32_t> cells(size_t(n_classes) * 3 * 2);
    img.ctr_rule.assign(1, n_rules);  // slot 0: default DENY
    std::vector<uint32_t> cand;
    for (uint32_t c = 0; c < n_classes; ++c) {
        // merge candidate rule positions: chain of covering prefixes + ANY
        cand.clear();
        for (int p = class_pfx[c]; p >= 0; p = parent[p])
            cand.insert(cand.end(), by_pfx[p].begin(), by_pfx[p].end());
        cand.insert(cand.end(), any_src.begin(), any_src.end());
        std::sort(cand.begin(), cand.end());
        for (int pr = 0; pr < 3; ++pr) {
            std::vector<uint16_t> seq;
            const uint32_t ctr_base = uint32_t(img.ctr_rule.size());
            for (uint32_t pos : cand) {
                const SemRule& s = sem[pos];
                const Term& t = s.t[pr];
                if (!t.term) continue;
                TmplKey key{0, 0, pack_port(t), t.res};
                if (!s.dst_any) {
                    key.m = v4_mask(s.dst.len);
                    key.a = v4_word(s.dst.addr) & key.m;
                }
                auto it = tmpl_id.find(key);
                uint32_t id;
                if (it == tmpl_id.end()) {
                    id = uint32_t(tmpls.size());
                    if (id > 0xFFFF) { why = "more than 65536 templates"; return false; }
                    tmpl_id.emplace(key, id);
                    tmpls.push_back(key);
                } else {
                    id = it->second;
                }
                seq.push_back(uint16_t(id));
                img.ctr_rule.push_back(s.index);
                if (s.dst_any && t.lo == 0 && t.hi == 0xFFFF) break;  // catch-all for the cell
            }
            if (seq.size() > 0xFFFF) { why = "candidate list longer than 65535"; return false; }
            uint32_t start = 0;
            if (!seq.empty()) {
                auto it = list_id.find(seq);
                if (it == list_id.end()) {
                    start = uint32_t(lists.size());
                    list_id.emplace(seq, start);
                    lists.insert(lists.end(), seq.begin(), seq.end());
                } else {
                    start = it->second;
                }
            }
            if (start > 0xFFFF) { why = "candidate list storage exceeds 65536 entries"; return false; }
            cells[(size_t(c) * 3 + pr) * 2 + 0] = start | (uint32_t(seq.size()) << 16);
            cells[(size_t(c) * 3 + pr) * 2 + 1] = ctr_base;
        }
    }

    // serialise (u32 words, each section 16 B aligned)
    std::vector<uint32_t>& w = img.words;
    img.off_bounds = 0;
    w.insert(w.end(), bounds.begin(), bounds.end());
    w.resize(align4(uint32_t(w.size())));
    img.off_iclass = uint32_t(w.size()) * 4;
    w.resize(w.size() + (bounds.size() + 1) / 2);
    std::memcpy(reinterpret_cast<uint8_t*>(w.data()) + img.off_iclass, iclass.data(), iclass.size() * 2);
    w.resize(align4(uint32_t(w.size())));
    img.off_cells = uint32_t(w.size()) * 4;
    w.insert(w.end(), cells.begin(), cells.end());
    w.resize(align4(uint32_t(w.size())));
    img.off_lists = uint32_t(w.size()) * 4;
    {
        const size_t base = w.size();
        w.resize(base + (lists.size() + 1) / 2);
        if (!lists.empty())
            std::memcpy(reinterpret_cast<uint8_t*>(w.data() + base), lists.data(), lists.size() * 2);
    }
    w.resize(align4(uint32_t(w.size())));
    img.off_tmpl = uint32_t(w.size()) * 4;
    for (const auto& t : tmpls) {
        w.push_back(t.a);
        w.push_back(t.m);
        w.push_back(t.pw);
        w.push_back(t.res);
    }
    w.resize(align4(uint32_t(w.size())));
    img.img_bytes = uint32_t(w.size()) * 4;
    img.n_bounds = n_real_bounds;
    img.n_classes = n_classes;
    img.n_tmpl = uint32_t(tmpls.size());
    img.n_list_entries = uint32_t(lists.size());
    img.n_ctr = uint32_t(img.ctr_rule.size());
    img.search_top = top;
    img.lds_bytes = img.img_bytes + ((img.n_ctr * 4 + 15u) & ~15u);
    return true;
}

}  // namespace cls
