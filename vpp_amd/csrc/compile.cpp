// Rule-set compiler (see compile.hpp for the design).
#include "compile.hpp"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
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
            if (fam && s.src.fam != fam) continue;           // never Contains() this family
            s.src_any = false;
        }
        bool dst_fail = false;
        if (nonempty(r.dst_network)) {                       // :513-524
            s.dst = parse_cidr(r.dst_network);
            if (s.dst.fam == 0) dst_fail = true;
            else if (fam && s.dst.fam != fam) continue;
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

// An ICMP / OTHER term spans every port (the compact forms rely on it).
static void check_port_free(const SemRule& s) {
    for (int p = P_ICMP; p < NPROTO; ++p)
        if (s.t[p].term && (s.t[p].lo != 0 || s.t[p].hi != 0xFFFF)) std::abort();
}

std::vector<ConnRule4> conn_rules4(const std::vector<SemRule>& sem) {
    std::vector<ConnRule4> v(sem.size());
    for (size_t i = 0; i < sem.size(); ++i) {
        const SemRule& s = sem[i];
        check_port_free(s);
        ConnRule4& c = v[i];
        std::memset(&c, 0, sizeof c);
        if (!s.src_any) { c.src_mask = v4_mask(s.src.len); c.src_addr = v4_word(s.src.addr) & c.src_mask; }
        if (!s.dst_any) { c.dst_mask = v4_mask(s.dst.len); c.dst_addr = v4_word(s.dst.addr) & c.dst_mask; }
        c.port[0] = pack_port(s.t[P_TCP]);
        c.port[1] = pack_port(s.t[P_UDP]);
        c.meta = pack_meta(s);
        c.index = s.index;
    }
    return v;
}

// A prefix as 4 little-endian words of its 16 network-order bytes and masks
// (ConnRule16); returns the fam bit (1: IPv6 prefix).
static uint32_t conn_prefix16(const Prefix& p, uint32_t* a, uint32_t* m) {
    uint8_t ab[16] = {}, mb[16] = {};
    int off = 0, len = p.len;
    if (p.fam == 4) {                        // ::ffff:a.b.c.d/(96 + len)
        ab[10] = ab[11] = 0xFF;
        std::memcpy(ab + 12, p.addr, 4);
        off = 12;
        std::memset(mb, 0xFF, 12);
    } else {
        std::memcpy(ab, p.addr, 16);
    }
    for (int b = off; b < 16; ++b) {
        const int ones = len - 8 * (b - off);
        mb[b] = ones >= 8 ? 0xFF : ones <= 0 ? 0 : uint8_t(0xFF << (8 - ones));
    }
    for (int w = 0; w < 4; ++w) {
        uint32_t x = 0, y = 0;
        for (int j = 3; j >= 0; --j) {
            x = (x << 8) | ab[4 * w + j];
            y = (y << 8) | mb[4 * w + j];
        }
        m[w] = y;
        a[w] = x & y;
    }
    return p.fam == 16 ? 1u : 0u;
}

std::vector<ConnRule16> conn_rules16(const std::vector<SemRule>& sem) {
    std::vector<ConnRule16> v(sem.size());
    for (size_t i = 0; i < sem.size(); ++i) {
        const SemRule& s = sem[i];
        check_port_free(s);
        ConnRule16& c = v[i];
        std::memset(&c, 0, sizeof c);
        uint32_t fam = 0;
        if (!s.src_any) fam |= conn_prefix16(s.src, c.src, c.smask);
        if (!s.dst_any) fam |= conn_prefix16(s.dst, c.dst, c.dmask) << 1;
        c.port[0] = pack_port(s.t[P_TCP]);
        c.port[1] = pack_port(s.t[P_UDP]);
        c.meta = pack_meta(s);
        c.index_fam = (s.index << 2) | fam;
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


// Two-table cuckoo hash of (key, class): table 0 at [0, cap), table 1 at
// [cap, 2 cap); entry = key | class << 32.
bool cuckoo_build(const std::vector<std::pair<uint32_t, uint32_t>>& keys, uint32_t cap, uint32_t mul,
                  std::vector<uint64_t>& tab) {
    const uint32_t L = uint32_t(__builtin_ctz(cap));
    std::vector<uint8_t> used(size_t(cap) * 2, 0);
    tab.assign(size_t(cap) * 2, 0ull);
    for (const auto& kv : keys) {
        uint64_t cur = uint64_t(kv.first) | (uint64_t(kv.second) << 32);
        bool cur_valid = true;
        int side = 0;
        for (int kick = 0; kick < 256 && cur_valid; ++kick) {
            const uint32_t k = uint32_t(cur);
            const size_t pos = side == 0 ? lpm_h0(k, mul, L) : size_t(cap) + lpm_h1(k, mul, L);
            std::swap(cur, tab[pos]);
            const bool was_used = used[pos];
            used[pos] = 1;
            cur_valid = was_used;
            side ^= 1;
        }
        if (cur_valid) return false;
    }
    // Empty slots hold a key that never probes them, so the kernel's hit test
    // is a plain key compare (no "occupied" bit, no branch).
    for (size_t pos = 0; pos < tab.size(); ++pos) {
        if (used[pos]) continue;
        const bool t1 = pos >= cap;
        const uint32_t slot = uint32_t(t1 ? pos - cap : pos);
        uint32_t k = 0;
        while ((t1 ? lpm_h1(k, mul, L) : lpm_h0(k, mul, L)) == slot) ++k;
        tab[pos] = k;
    }
    return true;
}

// odd multipliers tried in order by the hash-LPM builder
constexpr uint32_t kHashMuls[] = {0x9E3779B1u, 0x85EBCA77u, 0xC2B2AE3Du, 0x27D4EB2Fu, 0x165667B1u,
                                  0xD3A2646Du, 0xFD7046C5u, 0xB55A4F09u};

// Bit-vector arrays of one candidate list (k <= 32 entries), appended to `out`:
//   dst array:  2^S x {interval start, mask of entries whose dst prefix covers it}
//   port array: 2^S x {interval start, mask of entries whose port range covers it}
// S is the table-wide search depth, so every lane runs the same steps; the
// arrays are padded with {0xFFFFFFFF, last mask} and never need a bound check.
struct BvDesc {
    uint32_t off_rel;          // byte offset of the dst array inside the BV section
    uint64_t res;              // 2-bit result of entry j at bits 2j
};

void bv_bounds(const std::vector<TmplKey>& ents, std::vector<uint32_t>& db, std::vector<uint32_t>& pb) {
    std::vector<uint64_t> d{0};
    std::vector<uint32_t> p{0};
    for (const TmplKey& t : ents) {
        if (t.m) {
            const uint64_t hi = uint64_t(t.a | ~t.m);
            d.push_back(t.a);
            if (hi < 0xFFFFFFFFull) d.push_back(hi + 1);
        }
        const uint32_t lo = t.pw & 0xFFFFu, phi = lo + (t.pw >> 16);
        p.push_back(lo);
        if (phi < 0xFFFFu) p.push_back(phi + 1);
    }
    std::sort(d.begin(), d.end());
    d.erase(std::unique(d.begin(), d.end()), d.end());
    std::sort(p.begin(), p.end());
    p.erase(std::unique(p.begin(), p.end()), p.end());
    db.assign(d.begin(), d.end());
    pb = p;
}

BvDesc build_bv(const std::vector<TmplKey>& ents, uint32_t S, std::vector<uint32_t>& out) {
    const size_t k = ents.size();
    std::vector<uint32_t> db, pb;
    bv_bounds(ents, db, pb);
    uint64_t res = 0;
    for (size_t j = 0; j < k; ++j) res |= uint64_t(ents[j].res & 3u) << (2 * j);
    const BvDesc desc{uint32_t(out.size()) * 4, res};
    const size_t n = size_t(1) << S;
    uint32_t last = 0;
    // Entry 0's bound is always 0 and the search never reads it (probes start
    // at index >= 1): it carries the list's result bits instead (dst array:
    // low word, port array: high word).
    for (size_t i = 0; i < n; ++i) {
        if (i < db.size()) {
            const uint32_t x = db[i];
            uint32_t m = 0;
            for (size_t j = 0; j < k; ++j)
                if (((x ^ ents[j].a) & ents[j].m) == 0) m |= 1u << j;
            last = m;
            out.push_back(i == 0 ? uint32_t(res) : x);
        } else {
            out.push_back(0xFFFFFFFFu);
        }
        out.push_back(last);
    }
    for (size_t i = 0; i < n; ++i) {
        if (i < pb.size()) {
            const uint32_t x = pb[i];
            uint32_t m = 0;
            for (size_t j = 0; j < k; ++j) {
                const uint32_t lo = ents[j].pw & 0xFFFFu, hi = lo + (ents[j].pw >> 16);
                if (x >= lo && x <= hi) m |= 1u << j;
            }
            last = m;
            out.push_back(i == 0 ? uint32_t(res >> 32) : x);
        } else {
            out.push_back(0xFFFFFFFFu);
        }
        out.push_back(last);
    }
    // Blocks are 2^(S+4) bytes: without a stagger, probe i of every list would
    // sit on the same LDS bank pair and the lanes of a wave (different lists,
    // same step) would conflict 32-way.  One extra uint2 rotates the banks.
    out.push_back(0u);
    out.push_back(0u);
    return desc;
}

// Global port classes (list mode 2): the elementary intervals of the port
// ranges of every bit-vector list, G = sorted interval starts (G[0] = 0).
std::vector<uint32_t> port_classes(const std::vector<std::vector<TmplKey>>& lists) {
    std::vector<uint32_t> g{0};
    for (const auto& ents : lists)
        for (const TmplKey& t : ents) {
            const uint32_t lo = t.pw & 0xFFFFu, hi = lo + (t.pw >> 16);
            g.push_back(lo);
            if (hi < 0xFFFFu) g.push_back(hi + 1);
        }
    std::sort(g.begin(), g.end());
    g.erase(std::unique(g.begin(), g.end()), g.end());
    return g;
}

// Block of one list in mode 2, appended to `out` (8-B aligned):
//   dst array: 2^Sd x {interval start, mask} as in mode 1 (entry 0 = {result
//              bits lo, mask of interval 0}),
//   result bits hi (u32), then one mask per global port class (u32 x P),
//   padded so the block is an odd number of 8-B units: lanes probing the same
//   step of different lists then spread over all LDS bank pairs.
BvDesc build_bv2(const std::vector<TmplKey>& ents, uint32_t Sd, const std::vector<uint32_t>& G,
                 std::vector<uint32_t>& out) {
    const size_t k = ents.size();
    std::vector<uint32_t> db, pb;
    bv_bounds(ents, db, pb);
    uint64_t res = 0;
    for (size_t j = 0; j < k; ++j) res |= uint64_t(ents[j].res & 3u) << (2 * j);
    const size_t start = out.size();
    const BvDesc desc{uint32_t(start) * 4, res};
    uint32_t last = 0;
    for (size_t i = 0; i < (size_t(1) << Sd); ++i) {
        if (i < db.size()) {
            const uint32_t x = db[i];
            uint32_t m = 0;
            for (size_t j = 0; j < k; ++j)
                if (((x ^ ents[j].a) & ents[j].m) == 0) m |= 1u << j;
            last = m;
            out.push_back(i == 0 ? uint32_t(res) : x);
        } else {
            out.push_back(0xFFFFFFFFu);
        }
        out.push_back(last);
    }
    out.push_back(uint32_t(res >> 32));
    for (uint32_t x : G) {
        uint32_t m = 0;
        for (size_t j = 0; j < k; ++j) {
            const uint32_t lo = ents[j].pw & 0xFFFFu, hi = lo + (ents[j].pw >> 16);
            if (x >= lo && x <= hi) m |= 1u << j;
        }
        out.push_back(m);
    }
    if ((out.size() - start) % 2) out.push_back(0u);
    if (((out.size() - start) / 2) % 2 == 0) { out.push_back(0u); out.push_back(0u); }
    return desc;
}

// Port -> class radix (list modes 2, 3): per 256-port chunk h, the byte offset
// of a 256-byte window holding class x `scale` for each port of the chunk.
// Chunks inside one class point into any run of 256 equal bytes (shared).
void port_radix(const std::vector<uint32_t>& G, const std::vector<uint32_t>& cmap,
                std::vector<uint32_t>& toff, std::vector<uint8_t>& subs, uint32_t scale) {
    toff.assign(256, 0);
    subs.clear();
    auto cls_of = [&](uint32_t p) {   // cmap: global class -> stored class
        return cmap[uint32_t(std::upper_bound(G.begin(), G.end(), p) - G.begin()) - 1u];
    };
    std::vector<int> uni(256, -1);
    for (uint32_t h = 0; h < 256; ++h) {
        // merged classes are not intervals: uniform means every port of the chunk
        const uint32_t c0 = cls_of(h << 8);
        bool uniform = true;
        for (uint32_t x = 1; x < 256 && uniform; ++x) uniform = cls_of((h << 8) | x) == c0;
        if (!uniform) {
            toff[h] = uint32_t(subs.size());
            for (uint32_t x = 0; x < 256; ++x) subs.push_back(uint8_t(cls_of((h << 8) | x) * scale));
        } else {
            uni[h] = int(c0 * scale);
        }
    }
    for (uint32_t h = 0; h < 256; ++h) {
        if (uni[h] < 0) continue;
        const uint8_t v = uint8_t(uni[h]);
        size_t at = SIZE_MAX, run = 0;
        for (size_t i = 0; i < subs.size(); ++i) {
            run = subs[i] == v ? run + 1 : 0;
            if (run == 256) { at = i + 1 - 256; break; }
        }
        if (at == SIZE_MAX) {                      // extend the tail run to 256
            size_t tail = 0;
            while (tail < subs.size() && subs[subs.size() - 1 - tail] == v) ++tail;
            at = subs.size() - tail;
            subs.resize(at + 256, v);
        }
        toff[h] = uint32_t(at);
    }
}

// List mode 3: port-filtered sublists.  For a list and a global port class,
// the entries whose port range covers the class decide first-match by the dst
// address alone: the elementary dst intervals of the list each get an outcome
// o = result | (j + 1) << 2 (j = first matching entry, 0 = no entry matches:
// default DENY), adjacent intervals with equal outcomes merge.
struct Sublist {
    std::vector<uint32_t> start;   // interval starts, start[0] = 0
    std::vector<uint32_t> out;     // outcome per interval
    bool operator==(const Sublist& o) const { return start == o.start && out == o.out; }
};
struct SublistHash {
    size_t operator()(const Sublist& s) const {
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < s.start.size(); ++i) {
            h = (h ^ s.start[i]) * 1099511628211ull;
            h = (h ^ s.out[i]) * 1099511628211ull;
        }
        return size_t(h);
    }
};
std::vector<Sublist> port_sublists(const std::vector<TmplKey>& ents, const std::vector<uint32_t>& G) {
    std::vector<uint32_t> db, pb;
    bv_bounds(ents, db, pb);
    std::vector<uint64_t> dm(db.size(), 0);
    for (size_t k = 0; k < db.size(); ++k)
        for (size_t j = 0; j < ents.size(); ++j)
            if (((db[k] ^ ents[j].a) & ents[j].m) == 0) dm[k] |= 1ull << j;
    std::vector<Sublist> res(G.size());
    for (size_t p = 0; p < G.size(); ++p) {
        uint64_t pm = 0;
        for (size_t j = 0; j < ents.size(); ++j) {
            const uint32_t lo = ents[j].pw & 0xFFFFu, hi = lo + (ents[j].pw >> 16);
            if (G[p] >= lo && G[p] <= hi) pm |= 1ull << j;
        }
        Sublist& sl = res[p];
        for (size_t k = 0; k < db.size(); ++k) {
            const uint64_t m = dm[k] & pm;
            uint32_t o = 0;
            if (m) {
                const uint32_t j = uint32_t(__builtin_ctzll(m));
                o = (ents[j].res & 3u) | ((j + 1u) << 2);
            }
            if (sl.out.empty() || sl.out.back() != o) {
                sl.start.push_back(db[k]);
                sl.out.push_back(o);
            }
        }
    }
    return res;
}

// Source trie (src mode 4): the class of a source address from a 256-entry
// level over src >> 24, a 256-entry node over bits 16..23 and a short search
// in the /16 chunk's leaf, instead of a binary search over every elementary
// interval (compile.hpp Cls4Image::off_trie).  `bounds` (n sorted interval
// starts, bounds[0] = 0) and `iclass` as build_cls4_one computes them;
// `base`: the section's LDS byte address.  Entries:
//   level 1 [src >> 24]: byte address of a node;
//   node [(src >> 16) & 255]: leaf byte address << 8 | (m - 1), m <= 256;
//   leaf: m u32 {key | class << 16}: entry 0 = the interval holding the
//   chunk's first address (key 0xFFFF: never taken), entries 1..m-1 the
//   intervals starting inside the chunk (key = start - 1, low 16 bits).
//   Search (branch-free lower bound, no padding): a = leaf, len = m; per
//   step: h = len >> 1, a' = a + 4 h, a = key(a') < (src & 0xFFFF) ? a' : a,
//   len -= h; ceil(log2 m) steps (more are no-ops); class = word(a) >> 16.
// Chunks inside one interval share a one-entry leaf per class, /8s inside
// one interval a node per class, equal leaves one copy.
struct Trie {
    std::vector<uint32_t> words;
    uint32_t depth = 0;            // steps of the largest leaf
};

bool build_trie(const std::vector<uint32_t>& bounds, uint32_t n, const std::vector<uint16_t>& iclass, uint32_t base,
                uint32_t max_bytes, Trie& out) {
    out = Trie();
    auto interval = [&](uint64_t x) {                 // index of the interval holding x
        return uint32_t(std::upper_bound(bounds.begin(), bounds.begin() + n, uint32_t(x)) - bounds.begin()) - 1u;
    };
    auto next_bound = [&](uint64_t x) {               // first bound above x (n if none)
        return uint32_t(std::upper_bound(bounds.begin(), bounds.begin() + n, uint32_t(x)) - bounds.begin());
    };
    std::vector<uint32_t>& w = out.words;
    w.assign(256, 0u);                                 // level 1, filled below
    std::map<uint32_t, uint32_t> uniform_leaf, uniform_node;   // class -> word index
    std::map<std::vector<uint32_t>, uint32_t> leaf_of;         // leaf content -> word index
    auto addr = [&](uint32_t word) { return base + 4u * word; };
    auto leaf_uniform = [&](uint32_t cls) {
        auto it = uniform_leaf.find(cls);
        if (it != uniform_leaf.end()) return it->second;
        const uint32_t at = uint32_t(w.size());
        w.push_back(0xFFFFu | (cls << 16));
        uniform_leaf.emplace(cls, at);
        return at;
    };
    std::vector<uint32_t> node(256), leaf;
    for (uint32_t a = 0; a < 256; ++a) {
        const uint64_t lo8 = uint64_t(a) << 24, hi8 = lo8 + (1u << 24) - 1u;
        const uint32_t k8 = interval(lo8), nb8 = next_bound(lo8);
        if (nb8 >= n || bounds[nb8] > hi8) {           // the /8 inside one interval
            const uint32_t cls = iclass[k8];
            auto it = uniform_node.find(cls);
            if (it == uniform_node.end()) {
                const uint32_t lw = leaf_uniform(cls);
                const uint32_t at = uint32_t(w.size());
                w.insert(w.end(), 256, addr(lw) << 8);
                it = uniform_node.emplace(cls, at).first;
            }
            w[a] = addr(it->second);
            continue;
        }
        for (uint32_t b = 0; b < 256; ++b) {
            const uint64_t lo = lo8 | (uint64_t(b) << 16), hi = lo + 0xFFFFu;
            const uint32_t k0 = interval(lo);
            uint32_t j = next_bound(lo);
            if (j >= n || bounds[j] > hi) {
                node[b] = addr(leaf_uniform(iclass[k0])) << 8;
                continue;
            }
            leaf.assign(1, 0xFFFFu | (uint32_t(iclass[k0]) << 16));
            for (; j < n && bounds[j] <= hi; ++j)
                leaf.push_back(((bounds[j] - uint32_t(lo) - 1u) & 0xFFFFu) | (uint32_t(iclass[j]) << 16));
            if (leaf.size() > 256) return false;
            uint32_t d = 0;
            while ((size_t(1) << d) < leaf.size()) ++d;
            out.depth = std::max(out.depth, d);
            auto it = leaf_of.find(leaf);
            if (it == leaf_of.end()) {
                it = leaf_of.emplace(leaf, uint32_t(w.size())).first;
                w.insert(w.end(), leaf.begin(), leaf.end());
            }
            node[b] = (addr(it->second) << 8) | uint32_t(leaf.size() - 1);
        }
        w[a] = addr(uint32_t(w.size()));
        w.insert(w.end(), node.begin(), node.end());
        if (w.size() * 4 > max_bytes) return false;
    }
    return w.size() * 4 <= max_bytes && uint64_t(base) + w.size() * 4 < (1ull << 24);
}

}  // namespace

constexpr uint32_t kV16TrieMin = 64;    // src_mode 2 from this many IPv4 source intervals

uint32_t Cls4Image::row_of(uint32_t addr) const {
    const size_t k = size_t(std::upper_bound(h_bounds.begin(), h_bounds.end(), addr) - h_bounds.begin()) - 1;
    return off_cells + uint32_t(h_iclass[k]) * row_bytes;
}

// LDS of one classify workgroup available to the image and its counters
// (option lds_budget: diagnostics and tests, to exercise the counter tiers
// with small tables).
uint32_t lds_budget() {
    const int b = compile_opts().lds_budget;
    if (b >= 0) return std::min<uint32_t>(kLdsBudget - kLdsReserved, uint32_t(b));
    return kLdsBudget - kLdsReserved;
}

// Counter tiers of a serialised image (compile.hpp Cls4Image): per-lane u32
// rows for the hot slots, then u32 LDS counters for every slot when they fit,
// else u16 LDS counters (overflow carried to the global slot counters), and
// with `partial` only the first n_lctr slots in LDS, the rest counted in
// global memory.  Returns whether the image is LDS-resident.
bool place_counters(Cls4Image& img, uint32_t budget, bool partial) {
    const uint32_t hot = img.n_hot * 64u * 4u;
    auto a16 = [](uint32_t x) { return (x + 15u) & ~15u; };
    const uint32_t c32 = a16(img.n_ctr * 4u), c16 = a16(img.n_ctr * 2u);
    uint32_t region = c32;
    bool ok = true;
    img.ctr16 = 0;
    img.n_lctr = img.n_ctr;
    if (uint64_t(img.img_bytes) + c32 + hot <= budget) {
    } else if (uint64_t(img.img_bytes) + c16 + hot <= budget) {
        img.ctr16 = 1;
        region = c16;
    } else if (partial && uint64_t(img.img_bytes) + hot + a16(img.n_hot * 2u) <= budget) {
        // at least the hot slots: their totals go through these slots' rows
        img.ctr16 = 1;
        img.n_lctr = std::min(img.n_ctr, ((budget - img.img_bytes - hot) / 2u) & ~7u);
        region = a16(img.n_lctr * 2u);
    } else {
        ok = false;
    }
    img.off_hot = img.img_bytes + region;
    img.lds_bytes = img.off_hot + hot;
    img.lds_ok = ok;
    return ok;
}

static bool build_cls4_one(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img,
                std::string& why, const Cls4Opts* opt) {
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
    img.h_bounds = bounds;
    img.h_iclass = iclass;

    // Hash LPM (tuple space): when the classed prefixes use few distinct lengths
    // (a rendered global table has only pod /32s), the class of an address is
    // found by one cuckoo probe pair per length instead of the binary search.
    std::vector<std::vector<uint64_t>> hash_tabs;
    {
        std::map<int, std::vector<std::pair<uint32_t, uint32_t>>> keys;  // len -> (addr, class)
        int len0_class = -1;
        for (size_t i = 0; i < pfx.size(); ++i) {
            const int c = class_of_pfx[i + 1];
            if (c < 0) continue;                     // never the longest match anywhere
            if (pfx[i].len == 0) { len0_class = c; continue; }
            keys[pfx[i].len].push_back({pfx[i].addr, uint32_t(c)});
        }
        uint32_t dflt = 0;
        if (len0_class >= 0) dflt = uint32_t(len0_class);
        else if (class_of_pfx[0] >= 0) dflt = uint32_t(class_of_pfx[0]);
        if (opt && opt->other) {
            img.mode = 0;                            // the OTHER image: interval search (Cls4Opts)
        } else if (opt && opt->ext_src) {
            img.mode = 3;                            // the caller maps addresses to rows
        } else if (keys.size() <= kMaxHashLens && !compile_opts().src_search) {
            // (option src_search: the interval search always -- tests)
            img.mode = 1;
            img.default_class = dflt;
            for (const auto& kv : keys) {
                const auto& ks = kv.second;
                uint32_t cap = 16, mul = 0;
                while (cap < ks.size()) cap *= 2;
                std::vector<uint64_t> tab;
                for (bool ok = false; !ok;) {
                    for (uint32_t m : kHashMuls)
                        if (cuckoo_build(ks, cap, m, tab)) { ok = true; mul = m; break; }
                    if (!ok) cap *= 2;
                    if (cap > (1u << 16)) { img.mode = 0; break; }
                }
                if (img.mode == 0) break;
                const uint32_t i = uint32_t(hash_tabs.size());
                img.hash_mask[i] = v4_mask(kv.first);
                img.hash_shift[i] = 32u - uint32_t(__builtin_ctz(cap));
                img.hash_mul[i] = mul;
                img.hash_cap[i] = cap;
                hash_tabs.push_back(std::move(tab));
            }
            img.n_hash = img.mode == 1 ? uint32_t(hash_tabs.size()) : 0u;
            if (img.mode == 0) hash_tabs.clear();
        }
    }
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
    // cells per class: TCP, UDP, ICMP (the main image), or OTHER alone
    const uint32_t pr0 = opt && opt->other ? uint32_t(P_OTHER) : 0u;
    const uint32_t ncell = opt && opt->other ? 1u : opt && opt->with_other ? 4u : 3u;
    img.n_cells = ncell;
    std::vector<uint32_t> cells(size_t(n_classes) * ncell * 2);
    img.ctr_rule.assign(1, n_rules);  // slot 0: default DENY
    // Hot class: the one covering most of the address space (random sources
    // land there).  Its cells take the slots right after slot 0, so the
    // kernel can tell the heavily hit slots by `slot < n_hot` and count them
    // in per-lane LDS rows instead of one contended word.
    uint32_t hot_class = 0;
    std::vector<uint32_t> class_order;
    {
        std::vector<double> span(n_classes, 0.0);
        if (opt && !opt->src_weight.empty()) {
            // the sources' own weights (Cls4Opts::src_weight), summed per interval
            const auto& w = opt->src_weight;
            std::vector<double> pre(w.size() + 1, 0.0);
            for (size_t j = 0; j < w.size(); ++j) pre[j + 1] = pre[j] + w[j].second;
            auto below = [&](uint64_t x) {            // weight of the values < x
                size_t lo = 0, hi = w.size();
                while (lo < hi) {
                    const size_t mid = (lo + hi) / 2;
                    if (uint64_t(w[mid].first) < x) lo = mid + 1; else hi = mid;
                }
                return pre[lo];
            };
            for (uint32_t k = 0; k < n_real_bounds; ++k) {
                const uint64_t hi = k + 1 < n_real_bounds ? uint64_t(bounds[k + 1]) : (1ull << 32);
                span[iclass[k]] += below(hi) - below(bounds[k]);
            }
        } else {
            for (uint32_t k = 0; k < n_real_bounds; ++k) {
                const double hi = k + 1 < n_real_bounds ? double(bounds[k + 1]) : 4294967296.0;
                span[iclass[k]] += hi - double(bounds[k]);
            }
        }
        hot_class = uint32_t(std::max_element(span.begin(), span.end()) - span.begin());
        if (opt && opt->hot_addr >= 0) {
            const uint32_t x = uint32_t(opt->hot_addr);
            hot_class = iclass[uint32_t(std::upper_bound(bounds.begin(), bounds.begin() + n_real_bounds, x) -
                                        bounds.begin()) - 1u];
        }
        // Slot order: the hot class, then the classes by address space
        // covered, widest first (ties: class order).  When the counters only
        // partly fit LDS (slots < n_lctr), the classes most packets land in
        // are the ones counted there.
        class_order.resize(n_classes);
        for (uint32_t c = 0; c < n_classes; ++c) class_order[c] = c;
        std::stable_sort(class_order.begin(), class_order.end(), [&](uint32_t a, uint32_t b) {
            if ((a == hot_class) != (b == hot_class)) return a == hot_class;
            return span[a] > span[b];
        });
    }
    std::vector<uint32_t> cand;
    for (uint32_t ci = 0; ci < n_classes; ++ci) {
        const uint32_t c = class_order[ci];
        // merge candidate rule positions: chain of covering prefixes + ANY
        cand.clear();
        for (int p = class_pfx[c]; p >= 0; p = parent[p])
            cand.insert(cand.end(), by_pfx[p].begin(), by_pfx[p].end());
        cand.insert(cand.end(), any_src.begin(), any_src.end());
        std::sort(cand.begin(), cand.end());
        for (uint32_t k = 0; k < ncell; ++k) {
            const int pr = int(pr0 + k);
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
            cells[(size_t(c) * ncell + k) * 2 + 0] = start | (uint32_t(seq.size()) << 16);
            cells[(size_t(c) * ncell + k) * 2 + 1] = ctr_base;
        }
        if (ci == 0) img.n_hot = std::min<uint32_t>(uint32_t(img.ctr_rule.size()), kMaxHot);
    }

    // the scan kernel reads list/template entries speculatively (clamped
    // index): keep both sections non-empty
    if (lists.empty()) lists.push_back(0);
    if (tmpls.empty()) tmpls.push_back(TmplKey{0, 0, 0, 0});

    // bit-vector form of every distinct candidate list (lists <= 32 entries):
    // first match = ctz(mask of entries covering the dst interval & mask of
    // entries covering the port interval)
    std::vector<uint32_t> bv;
    std::unordered_map<uint32_t, BvDesc> bv_desc;        // list (start | len << 16) -> arrays
    bool all_bv = true;
    std::vector<uint32_t> bv_lists;                       // distinct cell list keys
    for (uint32_t c = 0; c < n_classes && all_bv; ++c)
        for (uint32_t k = 0; k < ncell; ++k) {
            const uint32_t x = cells[(size_t(c) * ncell + k) * 2];
            if ((x >> 16) > 32) { all_bv = false; break; }
            bv_lists.push_back(x);
        }
    std::sort(bv_lists.begin(), bv_lists.end());
    bv_lists.erase(std::unique(bv_lists.begin(), bv_lists.end()), bv_lists.end());
    auto ents_of = [&](uint32_t x) {
        std::vector<TmplKey> ents;
        for (uint32_t j = 0; j < (x >> 16); ++j) ents.push_back(tmpls[lists[(x & 0xFFFFu) + j]]);
        return ents;
    };
    // list mode: 2 = bit vectors with global port classes, 1 = bit vectors
    // with per-list port search, 0 = template scan; the fastest mode whose
    // image fits the workgroup's LDS (and the 16-bit cell fields) is chosen
    std::vector<std::vector<TmplKey>> bv_ents;
    uint32_t Sd = 0, Sp = 0;
    std::vector<uint32_t> G, toff;
    std::vector<uint8_t> psub;
    // (modes 1, 2 keep a 16-bit counter base in the cell: cell_ok below)
    if (all_bv) {
        for (uint32_t x : bv_lists) {
            bv_ents.push_back(ents_of(x));
            std::vector<uint32_t> db, pb;
            bv_bounds(bv_ents.back(), db, pb);
            while ((size_t(1) << Sd) < db.size()) ++Sd;
            while ((size_t(1) << Sp) < pb.size()) ++Sp;
        }
        G = port_classes(bv_ents);
    }
    uint32_t lmode = 0;
    if (all_bv && Sd <= kMaxBvSteps && G.size() <= kMaxPortClasses) lmode = 2;
    else if (all_bv && std::max(Sd, Sp) <= kMaxBvSteps) lmode = 1;
    // List modes 3, 4 work on merged port classes: global classes no list tells
    // apart collapse (rendered ContivRules have single ports or "any", so every
    // port between the table's ports lands in one class).  <= 64 merged classes:
    // the port lookup yields class x 4 in a byte.
    std::vector<uint32_t> pmerge, prep;                  // class -> merged, merged -> a port
    std::vector<uint32_t> ident(G.size());
    for (size_t p = 0; p < G.size(); ++p) ident[p] = uint32_t(p);
    if (lmode == 2) {
        std::map<std::vector<uint64_t>, uint32_t> sig_id;
        for (size_t p = 0; p < G.size(); ++p) {
            std::vector<uint64_t> sig;
            sig.reserve(bv_ents.size());
            for (const auto& ents : bv_ents) {
                uint64_t m = 0;
                for (size_t j = 0; j < ents.size(); ++j) {
                    const uint32_t lo = ents[j].pw & 0xFFFFu, hi = lo + (ents[j].pw >> 16);
                    if (G[p] >= lo && G[p] <= hi) m |= 1ull << j;
                }
                sig.push_back(m);
            }
            auto it = sig_id.find(sig);
            if (it == sig_id.end()) {
                it = sig_id.emplace(std::move(sig), uint32_t(prep.size())).first;
                prep.push_back(G[p]);
            }
            pmerge.push_back(it->second);
        }
    }
    std::vector<std::vector<uint32_t>> sub_of;           // list -> sublist id per merged class
    std::vector<Sublist> subs;
    uint32_t D = 0;
    if (lmode == 2 && prep.size() <= kMaxPortClasses3) {
        std::unordered_map<Sublist, uint32_t, SublistHash> sid;
        for (const auto& ents : bv_ents) {
            std::vector<uint32_t> ids;
            for (Sublist& sl : port_sublists(ents, prep)) {
                auto it = sid.find(sl);
                if (it == sid.end()) {
                    it = sid.emplace(sl, uint32_t(subs.size())).first;
                    while ((size_t(1) << D) < sl.start.size()) ++D;
                    subs.push_back(std::move(sl));
                }
                ids.push_back(it->second);
            }
            sub_of.push_back(std::move(ids));
        }
        if (D <= kMaxBvSteps) lmode = 3;
    }
    // List mode 4 = mode 3 with the port lookup as one probe of a perfect hash
    // of the ports outside the most common merged class (<= kMaxPortHash such
    // ports: rendered tables), instead of the two-level radix.
    std::vector<uint32_t> phash;                          // entries {port | class x 4 << 16}
    uint32_t phash_mul = 0, phash_mask4 = 0, phash_dflt = 0;
    if (lmode == 3) {
        auto mcls = [&](uint32_t x) {
            return pmerge[uint32_t(std::upper_bound(G.begin(), G.end(), x) - G.begin()) - 1u];
        };
        std::vector<uint32_t> count(prep.size(), 0);
        for (uint32_t x = 0; x < 65536; ++x) ++count[mcls(x)];
        const uint32_t d = uint32_t(std::max_element(count.begin(), count.end()) - count.begin());
        std::vector<uint32_t> special;
        for (uint32_t x = 0; x < 65536 && special.size() <= kMaxPortHash; ++x)
            if (mcls(x) != d) special.push_back(x);
        if (special.size() <= kMaxPortHash) {
            // A table of <= 32 words is bank-conflict free: ds_read_b32 serves
            // each 32-lane half in one cycle when every bank holds at most one
            // word of it (MI355X LDS: bank = (a/4) mod 32), so distinct ports
            // never collide.  Dense tables (load > 1/2) take a longer search
            // for a collision-free multiplier: 18 ports in 32 slots succeed
            // with p ~ 0.3 % per multiplier.  Option phash_dense=0: at
            // least 2 slots per port (diagnostics / A/B).
            const bool dense = compile_opts().phash_dense;
            uint64_t z = 0x243F6A8885A308D3ull;           // splitmix64 stream of odd multipliers
            for (uint32_t L = 4; L <= 11 && !phash_mul; ++L) {
                const bool half = (1u << L) >= 2 * special.size();
                if (!half && !(dense && L <= 5 && (1u << L) >= special.size())) continue;
                const int max_tries = half ? 256 : 16384;
                for (int tries = 0; tries < max_tries && !phash_mul; ++tries) {
                    z += 0x9E3779B97F4A7C15ull;
                    uint64_t m = z;
                    m = (m ^ (m >> 30)) * 0xBF58476D1CE4E5B9ull;
                    m = (m ^ (m >> 27)) * 0x94D049BB133111EBull;
                    const uint32_t mul = uint32_t(m ^ (m >> 31));
                    const uint32_t mask4 = (4u << L) - 4u;
                    // slot of port x: (mulhi(x, mul) & mask4) / 4
                    auto slot = [&](uint32_t x) { return uint32_t((uint64_t(x) * mul) >> 32) & mask4; };
                    std::vector<uint8_t> used(size_t(1) << L, 0);
                    bool ok = true;
                    for (uint32_t x : special) {
                        const uint32_t h = slot(x) / 4u;
                        if (used[h]) { ok = false; break; }
                        used[h] = 1;
                    }
                    if (!ok) continue;
                    phash_mul = mul;
                    phash_mask4 = mask4;
                    phash.assign(size_t(1) << L, 0);
                    for (uint32_t hslot = 0; hslot < (1u << L); ++hslot) {
                        uint32_t y = 0;                   // a port that never probes this slot
                        while (slot(y) / 4u == hslot) ++y;
                        phash[hslot] = y;
                    }
                    for (uint32_t x : special) phash[slot(x) / 4u] = x | ((mcls(x) * 4u) << 16);
                }
            }
            if (phash_mul) {
                phash_dflt = d * 4u;
                lmode = 4;
            }
        }
    }
    // diagnostics / tests: cap the list mode (option list_mode_max)
    if (compile_opts().list_mode_max >= 0) {
        const uint32_t cap = uint32_t(compile_opts().list_mode_max);
        if (lmode > cap)
            lmode = cap >= 3 && lmode >= 3 ? 3u
                  : cap >= 2 && lmode >= 2 ? 2u : (cap >= 1 && std::max(Sd, Sp) <= kMaxBvSteps ? 1u : 0u);
    }

    // mode 3 gives every cell its own "no entry matched" slot (rule R, default
    // DENY) in front of its entry slots, so the kernel's slot is cell base +
    // (j + 1) with no select; same cell order, so the hot class stays first
    const std::vector<uint32_t> ctr_base_rule = img.ctr_rule;
    const uint32_t hot_base = img.n_hot;
    std::vector<uint32_t> ctr3(1, n_rules), cb3(size_t(n_classes) * ncell);
    uint32_t hot3 = 1;
    for (uint32_t ci = 0; ci < n_classes; ++ci) {
        const uint32_t c = class_order[ci];
        for (uint32_t kk = 0; kk < ncell; ++kk) {
            const size_t k = size_t(c) * ncell + kk;
            cb3[k] = uint32_t(ctr3.size());
            ctr3.push_back(n_rules);
            const uint32_t len = cells[2 * k] >> 16, b = cells[2 * k + 1];
            for (uint32_t j = 0; j < len; ++j) ctr3.push_back(ctr_base_rule[b + j]);
        }
        if (ci == 0) hot3 = std::min<uint32_t>(uint32_t(ctr3.size()), kMaxHot);
    }
    // wide cells (list modes 5, 6: in global memory, 32-bit counter base)
    // keep the sublist form when the LDS cells cannot
    const uint32_t lmode_w = lmode >= 3 ? lmode : 0u;
    if (lmode >= 3 && ctr3.size() > 0x3FFFFu) lmode = 2;  // 18-bit counter base in the cell
    const uint32_t mode0 = img.mode;                      // the source lookup without the trie

    std::vector<uint32_t>& w = img.words;
    // trie: the source trie replaces the interval search (mode 0 only);
    // wide: list modes 3, 4 with the cells in global memory (gcells).
    // (Two round-3 variants were measured and removed: sublists as 4-ary
    // 16-B node trees, 0.613 against 0.600 ms on config 3, and hash entries
    // carrying their class's cells inline, 0.639 against 0.613 -- a random
    // ds_read_b128 costs about two random ds_read_b64 in bank cycles.)
    const uint32_t n_hash0 = img.n_hash;
    auto serialise = [&](uint32_t lm, bool trie, bool wide) -> bool {
        img.mode = trie ? 4u : mode0;
        img.n_hash = trie ? 0u : n_hash0;                 // the trie replaces the hash LPM
        img.off_trie = img.trie_depth = 0;
        img.gcells.clear();
        img.ctr_rule = lm >= 3 ? ctr3 : ctr_base_rule;
        img.n_hot = lm >= 3 ? hot3 : hot_base;
        // lists
        bv.clear();
        bv_desc.clear();
        const uint32_t S = std::max(Sd, Sp);
        for (size_t i = 0; i < bv_lists.size(); ++i) {
            if (lm == 2) bv_desc[bv_lists[i]] = build_bv2(bv_ents[i], Sd, G, bv);
            else if (lm == 1) bv_desc[bv_lists[i]] = build_bv(bv_ents[i], S, bv);
        }
        img.list_mode = lm;
        img.bv_steps_d = lm >= 3 ? D : lm == 2 ? Sd : S;
        img.bv_steps_p = lm >= 2 ? 0u : S;
        img.n_pclass = lm >= 3 ? uint32_t(prep.size()) : lm == 2 ? uint32_t(G.size()) : 0u;
        img.bv_wide = 0;
        for (const auto& e : bv_ents) img.bv_wide |= e.size() > 16 ? 1u : 0u;
        // serialise (u32 words, each section 16 B aligned); sections the chosen
        // modes never read are left out of the LDS image
        w.clear();
        img.off_bounds = img.off_iclass = img.off_lists = img.off_tmpl = img.off_bv = img.off_ptop = 0;
        img.port_mul = img.port_mask4 = img.port_dflt = 0;
        if (lm == 4) {
            // port perfect hash at LDS address 0
            w.assign(phash.begin(), phash.end());
            w.resize(align4(uint32_t(w.size())));
            img.port_mul = phash_mul;
            img.port_mask4 = phash_mask4;
            img.port_dflt = phash_dflt;
        } else if (lm >= 2) {
            // port radix at LDS address 0 (the kernel indexes it without a base):
            // top (256 x u32 = byte address of the chunk's window), then windows
            // of classes (mode 2: global classes; mode 3: merged classes x 4)
            port_radix(G, lm == 3 ? pmerge : ident, toff, psub, lm == 3 ? 4u : 1u);
            img.off_ptop = 0;
            for (uint32_t h = 0; h < 256; ++h) w.push_back(1024u + toff[h]);
            w.resize(256 + (psub.size() + 3) / 4);
            std::memcpy(reinterpret_cast<uint8_t*>(w.data() + 256), psub.data(), psub.size());
            w.resize(align4(uint32_t(w.size())));
        }
        std::unordered_map<uint32_t, uint32_t> ptr_off;  // list key -> byte offset of its pointer table
        std::vector<uint32_t> state0;                      // sublist -> initial state, region-relative
        std::vector<uint32_t> ptr_at;                      // word index of each list's pointer table
        if (lm >= 3) {
            // pointer tables next: their byte offsets live in the cell's low 16 bits
            for (size_t i = 0; i < bv_lists.size(); ++i) {
                ptr_off[bv_lists[i]] = uint32_t(w.size()) * 4;
                ptr_at.push_back(uint32_t(w.size()));
                w.resize(w.size() + prep.size(), 0u);        // filled once the region is placed
            }
            w.resize(align4(uint32_t(w.size())));
            img.sub_bytes = uint32_t(w.size()) * 4;
        }
        if (trie) {
            Trie tr;
            if (!build_trie(bounds, n_real_bounds, iclass, uint32_t(w.size()) * 4, lds_budget(), tr)) {
                if (compile_opts().debug_modes)
                    std::fprintf(stderr, "trie: does not fit (%zu words at depth %u)\n", tr.words.size(), tr.depth);
                return false;
            }
            img.off_trie = uint32_t(w.size()) * 4;
            img.trie_depth = tr.depth;
            w.insert(w.end(), tr.words.begin(), tr.words.end());
            w.resize(align4(uint32_t(w.size())));
        } else if (img.mode == 0) {
            img.off_bounds = uint32_t(w.size()) * 4;
            w.insert(w.end(), bounds.begin(), bounds.end());
            w.resize(align4(uint32_t(w.size())));
            img.off_iclass = uint32_t(w.size()) * 4;
            w.resize(w.size() + (bounds.size() + 1) / 2);
            std::memcpy(reinterpret_cast<uint8_t*>(w.data()) + img.off_iclass, iclass.data(), iclass.size() * 2);
            w.resize(align4(uint32_t(w.size())));
        }
        img.off_cells = wide ? 0u : uint32_t(w.size()) * 4;
        img.row_bytes = lm == 0 || wide ? 8u * ncell : 4u * ncell;   // cells of uint2 (scan, wide) / u32
        img.default_row = img.off_cells + img.default_class * img.row_bytes;
        if (lm == 0) {
            // scan cells: uint2 {list start | len << 16, counter base}
            w.insert(w.end(), cells.begin(), cells.end());
            w.resize(align4(uint32_t(w.size())));
            img.off_lists = uint32_t(w.size()) * 4;
            const size_t lbase = w.size();
            w.resize(lbase + (lists.size() + 1) / 2);
            std::memcpy(reinterpret_cast<uint8_t*>(w.data() + lbase), lists.data(), lists.size() * 2);
            w.resize(align4(uint32_t(w.size())));
            img.off_tmpl = uint32_t(w.size()) * 4;
            for (const auto& t : tmpls) {
                w.push_back(t.a);
                w.push_back(t.m);
                w.push_back(t.pw);
                w.push_back(t.res);
            }
            w.resize(align4(uint32_t(w.size())));
        } else if (wide) {
            // wide cells, in global memory: uint2 {pointer table byte
            // address, counter base (the cell's own no-match slot)}
            const size_t n_cells = size_t(n_classes) * ncell;
            img.gcells.resize(2 * n_cells);
            for (size_t i = 0; i < n_cells; ++i) {
                img.gcells[2 * i] = ptr_off.at(cells[2 * i]);
                img.gcells[2 * i + 1] = cb3[i];
            }
        } else if (lm >= 3) {
            // sublist cells: u32 {pointer table word offset (14 bits: the
            // tables lie in the first 64 KiB) | counter base << 14}, the base
            // being the cell's own no-match slot
            const size_t n_cells = size_t(n_classes) * ncell;
            for (size_t i = 0; i < n_cells; ++i) w.push_back((ptr_off.at(cells[2 * i]) >> 2) | (cb3[i] << 14));
            w.resize(align4(uint32_t(w.size())));
        } else {
            // bit-vector cells: u32 {list block offset / 8 | counter base << 16}
            const size_t n_cells = size_t(n_classes) * ncell;
            const uint32_t off_bv = uint32_t(align4(uint32_t(w.size() + n_cells))) * 4;
            img.off_bv = off_bv;
            for (size_t i = 0; i < n_cells; ++i) {
                const BvDesc& d = bv_desc.at(cells[2 * i]);
                const uint32_t off = off_bv + d.off_rel;
                w.push_back((off / 8) | (cells[2 * i + 1] << 16));
            }
            w.resize(align4(uint32_t(w.size())));
            w.insert(w.end(), bv.begin(), bv.end());
            w.resize(align4(uint32_t(w.size())));
        }
        for (uint32_t i = 0; i < img.n_hash; ++i) {
            w.resize(align4(uint32_t(w.size())));
            img.off_hash[i] = uint32_t(w.size()) * 4;
            for (uint64_t e : hash_tabs[i]) {               // entry {key, byte address of the class's cell row}
                w.push_back(uint32_t(e));
                w.push_back(img.off_cells + uint32_t(e >> 32) * img.row_bytes);
            }
            w.resize(align4(uint32_t(w.size())));
        }
        if (lm >= 3) {
            // Sublist region, 8-B slots.  A sublist of n intervals and depth s
            // (2^s >= n) sits at slot A: entries 1 .. n-1 in slots A+1 .. A+n-1
            // as {start - 1, outcome | (A + c) << 16}; the slots a probe may
            // read beyond them -- A+n .. A+2^s-1 and A + 2^i for s <= i < D --
            // must hold a never-taken sentinel {0xFFFFFFFF, 0} (the kernel
            // tests start - 1 < dst).  Sentinel slots are shared between
            // sublists; greedy first fit, deepest first.
            const uint32_t r0 = uint32_t(w.size()) / 2u + (w.size() & 1u);   // region slot base
            std::vector<uint8_t> kind;                    // 0 free, 1 entry, 2 sentinel
            std::vector<uint32_t> A(subs.size());
            std::vector<size_t> order(subs.size());
            for (size_t k = 0; k < order.size(); ++k) order[k] = k;
            std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
                return subs[a].start.size() > subs[b].start.size();
            });
            std::vector<uint32_t> need_e, need_s;
            uint32_t hint1 = 0;                           // first fit for single-interval sublists
            for (size_t k : order) {
                const uint32_t n = uint32_t(subs[k].start.size());
                uint32_t sd = 0;
                while ((1u << sd) < n) ++sd;
                need_e.clear();
                need_s.clear();
                for (uint32_t c = 1; c < n; ++c) need_e.push_back(c);
                for (uint32_t c = n; c < (1u << sd); ++c) need_s.push_back(c);
                for (uint32_t i2 = std::max(sd, n > 1 ? sd : 0u); i2 < D; ++i2) need_s.push_back(1u << i2);
                uint32_t a = n == 1 ? hint1 : 0u;
                for (;; ++a) {
                    bool ok = true;
                    for (uint32_t c : need_e) {
                        if (a + c < kind.size() && kind[a + c] != 0) { ok = false; break; }
                    }
                    if (ok)
                        for (uint32_t c : need_s) {
                            if (a + c < kind.size() && kind[a + c] == 1) { ok = false; break; }
                        }
                    if (ok) break;
                }
                if (n == 1) hint1 = a;
                const uint32_t top_slot = a + std::max<uint32_t>(1u << std::max(sd, D > 0 ? D - 1 : 0u), n) + 1;
                if (kind.size() < top_slot) kind.resize(top_slot, 0);
                for (uint32_t c : need_e) kind[a + c] = 1;
                for (uint32_t c : need_s) kind[a + c] = 2;
                A[k] = a;
            }
            if (kind.empty()) kind.resize(1, 0);
            w.resize(size_t(r0) * 2, 0u);
            const size_t reg = w.size();
            w.resize(reg + kind.size() * 2);
            for (size_t sl = 0; sl < kind.size(); ++sl) {
                w[reg + 2 * sl] = 0xFFFFFFFFu;
                w[reg + 2 * sl + 1] = 0u;
            }
            state0.resize(subs.size());
            for (size_t k = 0; k < subs.size(); ++k) {
                const uint32_t base_slot = r0 + A[k];
                for (uint32_t c = 1; c < subs[k].start.size(); ++c) {
                    w[reg + 2 * (A[k] + c)] = subs[k].start[c] - 1u;
                    w[reg + 2 * (A[k] + c) + 1] = subs[k].out[c] | ((base_slot + c) << 16);
                }
                state0[k] = subs[k].out[0] | (base_slot << 16);
            }
            img.off_bv = uint32_t(reg) * 4;
            if (r0 + kind.size() > 0x10000u) img.sub_bytes = 0xFFFFFFFFu;   // 16-bit slot field
            for (size_t i = 0; i < bv_lists.size(); ++i)
                for (size_t p = 0; p < prep.size(); ++p) w[ptr_at[i] + p] = state0[sub_of[i][p]];
            w.resize(align4(uint32_t(w.size())));
        }
        img.off_tail = uint32_t(w.size()) * 4;
        if (opt) {
            w.insert(w.end(), opt->tail.begin(), opt->tail.end());
            w.resize(align4(uint32_t(w.size())));
        }
        img.img_bytes = uint32_t(w.size()) * 4;
        img.n_bounds = n_real_bounds;
        img.n_classes = n_classes;
        img.n_tmpl = uint32_t(tmpls.size());
        img.n_list_entries = uint32_t(lists.size());
        img.n_ctr = uint32_t(img.ctr_rule.size());
        img.search_top = top;
        if (wide) img.list_mode = lm == 4 ? 5u : 6u;
        return true;
    };
    // The fastest list mode whose image and counters fit the workgroup's LDS:
    // first with every slot counted in LDS (u32, else u16), then with the
    // image resident and the coldest slots counted in global memory (Cls4Image
    // counter tiers).  With neither, the image stays in global memory (list
    // mode 1 when possible: its cells need no list scan).
    const bool dbg = compile_opts().debug_modes;   // diagnostics
    const uint32_t budget = lds_budget();
    std::vector<uint32_t> seq;
    for (uint32_t lm = lmode;;) {
        seq.push_back(lm);
        if (lm == 0) break;
        lm = lm >= 3 ? 2u : (lm == 2 && std::max(Sd, Sp) <= kMaxBvSteps) ? 1u : 0u;
    }
    if (opt && opt->other) seq.assign(1, 0u);     // the OTHER image: template scan (Cls4Opts)
    // diagnostics / tests: exactly this list mode when it is available
    // (option list_mode), so a test's LDS budget picks the counter tier
    else if (compile_opts().list_mode >= 0) {
        const uint32_t lm = uint32_t(compile_opts().list_mode);
        if (std::find(seq.begin(), seq.end(), lm) != seq.end()) seq.assign(1, lm);
    }
    // block offset field: 16 bits in 8-B units (modes 1, 2); mode 3: the
    // pointer tables in the first 64 KiB, sublist slots below 2^16
    auto cell_ok = [&](uint32_t lm) {
        if (img.list_mode >= 5) return img.sub_bytes != 0xFFFFFFFFu;   // wide cells: the state's slot field
        return lm == 0 || (lm >= 3 ? img.sub_bytes <= 0x10000u
                                   : img.img_bytes / 8u <= 0xFFFFu && img.ctr_rule.size() <= 0xFFFFu);
    };
    // The source trie where the interval search would run (sublist modes;
    // option trie=0 / 1: never / only -- diagnostics and tests), preferred
    // when it fits; wide cells only once no LDS-cell image fits
    // (option wide=1: first -- tests).
    const int tmode = compile_opts().trie;
    const bool wide_first = compile_opts().wide == 1, wide_never = compile_opts().wide == 0;
    // (the 16-byte core searching reps takes them too; not the OTHER image).
    // Behind a hash LPM the trie is the second choice (two probes beat it
    // when the hash tables fit; large ones -- many prefixes of few lengths,
    // e.g. reps -- do not).
    const bool trie_ok = (mode0 == 0 || mode0 == 1) && !(opt && (opt->other || opt->ext_src)) && tmode != 0;
    auto try_fit = [&](uint32_t lm, bool wide, bool partial) {
        int cand[2] = {0, -1};
        if (trie_ok && lm >= 3) {
            if (tmode == 1) cand[0] = 1;
            else if (mode0 == 0) cand[0] = 1, cand[1] = 0;
            else cand[1] = 1;
        }
        // dependent LDS reads per packet: interval search log2(top) + 1 steps
        // and the class read; trie level 1, node, its leaf steps, final read
        uint32_t isearch = 2;
        for (uint32_t s = top; s > 1; s >>= 1) ++isearch;
        for (int tr : cand) {
            if (tr < 0) continue;
            if (!serialise(lm, tr != 0, wide)) continue;
            // a small interval table searches in no more dependent reads than
            // the trie walks, in a fraction of its LDS (the trie's first level
            // alone is 1 KiB): take the interval search
            if (tr && tmode != 1 && cand[1] == 0 && 3u + img.trie_depth >= isearch) continue;
            const bool ok = cell_ok(lm) && place_counters(img, budget, partial);
            if (dbg)
                std::fprintf(stderr, "list mode %u%s%s%s: lds %u img %u ctr %u lctr %u ctr16 %u -> %s\n", img.list_mode,
                             tr ? " trie" : "", wide ? " wide" : "", partial ? " (partial)" : "", img.lds_bytes,
                             img.img_bytes, img.n_ctr, img.n_lctr, img.ctr16, ok ? "resident" : "no");
            if (ok) return true;
        }
        return false;
    };
    const bool wide_ok = lmode_w >= 3 && !(opt && opt->other) && !wide_never;
    if (wide_ok && wide_first && try_fit(lmode_w, true, true)) return true;
    for (int partial = 0; partial < 2; ++partial)
        for (uint32_t lm : seq)
            if (try_fit(lm, false, partial != 0)) return true;
    if (wide_ok && try_fit(lmode_w, true, true)) return true;
    for (uint32_t lm : seq) {
        if (lm > 1 && lm != seq.back()) continue;
        serialise(lm, false, false);
        if (!cell_ok(lm)) continue;
        place_counters(img, budget, false);
        if (dbg) std::fprintf(stderr, "list mode %u: global image\n", lm);
        return true;
    }
    return true;
}

}  // namespace cls

// ---------------------------------------------------------------------------
// 16-byte classifier image (compile.hpp: representatives)
// ---------------------------------------------------------------------------
namespace cls {
namespace {

using u128 = unsigned __int128;
constexpr u128 kAll = ~u128(0);
constexpr u128 kV4Lo = u128(0xFFFFu) << 32;          // ::ffff:0.0.0.0, To4()-able addresses
constexpr u128 kV4Hi = kV4Lo | 0xFFFFFFFFu;

struct Range {
    u128 lo, hi;
    bool operator<(const Range& o) const { return lo != o.lo ? lo < o.lo : hi > o.hi; }  // containers first
    bool operator==(const Range& o) const { return lo == o.lo && hi == o.hi; }
};

Range range_of(const Prefix& p) {
    if (p.fam == 4) {
        const uint32_t m = v4_mask(p.len);
        const u128 lo = kV4Lo | (v4_word(p.addr) & m);
        return {lo, lo | u128(~m)};
    }
    u128 a = 0;
    for (int i = 0; i < 16; ++i) a = (a << 8) | p.addr[i];
    const u128 host = p.len >= 128 ? u128(0) : (kAll >> p.len);
    return {a & ~host, (a & ~host) | host};
}

// One address side (src or dst): the prefix tree of each family, its blocks
// in rep space, and the front-end interval table.
struct Side {
    std::vector<Range> pf[2];          // 0 = IPv4, 1 = IPv6; sorted, distinct
    std::vector<uint32_t> base[2];
    std::vector<int> blen[2];
    uint32_t root[2] = {0u, 0x80000000u};

    int fam_of(const Prefix& p) const { return p.fam == 4 ? 0 : 1; }
    size_t find(int f, const Range& r) const {
        return size_t(std::lower_bound(pf[f].begin(), pf[f].end(), r) - pf[f].begin());
    }
    bool embed(std::string& why) {
        for (int f = 0; f < 2; ++f) {
            auto& P = pf[f];
            std::sort(P.begin(), P.end());
            P.erase(std::unique(P.begin(), P.end()), P.end());
            std::vector<std::vector<uint32_t>> kids(P.size() + 1);   // last = family root
            std::vector<uint32_t> stack;
            for (uint32_t i = 0; i < P.size(); ++i) {
                while (!stack.empty() && P[stack.back()].hi < P[i].lo) stack.pop_back();
                kids[stack.empty() ? P.size() : stack.back()].push_back(i);
                stack.push_back(i);
            }
            base[f].assign(P.size(), 0);
            blen[f].assign(P.size(), 0);
            auto assign = [&](const std::vector<uint32_t>& ks, uint32_t b, int l) {
                if (ks.empty()) return true;
                int bits = 0;
                while ((size_t(1) << bits) < ks.size() + 1) ++bits;
                if (l + bits > 32) return false;
                for (size_t j = 0; j < ks.size(); ++j) {
                    base[f][ks[j]] = b | uint32_t(uint64_t(j + 1) << (32 - l - bits));
                    blen[f][ks[j]] = l + bits;
                }
                return true;
            };
            bool ok = assign(kids[P.size()], root[f], 1);
            for (uint32_t i = 0; ok && i < P.size(); ++i) ok = assign(kids[i], base[f][i], blen[f][i]);
            if (!ok) {
                why = "prefix tree too deep for 32-bit representatives";
                return false;
            }
        }
        return true;
    }
    // interval table: starts (ascending, [0] = 0) and the rep of each interval
    void intervals(std::vector<u128>& start, std::vector<uint32_t>& rep) const {
        std::vector<u128> b{0, kV4Lo, kV4Hi + 1};
        for (int f = 0; f < 2; ++f)
            for (const auto& r : pf[f]) {
                b.push_back(r.lo);
                if (r.hi != kAll) b.push_back(r.hi + 1);
            }
        std::sort(b.begin(), b.end());
        b.erase(std::unique(b.begin(), b.end()), b.end());
        std::vector<int> lpm[2];
        for (int f = 0; f < 2; ++f) {
            lpm[f].assign(b.size(), -1);
            std::vector<int> stack;
            size_t next = 0;
            for (size_t k = 0; k < b.size(); ++k) {
                while (!stack.empty() && pf[f][stack.back()].hi < b[k]) stack.pop_back();
                while (next < pf[f].size() && pf[f][next].lo == b[k]) stack.push_back(int(next++));
                lpm[f][k] = stack.empty() ? -1 : stack.back();
            }
        }
        start.clear();
        rep.clear();
        for (size_t k = 0; k < b.size(); ++k) {
            const int f = (b[k] >= kV4Lo && b[k] <= kV4Hi) ? 0 : 1;
            const uint32_t r = lpm[f][k] < 0 ? root[f] : base[f][lpm[f][k]];
            if (!rep.empty() && rep.back() == r) continue;
            start.push_back(b[k]);
            rep.push_back(r);
        }
    }
};

void put_be32(uint8_t* a, uint32_t v) {
    a[0] = uint8_t(v >> 24); a[1] = uint8_t(v >> 16); a[2] = uint8_t(v >> 8); a[3] = uint8_t(v);
}

// 8-byte search keys (compile.hpp key8): exact for interval starts with hi64 0
// and lo64 <= 2^48 (the v4-mapped block and below), or lo64 0 (IPv6 prefixes
// up to /64)
constexpr uint64_t kK8Lo = 1ull << 48, kK8HiMax = ~0ull - kK8Lo;
bool has_key8(u128 b) {
    const uint64_t h = uint64_t(b >> 64), l = uint64_t(b);
    return h == 0 ? l <= kK8Lo : (l == 0 && h <= kK8HiMax);
}
uint64_t key8(u128 x) {
    const uint64_t h = uint64_t(x >> 64), l = uint64_t(x);
    return h == 0 ? std::min(l, kK8Lo) : kK8Lo + std::min(h, kK8HiMax);
}

// an address's 16 network-order bytes as the kernel loads them (4 little-endian words)
std::array<uint32_t, 4> raw_words(u128 a) {
    std::array<uint32_t, 4> w{};
    for (int i = 0; i < 16; ++i) w[i / 4] |= uint32_t(uint8_t(a >> (120 - 8 * i))) << (8 * (i % 4));
    return w;
}

// Two-table cuckoo hash of 16-byte keys (Cls16Image, IPv6 host routes):
// slot_key[s] = key index in slot s, or -1; empty slots are then given keys
// that never probe them (fill6).
uint32_t h6_slot(const std::array<uint32_t, 4>& k, uint32_t cap, uint32_t mul, const uint32_t* f, int side) {
    const uint32_t L = uint32_t(__builtin_ctz(cap));
    const uint32_t h = fold6(k[0], k[1], k[2], k[3], f) * mul;
    return side == 0 ? h >> (32u - L) : cap + ((h >> (32u - 2u * L)) & (cap - 1u));
}

bool cuckoo6(const std::vector<std::array<uint32_t, 4>>& keys, uint32_t cap, uint32_t mul, const uint32_t* f,
             std::vector<int>& slot_key) {
    slot_key.assign(size_t(cap) * 2, -1);
    for (int i = 0; i < int(keys.size()); ++i) {
        int cur = i, side = 0;
        for (int kick = 0; kick < 256 && cur >= 0; ++kick) {
            const uint32_t pos = h6_slot(keys[size_t(cur)], cap, mul, f, side);
            std::swap(cur, slot_key[pos]);
            side ^= 1;
        }
        if (cur >= 0) return false;
    }
    return true;
}

}  // namespace

static bool build_cls16_one(const std::vector<SemRule>& sem, uint32_t n_rules, Cls16Image& img, std::string& why) {
    img = Cls16Image();
    Side side[2];                                         // 0 src, 1 dst
    for (const SemRule& s : sem) {
        if (!s.src_any) side[0].pf[side[0].fam_of(s.src)].push_back(range_of(s.src));
        if (!s.dst_any) side[1].pf[side[1].fam_of(s.dst)].push_back(range_of(s.dst));
    }
    for (auto& sd : side)
        if (!sd.embed(why)) return false;
    // rules in rep space
    img.sem.clear();
    for (const SemRule& s : sem) {
        SemRule r = s;
        for (int sd = 0; sd < 2; ++sd) {
            const bool any = sd == 0 ? r.src_any : r.dst_any;
            if (any) continue;
            Prefix& p = sd == 0 ? r.src : r.dst;
            const int f = side[sd].fam_of(p);
            const size_t id = side[sd].find(f, range_of(p));
            Prefix q;
            q.fam = 4;
            put_be32(q.addr, side[sd].base[f][id]);
            q.len = side[sd].blen[f][id];
            p = q;
        }
        img.sem.push_back(r);
    }
    // Source front end: host-route hashes when every source prefix is a host
    // route (option v16_src_search=1 forces the interval search, src_mode
    // 0: tests)
    bool hosts = true;
    for (int f = 0; f < 2; ++f)
        for (const auto& r : side[0].pf[f]) hosts = hosts && r.lo == r.hi;
    if (compile_opts().v16_src_search >= 0) hosts = hosts && compile_opts().v16_src_search == 0;
    img.src_mode = hosts ? 1u : 0u;

    // interval tables: per side, keys (start - 1 as u64 hi, lo; padding all
    // ones) then reps
    auto search_list = [&](const std::vector<u128>& start, const std::vector<uint32_t>& rep, std::vector<uint32_t>& out,
                           uint32_t& top, uint32_t& nval, uint32_t& rel_val, uint32_t& k8) {
        uint32_t K = 1;
        while (K < start.size()) K *= 2;
        top = K;
        nval = uint32_t(rep.size());
        // 8-B keys (key8, compile.hpp) when every interval start has a key8
        k8 = 1;
        for (size_t k = 1; k < start.size(); ++k) k8 &= has_key8(start[k]) ? 1u : 0u;
        for (uint32_t k = 0; k < K; ++k) {
            if (k8) {
                const uint64_t key = (k >= 1 && k < start.size()) ? key8(start[k]) - 1 : ~0ull;
                out.push_back(uint32_t(key));
                out.push_back(uint32_t(key >> 32));
                continue;
            }
            const u128 key = (k >= 1 && k < start.size()) ? start[k] - 1 : kAll;
            const uint64_t h = uint64_t(key >> 64), l = uint64_t(key);
            out.push_back(uint32_t(h));
            out.push_back(uint32_t(h >> 32));
            out.push_back(uint32_t(l));
            out.push_back(uint32_t(l >> 32));
        }
        out.resize(align4(uint32_t(out.size())));
        rel_val = uint32_t(out.size()) * 4;
        out.insert(out.end(), rep.begin(), rep.end());
        out.resize(align4(uint32_t(out.size())));
    };
    auto search_table = [&](int sd, std::vector<uint32_t>& out, uint32_t& top, uint32_t& nval, uint32_t& rel_val,
                            uint32_t& k8) {
        std::vector<u128> start;
        std::vector<uint32_t> rep;
        side[sd].intervals(start, rep);
        search_list(start, rep, out, top, nval, rel_val, k8);
    };
    // Source front end, src_mode 2 (not every source a host route, many
    // IPv4 intervals -- e.g. the IP-block lists of gen-policy.py): IPv4-mapped
    // sources go through a trie over their IPv4 word straight to the class
    // row (the IPv4 classifier's source trie, compile.cpp build_trie, with the
    // core's classes), other sources through a search over the non-IPv4
    // intervals whose values are rows; the whole interval table stays in
    // global memory for protocols > 2 (they need the rep).
    // option v16_src_trie=0 / 1: never / whenever sources are not all host
    // routes (tests).
    std::vector<u128> s_start;
    std::vector<uint32_t> s_rep;
    side[0].intervals(s_start, s_rep);
    std::vector<uint32_t> v4b, v4rep;                      // intervals of ::ffff:0.0.0.0/96, rel. bounds
    std::vector<u128> v6start;                            // the others (the IPv4 block as one interval)
    std::vector<uint32_t> v6rep;
    {
        size_t k = size_t(std::upper_bound(s_start.begin(), s_start.end(), kV4Lo) - s_start.begin()) - 1;
        v4b.push_back(0u);
        v4rep.push_back(s_rep[k]);
        for (size_t j = k + 1; j < s_start.size() && s_start[j] <= kV4Hi; ++j) {
            v4b.push_back(uint32_t(s_start[j] - kV4Lo));
            v4rep.push_back(s_rep[j]);
        }
        for (size_t j = 0; j < s_start.size(); ++j) {
            if (s_start[j] > kV4Lo && s_start[j] <= kV4Hi) continue;
            v6start.push_back(s_start[j]);
            v6rep.push_back(s_rep[j]);
        }
    }
    bool trie = !hosts && v4b.size() >= kV16TrieMin && compile_opts().v16_src_search < 0;
    if (compile_opts().v16_src_trie >= 0) trie = !hosts && compile_opts().v16_src_trie != 0;
    if (trie) img.src_mode = 2;
    Cls4Opts opt;
    opt.ext_src = hosts || trie;
    uint32_t rel_key[2] = {}, rel_val[2] = {};
    for (int sd = opt.ext_src ? 1 : 0; sd < 2; ++sd) {
        rel_key[sd] = uint32_t(opt.tail.size()) * 4;
        search_table(sd, opt.tail, img.fe_top[sd], img.fe_n[sd], rel_val[sd], img.fe_k8[sd]);
    }
    // src_mode 2: the non-IPv4 source search (values patched to rows below)
    // and room for the trie (its size with one provisional class per distinct
    // rep -- the core's classes can only merge them, so the final trie fits)
    uint32_t rel_trie = 0, trie_words = 0;
    std::vector<uint16_t> prov;
    if (trie) {
        rel_key[0] = uint32_t(opt.tail.size()) * 4;
        search_list(v6start, v6rep, opt.tail, img.fe_top[0], img.fe_n[0], rel_val[0], img.fe_k8[0]);
        std::map<uint32_t, uint16_t> id;
        for (uint32_t r : v4rep) {
            if (id.size() >= 0xFFFFu && !id.count(r)) { why = "too many source classes for the IPv4 trie"; return false; }
            prov.push_back(id.emplace(r, uint16_t(id.size())).first->second);
        }
        Trie tr;
        if (!build_trie(v4b, uint32_t(v4b.size()), prov, 0u, 1u << 22, tr)) { why = "IPv4 source trie too large"; return false; }
        trie_words = uint32_t(tr.words.size());
        rel_trie = uint32_t(opt.tail.size()) * 4;
        opt.tail.resize(opt.tail.size() + trie_words, 0u);
        opt.tail.resize(align4(uint32_t(opt.tail.size())));
        img.src_search.clear();
        uint32_t n0;
        search_list(s_start, s_rep, img.src_search, img.src_search_top, n0, img.src_search_val, img.src_search_k8);
    }
    // host-route hashes; their values (rows) are patched in once the core is laid out
    std::vector<uint32_t> pfx4, pfx6;                     // prefix index per hashed key
    std::vector<uint64_t> tab4;
    std::vector<int> slot6;
    uint32_t rel_h4 = 0, rel_k6 = 0, rel_r6 = 0;
    if (hosts) {
        img.src_search.clear();
        uint32_t top0, n0, rv0;
        search_table(0, img.src_search, top0, n0, rv0, img.fe_k8[0]);
        img.fe_top[0] = top0;
        img.fe_n[0] = n0;
        img.src_search_val = rv0;
        img.src_search_top = top0;
        img.src_search_k8 = img.fe_k8[0];
        // IPv4-mapped: key = last 4 address bytes as a little-endian word
        std::vector<std::pair<uint32_t, uint32_t>> k4;
        for (uint32_t i = 0; i < side[0].pf[0].size(); ++i)
            k4.push_back({raw_words(side[0].pf[0][i].lo)[3], i});
        uint32_t cap = 16;
        while (cap < k4.size()) cap *= 2;
        for (bool ok = false; !ok;) {
            for (uint32_t m : kHashMuls)
                if (cuckoo_build(k4, cap, m, tab4)) { ok = true; img.mul4 = m; break; }
            if (!ok) cap *= 2;
            if (cap > (1u << 16)) { why = "IPv4 host-route hash failed"; return false; }
        }
        img.cap4 = cap;
        rel_h4 = uint32_t(opt.tail.size()) * 4;
        for (uint64_t e : tab4) {
            opt.tail.push_back(uint32_t(e));
            opt.tail.push_back(0u);
        }
        opt.tail.resize(align4(uint32_t(opt.tail.size())));
        // IPv6: full 16-byte keys
        std::vector<std::array<uint32_t, 4>> k6;
        for (const auto& r : side[0].pf[1]) k6.push_back(raw_words(r.lo));
        cap = 16;
        while (cap < k6.size()) cap *= 2;
        uint64_t z = 0x3C6EF372FE94F82Bull;               // splitmix64 stream of odd fold multipliers
        auto next = [&z]() {
            z += 0x9E3779B97F4A7C15ull;
            uint64_t m = z;
            m = (m ^ (m >> 30)) * 0xBF58476D1CE4E5B9ull;
            m = (m ^ (m >> 27)) * 0x94D049BB133111EBull;
            return uint32_t(m ^ (m >> 31)) | 1u;
        };
        for (bool ok = false; !ok;) {
            for (int tries = 0; tries < 16 && !ok; ++tries) {
                for (auto& f : img.fold) f = next();
                img.mul6 = next();
                ok = cuckoo6(k6, cap, img.mul6, img.fold, slot6);
            }
            if (!ok) cap *= 2;
            if (cap > (1u << 16)) { why = "IPv6 host-route hash failed"; return false; }
        }
        img.cap6 = cap;
        rel_k6 = uint32_t(opt.tail.size()) * 4;
        for (uint32_t pos = 0; pos < 2 * cap; ++pos) {
            std::array<uint32_t, 4> w{};
            if (slot6[pos] >= 0) {
                w = k6[size_t(slot6[pos])];
            } else {                                      // a key that never probes this slot
                const int sdx = pos >= cap ? 1 : 0;
                for (uint32_t c = 0; h6_slot(w = {0u, 0u, 0u, c}, cap, img.mul6, img.fold, sdx) == pos; ++c) {}
            }
            opt.tail.insert(opt.tail.end(), w.begin(), w.end());
        }
        rel_r6 = uint32_t(opt.tail.size()) * 4;
        opt.tail.resize(opt.tail.size() + 2 * size_t(cap), 0u);
        opt.tail.resize(align4(uint32_t(opt.tail.size())));
    }
    opt.hot_addr = side[0].root[0];                       // IPv4 sources matching no prefix
    {
        // each source rep's address space: IPv4-mapped parts in IPv4
        // addresses, the rest scaled so all of it weighs as much as the IPv4
        // block (the slot order then follows the addresses, not the reps)
        std::map<uint32_t, double> w;
        for (size_t j = 0; j < s_start.size(); ++j) {
            const u128 lo = s_start[j];
            const bool last = j + 1 == s_start.size();
            const u128 hi = last ? ~u128(0) : s_start[j + 1] - 1;     // inclusive
            const u128 a = lo > kV4Lo ? lo : kV4Lo, b = hi < kV4Hi ? hi : kV4Hi;
            double v4 = 0.0;
            if (a <= b) v4 = double(uint64_t(b - a)) + 1.0;
            const double all = double(uint64_t((hi - lo) >> 64)) * 18446744073709551616.0 + double(uint64_t(hi - lo)) + 1.0;
            w[s_rep[j]] += v4 + (all - v4) / 79228162514264337593543950336.0;   // / 2^96
        }
        opt.src_weight.assign(w.begin(), w.end());
    }
    if (!build_cls4_one(img.sem, n_rules, img.core, why, &opt)) return false;
    const uint32_t tail = img.core.off_tail;
    for (int sd = hosts ? 1 : 0; sd < 2; ++sd) {
        img.fe_key[sd] = tail + rel_key[sd];
        img.fe_val[sd] = tail + rel_val[sd];
    }
    if (trie) {
        Cls4Image& c = img.core;
        for (uint32_t k = 0; k < img.fe_n[0]; ++k) c.words[img.fe_val[0] / 4 + k] = c.row_of(v6rep[k]);
        std::vector<uint16_t> cls(v4rep.size());
        for (size_t k = 0; k < v4rep.size(); ++k) cls[k] = uint16_t((c.row_of(v4rep[k]) - c.off_cells) / c.row_bytes);
        Trie tr;
        if (!build_trie(v4b, uint32_t(v4b.size()), cls, tail + rel_trie, 1u << 22, tr) || tr.words.size() > trie_words) {
            why = "IPv4 source trie does not fit its reserved room";
            return false;
        }
        std::copy(tr.words.begin(), tr.words.end(), c.words.begin() + (tail + rel_trie) / 4);
        c.off_trie = tail + rel_trie;
        c.trie_depth = tr.depth;
    }
    if (hosts) {
        Cls4Image& c = img.core;
        img.h4 = tail + rel_h4;
        img.k6 = tail + rel_k6;
        img.r6 = tail + rel_r6;
        for (int f = 0; f < 2; ++f) img.dflt_row[f] = c.row_of(side[0].root[f]);
        // (an empty slot's filler key never probes it: its row is never read)
        if (!side[0].pf[0].empty())
            for (size_t pos = 0; pos < tab4.size(); ++pos)
                c.words[(img.h4 + 8 * pos) / 4 + 1] = c.row_of(side[0].base[0][uint32_t(tab4[pos] >> 32)]);
        for (size_t pos = 0; pos < slot6.size(); ++pos)
            if (slot6[pos] >= 0) c.words[img.r6 / 4 + pos] = c.row_of(side[0].base[1][size_t(slot6[pos])]);
    }
    return true;
}

}  // namespace cls

// ---------------------------------------------------------------------------
// Orientation: the classifier keys its classes on the packet's source
// address.  evalACL tests the two networks symmetrically (a dst parse error
// is a FAIL term once the src matched, aclengine_mock.go:513-524, which
// SemRule already states as dst ANY + FAIL), so the same rules with src and
// dst exchanged, run on packets with src and dst exchanged, give the same
// first match.  Tables keyed on destinations (a pod's egress list from IP
// blocks: one source class, every rule in one long list) compile far better
// that way.
// ---------------------------------------------------------------------------
namespace cls {

std::vector<SemRule> swap_sides(const std::vector<SemRule>& sem) {
    std::vector<SemRule> out(sem);
    for (SemRule& r : out) {
        std::swap(r.src_any, r.dst_any);
        std::swap(r.src, r.dst);
    }
    return out;
}

namespace {

// (LDS-resident, every slot in LDS, cells in LDS, not the template scan,
// list mode, -LDS bytes); wide list modes 5, 6 rank as 4, 3
std::array<int64_t, 6> image_rank(const Cls4Image& m) {
    const bool wide = m.list_mode >= 5;
    const uint32_t lm = m.list_mode == 5 ? 4u : m.list_mode == 6 ? 3u : m.list_mode;
    return {m.lds_ok ? 1 : 0, m.n_lctr == m.n_ctr ? 1 : 0, wide ? 0 : 1, lm >= 1 ? 1 : 0, int64_t(lm),
            -int64_t(m.lds_bytes)};
}

bool good_enough(const Cls4Image& m) {
    return m.lds_ok && m.n_lctr == m.n_ctr && m.list_mode >= 1 && m.list_mode <= 4;
}

// option orient=src|dst (diagnostics, tests): one orientation only
int forced_orient() { return compile_opts().orient; }

}  // namespace

bool build_cls4(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img, std::string& why,
                const Cls4Opts* opt) {
    const int f = opt ? 0 : forced_orient();
    if (f == 1) {
        if (!build_cls4_one(swap_sides(sem), n_rules, img, why, opt)) return false;
        img.swap = 1;
        return true;
    }
    const bool ok = build_cls4_one(sem, n_rules, img, why, opt);
    if (f == 0 || opt || (ok && good_enough(img))) return ok;
    Cls4Image alt;
    std::string why2;
    if (!build_cls4_one(swap_sides(sem), n_rules, alt, why2, nullptr)) return ok;
    if (ok && !(image_rank(alt) > image_rank(img))) return true;
    img = std::move(alt);
    img.swap = 1;
    return true;
}

bool build_other4(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img, std::string& why) {
    Cls4Opts opt;
    opt.other = true;
    return build_cls4_one(sem, n_rules, img, why, &opt);
}

bool build_pair4(const std::vector<SemRule>& sem, uint32_t n_rules, bool swap, Cls4Image& img, std::string& why) {
    Cls4Opts opt;
    opt.with_other = true;
    if (!build_cls4_one(swap ? swap_sides(sem) : sem, n_rules, img, why, &opt)) return false;
    img.swap = swap ? 1 : 0;
    return true;
}

bool build_cls16(const std::vector<SemRule>& sem, uint32_t n_rules, Cls16Image& img, std::string& why) {
    const int f = forced_orient();
    if (f == 1) {
        if (!build_cls16_one(swap_sides(sem), n_rules, img, why)) return false;
        img.core.swap = 1;
        return true;
    }
    const bool ok = build_cls16_one(sem, n_rules, img, why);
    if (f == 0 || (ok && good_enough(img.core))) return ok;
    Cls16Image alt;
    std::string why2;
    if (!build_cls16_one(swap_sides(sem), n_rules, alt, why2)) return ok;
    if (ok && !(image_rank(alt.core) > image_rank(img.core))) return true;
    img = std::move(alt);
    img.core.swap = 1;
    return true;
}

}  // namespace cls
