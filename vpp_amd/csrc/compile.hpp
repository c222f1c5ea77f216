// Rule-set compiler: ACL rules (cls_rule) -> device layouts.
//
// Stage 1 (semantic): every rule is reduced, per packet address family, to
// the decision evalACL makes for it (mock/aclengine/aclengine_mock.go:480-664):
//   src prefix | ANY, dst prefix | ANY, and per packet protocol
//   (TCP, UDP, ICMP, OTHER) either SKIP (the `continue` branches) or
//   TERM(port range, result) where result is DENY/PERMIT/REFLECT/FAILURE.
//   Unconditional failures (MacipRule, missing IpRule/Ip, Other section, src
//   parse error) become an ANY/ANY rule that terminates every protocol with
//   FAILURE; a dst parse error does the same once the src prefix matched.
//   Rules after an unconditional terminator are unreachable and dropped.
//
// Stage 2a (linear): the semantic rules in order, 48 B each -- the table of the
//   ballot kernel (small tables, GPU cross-check, OTHER-protocol fallback).
// Stage 2b (classifier, IPv4): first-match is decided per packet by
//   (1) the source address's elementary interval (binary search over the
//       sorted boundaries of every source prefix), which fixes the set of
//       source prefixes covering it (they nest: a laminar family) -> class;
//   (2) the cell (class, protocol) -> the ordered candidate list of rules that
//       cover that class and do not SKIP that protocol, truncated after the
//       first rule that matches every packet of the cell;
//   (3) a scan of the candidate list comparing only dst prefix and dst port.
//   Candidates are stored as 16-bit ids of deduplicated templates
//   (dst, port range, result); identical lists are stored once.  Hit counters
//   are one u32 per (cell, position) "slot", mapped back to rule indices
//   after the kernel (slot 0 = default DENY = counter R).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/contivcls.h"
#include "goparse.hpp"
#include "options.hpp"

namespace cls {

// Cuckoo hash pair of the hash-LPM source lookup (shared by compiler and kernel).
constexpr uint32_t kMaxHashLens = 3;
constexpr uint32_t kMaxHot = 16;       // hot slots counted in per-lane LDS rows
constexpr uint32_t kMaxBvSteps = 7;    // bit-vector search depth (lists <= 32 entries)
constexpr uint32_t kMaxTrieDepth = 8;  // source trie: deepest leaf search (src mode 4)
constexpr uint32_t kMaxPortClasses = 256;  // list modes 2, 3: global port classes
constexpr uint32_t kPortUniform = 1u << 19;  // port radix: chunk inside one class
constexpr uint32_t kMaxPortClasses3 = 64;   // list modes 3, 4: class x 4 fits a byte
constexpr uint32_t kMaxPortHash = 64;       // list mode 4: ports outside the default class
constexpr uint32_t kLdsBudget = 160 * 1024;  // LDS of one classify workgroup
constexpr uint32_t kLdsReserved = 16;        // after the image's LDS: the OTHER-queue fill counter
// One multiply per key: p = key x mul; table 0 takes the top L bits of p,
// table 1 the next L bits (L = log2 cap <= 16).  The compiler picks mul from a
// fixed list until the cuckoo build succeeds.
__host__ __device__ inline uint32_t lpm_h0(uint32_t k, uint32_t mul, uint32_t L) {
    return (k * mul) >> (32u - L);
}
__host__ __device__ inline uint32_t lpm_h1(uint32_t k, uint32_t mul, uint32_t L) {
    return ((k * mul) >> (32u - 2u * L)) & ((1u << L) - 1u);
}

enum : uint8_t { RES_DENY = 0, RES_PERMIT = 1, RES_REFLECT = 2, RES_FAIL = 3 };
enum : int { P_TCP = 0, P_UDP = 1, P_ICMP = 2, P_OTHER = 3, NPROTO = 4 };


struct Term {
    bool term = false;     // false = SKIP (rule never matches this protocol)
    uint16_t lo = 0, hi = 0xFFFF;
    uint8_t res = RES_DENY;
};

struct SemRule {
    uint32_t index = 0;    // rule index in the ACL
    bool src_any = true;
    Prefix src;
    bool dst_any = true;
    Prefix dst;
    Term t[NPROTO];
};

// Reduce the ACL for packets of family `fam` (4: both addresses IPv4; 0: each
// address of either family -- networks of both families kept).  Returns CLS_OK or
// CLS_E_INVAL (a rule with nil Matches: Go would panic).
int semantic_rules(const cls_rule* rules, uint32_t n, int fam, std::vector<SemRule>& out,
                   std::string& err);

// ---- linear table (device layout, 48 B per rule) ---------------------------
struct alignas(16) LinRule4 {
    uint32_t src_addr, src_mask, dst_addr, dst_mask;
    uint32_t port[NPROTO];   // lo | (hi - lo) << 16
    uint32_t meta;           // byte p: bit7 = TERM, bits0-1 = result
    uint32_t index;          // rule index in the ACL
    uint32_t pad[2];
};
static_assert(sizeof(LinRule4) == 48, "LinRule4 layout");

std::vector<LinRule4> linear4(const std::vector<SemRule>& sem);
// the rules with src and dst exchanged (Cls4Image::swap)
std::vector<SemRule> swap_sides(const std::vector<SemRule>& sem);

// ---- connection-path rules (cls_connect_batch; staged in LDS) -------------
// Only the TCP and UDP terms carry a port range: an ICMP or OTHER term always
// spans every port (icmp_term, and evalACL's fall-through), so the compact
// forms drop those two port words.  meta byte p: bit7 = TERM, bits0-1 = result.
struct alignas(16) ConnRule4 {
    uint32_t src_addr, src_mask, dst_addr, dst_mask;
    uint32_t port[2];        // TCP, UDP: lo | (hi - lo) << 16
    uint32_t meta;
    uint32_t index;          // rule index in the ACL
};
static_assert(sizeof(ConnRule4) == 32, "ConnRule4 layout");
// 16-byte packets: addresses compared as loaded (network-order bytes in
// little-endian words).  An IPv4 prefix is stored in its IPv4-mapped form
// with full masks on words 0-2, so only IPv4-mapped packets can match it; an
// IPv6 prefix sets fam bit 0 (src) / 1 (dst), and an IPv4-mapped packet never
// matches it (Go 1.9 IPNet.Contains compares lengths after To4,
// aclengine_mock.go:506,520).  ANY: masks zero, fam bit clear.
struct alignas(16) ConnRule16 {
    uint32_t src[4], smask[4], dst[4], dmask[4];
    uint32_t port[2];
    uint32_t meta;
    uint32_t index_fam;      // rule index << 2 | fam bits
};
static_assert(sizeof(ConnRule16) == 80, "ConnRule16 layout");
// sem from semantic_rules(..., fam 4) / (..., fam 0) respectively
std::vector<ConnRule4> conn_rules4(const std::vector<SemRule>& sem);
std::vector<ConnRule16> conn_rules16(const std::vector<SemRule>& sem);

// ---- IPv4 classifier image -------------------------------------------------
struct Cls4Image {
    std::vector<uint32_t> words;   // read-only LDS image, 16 B aligned sections
    uint32_t off_bounds = 0, off_iclass = 0, off_cells = 0, off_lists = 0, off_tmpl = 0;
    uint32_t img_bytes = 0;        // size of the read-only image
    uint32_t n_bounds = 0, n_classes = 0, n_tmpl = 0, n_list_entries = 0, n_ctr = 0;
    uint32_t search_top = 0;       // largest power of two <= n_bounds
    uint32_t lds_bytes = 0;        // image + counters (u32 per slot), 16 B aligned
    std::vector<uint32_t> ctr_rule;  // slot -> rule index (R = default DENY)
    // source lookup: mode 0 = interval binary search, 1 = hash LPM, 3 = rows
    // given by the caller (16-byte core), 4 = source trie (off_trie)
    uint32_t mode = 0;
    // mode 4: level 1 (256 u32, indexed by src >> 24) at off_trie, then the
    // nodes and leaves (compile.cpp build_trie); trie_depth = deepest leaf
    uint32_t off_trie = 0, trie_depth = 0;
    uint32_t default_class = 0;    // hash mode: class of addresses no hashed prefix covers
    uint32_t n_hash = 0;           // hashed prefix lengths, ascending
    uint32_t hash_mask[kMaxHashLens] = {}, hash_shift[kMaxHashLens] = {};  // shift = 32 - L
    uint32_t hash_mul[kMaxHashLens] = {};
    uint32_t hash_cap[kMaxHashLens] = {}, off_hash[kMaxHashLens] = {};
    // class rows: a class's n_cells cells at off_cells + class x
    // row_bytes; hash entries hold that byte address, not the class index
    uint32_t row_bytes = 12;
    uint32_t default_row = 0;      // hash mode: row of default_class
    // candidate lists: mode 0 = scan of template ids, 1 = bit vectors (all lists
    // <= 32) with per-list port search, 2 = bit vectors with global port
    // classes, 3 = port-filtered sublists (per list and port class, the dst
    // intervals with their first-match outcome; searched with one state word),
    // 4 = 3 with hashed port classes; 5, 6 = 4, 3 with wide cells in global
    // memory (gcells)
    uint32_t list_mode = 0;
    // list modes 5, 6: the cells are not in the LDS image but in gcells
    // (global memory, after the image in the device buffer): uint2 {pointer
    // table LDS byte address, counter base} per (class, protocol), so the
    // counter base has 32 bits and the classes any number; a class row is a
    // byte offset into gcells (off_cells 0, row_bytes 8 x n_cells)
    std::vector<uint32_t> gcells;
    uint32_t sub_bytes = 0;        // modes 3, 4: end of the pointer tables (< 64 KiB)
    // mode 4: port perfect hash at LDS 0: e = u32 at byte mulhi(port, mul) &
    // mask4, class x 4 = (e & 0xFFFF) == port ? e >> 16 : port_dflt
    uint32_t port_mul = 0, port_mask4 = 0, port_dflt = 0;
    uint32_t off_bv = 0;
    uint32_t bv_steps_d = 0, bv_steps_p = 0;   // largest search depths over the lists
    // list mode 2: global port classes (radix at off_ptop), result-hi word used
    uint32_t off_ptop = 0, n_pclass = 0, bv_wide = 0;
    // slots [0, n_hot) -- default DENY and the cells of the class covering
    // most of the address space -- are counted in per-lane LDS rows
    // (n_hot x 64 u32 at off_hot, after the slot counters)
    uint32_t n_hot = 1;
    uint32_t off_hot = 0;
    // Counter tiers: slots [n_hot, n_lctr) are LDS counters after the image,
    // u32 (ctr16 = 0, then n_lctr = n_ctr) or u16 (ctr16 = 1: a lane whose
    // add takes a counter to 0x8000 moves 0x8000 to the slot's global
    // counter); slots [n_lctr, n_ctr) are counted in global memory
    // (wave-aggregated atomics).
    uint32_t n_lctr = 0;
    uint32_t ctr16 = 0;
    // Cells per class: 3 -- TCP, UDP, ICMP (a packet's cell is min(proto,
    // 2)); 1 -- OTHER alone (Cls4Opts::other)
    uint32_t n_cells = 3;
    bool lds_ok = false;           // image and LDS counters fit the LDS budget (place_counters)
    // 1: classes are keyed on the packet's DESTINATION address (built from the
    // rules with src and dst exchanged, compile.cpp build_cls4): the caller
    // passes the packet's dst as the kernel's src and vice versa; the linear
    // fallback rules (lin) are in that exchanged frame too
    uint32_t swap = 0;
    uint32_t off_tail = 0;         // Cls4Opts::tail words (read-only, after the sections above)
    // host only: the elementary source intervals and their classes
    std::vector<uint32_t> h_bounds;
    std::vector<uint16_t> h_iclass;
    uint32_t row_of(uint32_t addr) const;   // byte address of the class row of `addr`
};

struct Cls4Opts {
    std::vector<uint32_t> tail;    // extra read-only words appended to the image
    int64_t hot_addr = -1;         // the hot class is this address's (default: the widest)
    // The address space each source value stands for, as sorted (value,
    // weight) pairs (default: 1 per value).  A core compiled in rep space
    // (the 16-byte layout) passes its reps' real widths, so the slot order
    // below ranks classes by the addresses they cover, not by their reps.
    std::vector<std::pair<uint32_t, double>> src_weight;
    bool ext_src = false;          // no source lookup sections (mode 3: the caller finds rows)
    // The OTHER image: one cell per class for protocol values outside
    // ProtocolType (evalACL's switch has no case for them,
    // aclengine_mock.go:527-643: the networks alone decide), interval search
    // and template scan, read from global memory by the few lanes holding
    // such a packet (kernels.hip run_n).  Its slots follow the main image's.
    bool other = false;
    // The pair launch's image (k4_pair.hip): a fourth cell per class for
    // protocols > 2 beside TCP, UDP and ICMP, so a connection batch
    // classifies those connections with the others -- no OTHER queue, no
    // second image.  Its slots are its own (ctr_rule).
    bool with_other = false;
};

// The OTHER image of a rule set (in the main image's orientation: pass the
// swapped rules for a destination-keyed one).
bool build_other4(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img, std::string& why);
// The pair launch's image of `sem` in the orientation `swap` (Cls4Opts::with_other)
bool build_pair4(const std::vector<SemRule>& sem, uint32_t n_rules, bool swap, Cls4Image& img, std::string& why);

uint32_t lds_budget();
bool place_counters(Cls4Image& img, uint32_t budget, bool partial);

// Build the image in the better orientation (Cls4Image::swap); returns false
// (with reason) if the table does not fit the 16-bit list / template indices.
// With opt (the 16-byte core): the given orientation only.
bool build_cls4(const std::vector<SemRule>& sem, uint32_t n_rules, Cls4Image& img,
                std::string& why, const Cls4Opts* opt = nullptr);

// ---- 16-byte (IPv6 and IPv4-mapped) classifier image ----------------------
// evalACL's Contains (Go 1.9 net.IPNet.Contains) reduces a v4-mapped packet
// address to 4 bytes and never matches an address of one family against a
// network of the other.  The 16-byte path maps both families into one 32-bit
// space of *representatives* that preserves every containment the rule set
// can observe, then runs the IPv4 classifier over it:
//   - the prefixes of one side (src or dst) of one family form a tree (any
//     two prefixes nest or are disjoint); each node gets a block (base, len)
//     of the 32-bit space inside its parent's block -- children at sub-block
//     indices 1..k of the parent's next ceil(log2(k+1)) bits, index 0 left to
//     the node itself -- under a family root block (IPv4 0/1, IPv6 1/1);
//   - a packet address maps to the base of its longest matching prefix's
//     block (the family root's base when none matches), found by one binary
//     search over the 128-bit elementary intervals of all prefixes (IPv4
//     prefixes at ::ffff:a.b.c.d, the v4-mapped range holding IPv4 packets;
//     inside it only IPv4 prefixes count, outside it only IPv6 prefixes);
//   - a rule's prefix becomes its block: the rep of an address lies in a
//     block iff the address lies in the prefix.
// Front-end tables per side s (0 src, 1 dst), in the image's tail: fe_top[s]
// keys of 16 B (interval start - 1 as u64 hi, u64 lo; padding all-ones),
// then fe_n[s] u32 reps.  When every interval start b has hi64(b) = 0 and
// lo64(b) <= 2^48, or lo64(b) = 0 (IPv4 and IPv6 prefixes up to /64), the
// keys are 8 B: key8(x) = hi64 == 0 ? min(lo64, 2^48) : 2^48 + min(hi64,
// 2^64 - 1 - 2^48), monotone and exact against such starts.
//
// Source front end, src_mode 1 (every source prefix a host route -- rendered
// global tables: pod /32s and /128s): exact cuckoo hashes straight to the
// class row (core mode 3, no rep on the hot path).  IPv4-mapped addresses:
// key = the address's last 4 bytes as loaded (little-endian word), entries
// {key, row} 8 B, h = key x mul4 (lpm_h0 / lpm_h1).  IPv6: keys are the 16
// bytes as loaded (k6: 16 B per slot), rows at r6 (u32 per slot); f = w0 x
// fold[0] ^ w1 x fold[1] ^ w2 x fold[2] ^ w3, h = f x mul6.  Misses take the
// family's default row.  The source interval table (src_mode 0's) stays in
// global memory for the protocol > 2 fallback, which needs the rep.
//
// Source front end, src_mode 2 (sources not all host routes, many IPv4
// intervals -- the IP-block lists of gen-policy.py): IPv4-mapped sources
// through a trie over the address's IPv4 word straight to the class row (the
// IPv4 classifier's source trie, at core.off_trie / core.trie_depth, leaves
// carrying the core's classes), every other source through the interval
// search of side 0 restricted to the non-IPv4 intervals, whose values are
// rows (core mode 3).  The whole interval table stays in global memory for
// protocols > 2, as in src_mode 1.
struct Cls16Image {
    Cls4Image core;                // classifier over the rules in rep space
    std::vector<SemRule> sem;      // the rules in rep space (linear fallback)
    uint32_t fe_key[2] = {}, fe_val[2] = {}, fe_top[2] = {}, fe_n[2] = {};
    uint32_t fe_k8[2] = {};        // 8-B keys: key8(start) - 1 (see key8)
    uint32_t src_mode = 0;         // 0: interval search -> rep; 1: host-route hashes -> row; 2: IPv4 trie -> row
    uint32_t h4 = 0, cap4 = 0, mul4 = 0;
    uint32_t k6 = 0, r6 = 0, cap6 = 0, mul6 = 0, fold[3] = {};
    uint32_t dflt_row[2] = {};     // per family (0 IPv4, 1 IPv6)
    std::vector<uint32_t> src_search;  // src_mode 1, 2: the source interval table (keys, reps), global memory
    uint32_t src_search_val = 0;   // byte offset of its reps
    uint32_t src_search_top = 0, src_search_k8 = 0;   // its padded key count, 8-B keys
};
__host__ __device__ inline uint32_t fold6(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                          const uint32_t* f) {
    return (w0 * f[0]) ^ (w1 * f[1]) ^ (w2 * f[2]) ^ w3;
}
// sem: semantic_rules(..., fam 0, ...) -- a packet's src and dst may be of
// different families (Contains tests each address on its own).
bool build_cls16(const std::vector<SemRule>& sem, uint32_t n_rules, Cls16Image& img, std::string& why);

}  // namespace cls
