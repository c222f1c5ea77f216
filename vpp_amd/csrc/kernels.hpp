// Launch interface of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "compile.hpp"

namespace cls {

// IPv4 packet batch in device memory (structure of arrays)
struct Pkts4 {
    const uint32_t* src;
    const uint32_t* dst;
    const uint16_t* dport;
    const uint8_t* proto;
    uint64_t n;
};

// 16-byte packet batch: network-order addresses (IPv4-mapped = IPv4 packet)
struct Pkts16 {
    const uint4* src;          // 16-B aligned
    const uint4* dst;
    const uint16_t* dport;
    const uint8_t* proto;
    uint64_t n;
    uint32_t vec;              // dport 8-B, proto and verdict 4-B aligned: 4 packets per lane
};

// 16-byte front end (Cls16Image): per side (0 src, 1 dst) the key array's
// and the rep array's LDS byte offsets and the padded key count
struct Fe16 {
    uint32_t key[2], val[2], top[2];
    uint32_t k8[2];            // 8-B keys (compile.hpp key8)
    uint32_t src_mode;         // 1: host-route hashes -> class row (Cls16Image)
    uint32_t h4, cap4, mul4, s4_0, s4_1, L4;             // IPv4-mapped hash (s0 = 32 - L, s1 = 32 - 2 L)
    uint32_t k6, r6, cap6, mul6, s6_0, s6_1, L6, fold[3]; // IPv6 hash
    uint32_t dflt4, dflt6;     // rows of the families' sources no prefix covers
    const uint8_t* gsrc;       // src_mode 1, 2: the source interval table in global memory
    uint32_t gval;             // (keys at 0, reps at gval; gtop keys, 8 B when gk8)
    uint32_t gtop, gk8;
};

struct Cls4Dev {
    const uint32_t* img;       // classifier image (device)
    uint32_t img_bytes;
    uint32_t off_bounds, off_iclass, off_cells, off_lists, off_tmpl;
    uint32_t search_top;       // power of two; bounds padded to 2*search_top
    uint32_t n_ctr;            // slot counters in the image's LDS tail
    uint32_t lds_bytes;
    const LinRule4* lin;       // linear rules (the 16-byte kernel's FORCE_LINEAR cross-check)
    uint32_t n_lin;
    uint32_t n_rules;          // R
    uint32_t mode;             // 0 interval search, 1 hash LPM, 4 source trie
    uint32_t off_trie, trie_depth;   // mode 4: level 1 at off_trie (compile.cpp build_trie)
    const uint8_t* gcells;     // list modes 5, 6: wide cells (uint2 {pointer table, counter base})
    uint32_t default_row;      // source lookup miss: byte address of the default class's cells
    uint32_t n_hash;
    uint32_t hash_mask[kMaxHashLens], hash_shift[kMaxHashLens], hash_cap[kMaxHashLens];
    uint32_t off_hash[kMaxHashLens];
    uint32_t hash_mul[kMaxHashLens], hash_shift1[kMaxHashLens];   // shift1 = 32 - 2 L
    uint32_t list_mode;        // 0 template scan, 1 bit vectors, 2 + global port classes,
                               // 3 port-filtered sublists, 4 + hashed port classes
    uint32_t bv_steps;         // bit-vector search depth (max over lists, both dims)
    uint32_t n_hot;            // slots [0, n_hot) are counted in per-lane LDS rows
    uint32_t off_hot;          // byte offset of the rows (n_hot x 64 u32) in LDS
    uint32_t off_ptop;         // list mode 2: port radix
    uint32_t bv_wide;          // some list > 16 entries: result bits need the hi word
    uint32_t row_bytes;        // cells per class row x cell size (interval search scales by it)
    uint32_t port_mul, port_mask4, port_dflt;   // list mode 4: port perfect hash at LDS 0
    uint32_t n_lctr;           // LDS-resident image: slots [0, n_lctr) counted in LDS, the rest in gslot
    uint32_t ctr16;            // LDS counters are u16 (compile.hpp counter tiers)
    uint32_t* part;            // LDS-resident image: per-workgroup slot counters [grid][n_lctr]
    uint32_t* oq;              // OTHER queue {fill per wave, a segment of oq_cap indices per wave}
                               // (null: classify such packets in place)
    uint32_t oq_cap;
    unsigned long long* zero = nullptr;   // the call's rule counters, cleared by the launch's
    uint32_t n_zero = 0;                  // workgroups before the finish launch adds to them
};

// Whether the classify dispatchers have a kernel for an image of source
// lookup `mode` and `list_mode`, LDS-resident or not; rep16: the 16-byte
// core (mode 3 = rows from the front end's host-route hashes).  The source
// trie and the wide cells exist only in LDS.
inline bool cls_kernel_exists(uint32_t mode, uint32_t list_mode, bool lds, bool rep16) {
    if (list_mode > 6 || (list_mode >= 5 && !lds)) return false;
    switch (mode) {
    case 0: case 1: return true;
    case 3: return rep16;
    case 4: return lds && list_mode >= 3;
    default: return false;
    }
}

struct LaunchCfg {
    int grid;                  // workgroups (persistent, grid-stride)
    hipStream_t stream;
    Cls4Dev other;             // classify kernels: the OTHER image (protocols > 2), global memory
    // classify kernels: events stamped with the kernel's own start / stop
    // (hipExtLaunchKernel: part of the dispatch, no marker packets between
    // kernels); null: none
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
};

// verdict may be null; gslot: u64 slot counters (added to)
hipError_t launch_classify4_cls(const Cls4Dev& t, const Pkts4& p, uint8_t* verdict,
                                unsigned long long* gslot, bool lds_resident, bool vec,
                                const LaunchCfg& cfg);
// lin: linear first match over the rep-space rules (t.lin) after the front end
hipError_t launch_classify16_cls(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint8_t* verdict,
                                 unsigned long long* gslot, bool lds_resident, bool lin,
                                 const LaunchCfg& cfg);
// rule_out (not null): each packet's terminating rule (R: the default DENY)
// instead of counting into gslot
hipError_t launch_classify4_linear(const LinRule4* rules, uint32_t n_lin, uint32_t n_rules,
                                   const Pkts4& p, uint8_t* verdict, unsigned long long* gslot,
                                   const LaunchCfg& cfg, uint32_t* rule_out = nullptr);
// slot-mode words (result | slot << 2) -> verdict (may be null) and
// slot_rule[slot] per packet; rule may alias words
hipError_t launch_slot_rules(const uint32_t* words, const uint32_t* slot_rule, uint32_t n, uint8_t* verdict,
                             uint32_t* rule, hipStream_t s);
// slot_val[i] += sum_w part[w * n + i], w < rows (the classify kernel's
// partials); zero[0, n_zero) = 0 in the same launch (zero may be null)
hipError_t launch_fold(const uint32_t* part, uint32_t rows, uint32_t n, unsigned long long* slot_val,
                       unsigned long long* zero, uint32_t n_zero, hipStream_t s);
// out[csr[k].y] += slot_val[csr[k].x], then slot_val[csr[k].x] = 0, for k < n
// (csr: every slot once, grouped by rule); out null: clear only
hipError_t launch_remap(unsigned long long* slot_val, const uint2* csr, uint32_t n, unsigned long long* out,
                        hipStream_t s);
// The end of a classify call, one launch: tiles of 64 slots fold the
// workgroups' LDS partials (part, rows x n_lctr; null: none) and, with
// remap, move slot_val + partials to the rule counters out (slot -> rule:
// slot_rule, entries kHotRule | h for the hot rules -- rules with many slots,
// summed per tile in LDS -- then their n_hot rule ids) and clear slot_val;
// without remap (an earlier chunk of a long batch) slot_val += partials.
// out must be cleared before (the classify launch's zero).
constexpr uint32_t kOtherSegs = 16;   // OTHER queue segments per classify workgroup (its waves)
constexpr uint32_t kHotRule = 0x80000000u;
constexpr uint32_t kMaxHotRules = 64;
struct FinishArgs {
    const uint32_t* part;
    uint32_t rows, n_lctr;
    unsigned long long* slot_val;
    uint32_t n_slots;
    const uint32_t* slot_rule;
    uint32_t n_hot;
    unsigned long long* out;
    bool remap;
    // the OTHER queue of the classify launch (null: none): oq_rows (its
    // workgroups) x kOtherSegs fills, then as many segments of oq_cap
    // entries, one per classify wave; blocks after the tiles classify a
    // workgroup's queued packets (protocols > 2) on the OTHER image and count
    // them per rule -- other_map: compact rule index of each of the n_other
    // OTHER slots, then the n_orules rules
    const uint32_t* oq;
    uint32_t oq_rows, oq_cap;
    uint32_t qmask = 0;          // entries are (packet >> 2) | mask << 28: the packets 4 g + q of the
                                 // mask's bits (IPv4 launches: one entry per lane and wave step)
    const uint32_t* other_map;
    uint32_t n_other, n_orules;
    uint32_t split = 1;          // blocks per tile of 64 slots, each folding a share of the rows
                                 // (remap with partials only; the host's fold_split)
};
// finish4 / finish16: the OTHER packets' loads from the 4- / 16-byte batch
hipError_t launch_finish4(const FinishArgs& f, const Cls4Dev& o, const Pkts4& p, uint8_t* verdict, hipStream_t s);
hipError_t launch_finish16(const FinishArgs& f, const Cls4Dev& t, const Cls4Dev& o, const Fe16& fe, const Pkts16& p,
                           uint8_t* verdict, hipStream_t s);
// the classify kernels' packet stream without the lookups (stream floor);
// exactly one of p4 / p16; p4 needs 16-B aligned src/dst, 8-B dport, 4-B
// proto and verdict (variant bit 0: load and use instead of the next step's
// loads in flight; bit 1: the protocol stream a cached load, not
// non-temporal); p16 covers whole 256-packet wave steps only
hipError_t launch_stream(const Pkts4* p4, const Pkts16* p16, uint8_t* verdict, int grid, int variant,
                         hipStream_t s);

// Slot mode of the classify kernels (connection batches): out[i] = result |
// slot << 2 (u32), no counting; protocols > 2 in place, their slots after
// the main image's.  p4: one packet per lane (no vector requirements).
hipError_t launch_classify4_slots(const Cls4Dev& t, const Pkts4& p, uint32_t* out, bool lds_resident,
                                  const LaunchCfg& cfg);
hipError_t launch_classify16_slots(const Cls4Dev& t, const Fe16& fe, const Pkts16& p, uint32_t* out,
                                   bool lds_resident, const LaunchCfg& cfg);
// The pair image's slot -> rule map as u16 (map, n16 16-B units), staged at
// LDS byte srl after the image (0: none; the launch reads slot_rule)
struct PairMap {
    const uint16_t* map = nullptr;
    uint32_t srl = 0, n16 = 0;
};
// Both tuples of a connection batch in one launch (LDS-resident IPv4 image):
// out[i] = the SYN tuple (p.src, p.dst, p.dport) and out[stride + i] the
// SYN-ACK tuple (p.dst, p.src, sport), result | slot << 2 each.  The OTHER
// image (o, offsets rebased to LDS byte o_at) is staged beside the main one
// when o_at != 0; with o_late (o_at 0, offsets image-relative) it is staged
// at LDS 0, over the main image, once every wave of the workgroup has left
// its main loop.  Connections of protocol > 2 go to the wave's queue
// segment -- lq_cap entries in the LDS after the images, then oq_cap in oq
// (segment w of the grid's waves) -- and are classified on the OTHER image
// after the wave's main loop, one per lane (in place when the segment is
// full, from global memory unless the image sits beside the main one).
// cdiv != 0 (ceil(2^32 / t.row_bytes)): the OTHER image's source classes are
// t's, so a queued connection carries its two classes and the drain skips
// the OTHER source search.  o4: t is the pair image (compile.hpp
// Cls4Opts::with_other, four cells per class): protocols > 2 are classified
// with the others -- no queue, no OTHER image, slots of t's own.
// Needs 16-B aligned src / dst / out / out + stride, 8-B dport / sport, 4-B
// proto; stride a multiple of 4.
// slot_rule (may be null): write each word's counter index ctr_base +
// slot_rule[slot] in place of the slot (counting connection batches).
// wbytes: 4 -- u32 words (SYN at out[i], SYN-ACK at out[stride + i]); 2 --
// u16 words (counter indices < 2^14), the two in one u32 at out[i] (SYN |
// SYN-ACK << 16: one load for the connection kernel); 1 -- only
// the two ACLActions, one byte per connection (SYN result | SYN-ACK result
// << 2) at byte i (batches that do not count)
hipError_t launch_classify4_pair(const Cls4Dev& t, const Cls4Dev& o, uint32_t o_at, const Pkts4& p,
                                 const uint16_t* sport, uint32_t* out, uint64_t stride, uint32_t* oq,
                                 uint32_t oq_cap, const uint32_t* slot_rule, uint32_t ctr_base, uint32_t wbytes,
                                 uint32_t lq_cap, bool o_late, uint32_t cdiv, bool o4, const PairMap& sm,
                                 const LaunchCfg& cfg);
// LDS byte offset of the pair launch's queue segments: after the main image,
// the OTHER image beside it (o_at != 0), or the larger of the two (o_late)
inline uint32_t pair_queue_lds(uint32_t img_bytes, uint32_t o_at, uint32_t o_bytes, bool o_late) {
    const uint32_t end = o_at ? o_at + o_bytes : o_late && o_bytes > img_bytes ? o_bytes : img_bytes;
    return (end + 15u) & ~15u;
}
// The OTHER queue segment of one pair-launch workgroup (kPairBlock threads)
// that holds every connection its lanes visit, 4 per lane per step, in 16-B
// entries; the engine caps the segment (oq_cap entries; the overflow is
// classified in place)
constexpr int kPairBlock = 1024;
inline uint64_t pair_queue_words(uint64_t n, int grid) {
    const uint64_t nsteps = n / 4, nthreads = uint64_t(grid) * kPairBlock;
    return 4ull * kPairBlock * ((nsteps + nthreads - 1) / nthreads);
}

struct ConnDesc {                // one bound ACL for the connection kernel
    uint32_t rule_off;           // linear ACLs: first rule in the call's rule pool
    uint32_t n;                  // linear rules
    uint32_t n_rules;            // R (default DENY: rule R)
    uint32_t ctr_off;            // counting: counter of rule 0 in the call's counter space
    int32_t pre_blk;             // classifier slot words' block in ConnArgs::pre (-1: none)
    uint32_t pad;
    const uint32_t* slot_rule;   // pre_blk >= 0: slot -> rule index
    uint32_t bm_off;             // bitmap form (IPv4): byte offset of its tables in the pool; ~0u: none
    uint32_t bm_sd;              // bitmap form: source | destination interval counts << 16
    uint32_t bm_tu;              // bitmap form: TCP | UDP port interval counts << 16
    uint32_t bm_w;               // bitmap form: u32 words per row
};
struct IfAcls {                  // interface -> (inbound, outbound) ConnDesc index, -1 = nil
    int32_t in, out;
    int32_t in_pre, out_pre;     // their classifier slot words' block in ConnArgs::pre (-1: none)
};
static_assert(sizeof(ConnDesc) == 48 && sizeof(IfAcls) == 16, "connect_kernel reads the staged tables as 16-B words");
// The bitmap form of a linear IPv4 ACL in the connection pool (engine.cpp
// conn_bitmap4), u32 words from a 16-B aligned base: header {W, ns, nd, nr,
// n0, n1, n2, n3} (its counts also in the ACL's ConnDesc), then the src
// table {ns keys, ns x W row words}, the dst table, the four protocol tables
// (TCP, UDP by destination port; ICMP and OTHER one row each: n2 = n3 = 1),
// then nr {meta, index} pairs.  Keys are the starts of
// the elementary intervals (key 0 first); a row has bit i set when pool
// rule i matches that interval's addresses (ports); the first match is the
// lowest set bit of src row & dst row & protocol row.
constexpr uint32_t kConnBmHeader = 32;
// Connection counting: the call counters come in kConnCtrCopies copies, so
// that the workgroups' end-of-launch adds to a popular counter spread over
// that many addresses (same-address device atomics serialise); the scatter
// launch sums the copies.  LDS counters are u16 pairs: a workgroup takes at
// most kConnWgConns connections per launch (4 calls each stay below 2^16).
// Connection batches with at most this many large ACLs load every one's
// result words together with the connection's fields (no second dependent
// global round trip behind the interface lookup).
// The connection kernel's state-machine table: one byte per (4 call
// results, same interface, unknown interface).
constexpr uint32_t kConnStateEntries = 1024;
constexpr uint32_t kConnEarlyBlocks = 2;
constexpr uint32_t kConnCtrCopies = 16;
constexpr uint32_t kConnWgConns = 16383;
__host__ __device__ constexpr uint32_t conn_lds_ctr_bytes(uint32_t n_ctr) { return (n_ctr + 1u) / 2u * 4u; }

struct ConnArgs {
    const ConnDesc* desc;
    const IfAcls* ifs;
    uint32_t n_ifs;
    const void* rules;           // ConnRule4 / ConnRule16 pool (global memory)
    uint32_t rules_bytes;        // staged into LDS at address 0 when the launch says so
    uint32_t n_ctr;              // counting: counter space (sum of R + 1 over the descriptors)
    uint32_t ctr_lds;            // counting: LDS byte offset of the counters (LDS variant; u16
                                 // pairs: counter j in half j & 1 of word j >> 1, a workgroup
                                 // evaluates at most kConnWgConns connections per launch)
    uint32_t sm_lds;             // LDS byte offset of the state machine's table (kConnStateEntries B)
    uint32_t ctr16;              // counting, LDS variant: u16 counter pairs (else u32 counters)
    uint32_t* ctr_rows;          // counting, LDS variant: workgroup b stores its LDS counter words
                                 // as row b (null: device atomics into the copies of ctr)
    unsigned long long* ctr;     // counting: the call's u64 counters, kConnCtrCopies copies of
                                 // n_ctr (workgroup b adds to copy b % kConnCtrCopies)
    const uint32_t* src_if;
    const uint32_t* dst_if;
    const void* src;             // u32 host order, or 16-B network-order addresses
    const void* dst;
    const uint16_t* sport;
    const uint16_t* dport;
    const uint8_t* proto;
    uint64_t n;
    uint8_t* out;
    uint32_t n_desc;             // descriptors in desc
    uint32_t meta_lds;           // LDS byte offset of the staged desc + ifs tables; ~0u: global reads
    const uint32_t* pre;         // classifier slot words of the large ACLs: block b at pre + 2 b pre_stride
                                 // (SYN tuple, then SYN-ACK at + pre_stride); null when there are none
    uint64_t pre_stride;
    uint32_t n_big;              // blocks at pre (the large ACLs); <= kConnEarlyBlocks: every block's
                                 // words loaded with the connection's fields, before the interfaces
    uint32_t pre_rules;          // the words carry counter indices (descriptor base + rule), not slots
    uint32_t pre_bytes;          // the words' width: 4; 2 (u16 counter-index words, both tuples'
                                 // in one u32 per connection, SYN | SYN-ACK << 16, block b at
                                 // pre + b pre_stride); 1 (block b is one byte per
                                 // connection at (uint8_t*) pre + b pre_stride: SYN result |
                                 // SYN-ACK result << 2, batches that do not count)
    uint32_t bm_steps;           // bitmap forms: lower-bound steps of the largest interval table
    uint32_t job_lds;            // IPv4: LDS byte offset of the waves' job lists (512 B per wave)
};
// k16: 16-byte addresses; lds_rules: stage the pool; count: 0 none, 1 LDS
// counters, 2 global (wave-aggregated) counters; grid: persistent workgroups
// of `block` threads (512, 768 or 1024); lds: dynamic LDS bytes (pool, LDS
// counters, a.meta_lds tables)
hipError_t launch_connect(const ConnArgs& a, bool k16, bool lds_rules, int count, int grid, int block, size_t lds,
                          hipStream_t s);
// the connection batch's stream without the evaluation (whole 4-connection
// groups of an IPv4 batch; 16-B aligned src / dst / src_if / dst_if, 8-B
// ports, 4-B proto and out)
hipError_t launch_stream_conn(const ConnArgs& a, int grid, hipStream_t s);
// tables' connection counters += the call's counters (ConnDesc ctr_off ..
// + n_rules), which are cleared: a workgroup per descriptor and 256
// counters (max_rules: the largest n_rules of the descriptors)
// rows of the LDS counter words (n_rows rows of nw words; ctr16: u16 pairs)
// -> the tables' connection counters (descriptor d's counters start at
// desc[d].ctr_off, ascending), summed kConnRowsPerSlab rows per thread
constexpr uint32_t kConnRowsPerSlab = 64;
hipError_t launch_conn_rows(const uint32_t* rows, uint32_t n_rows, uint32_t nw, bool ctr16, uint32_t n_ctr,
                            const ConnDesc* desc, uint32_t n_desc, unsigned long long* const* table_ctr,
                            hipStream_t s);
// the call counters (n_slabs copies of n_ctr u64, summed; clear: zero what
// was read) -> the tables' connection counters
hipError_t launch_conn_scatter(const ConnDesc* desc, unsigned long long* const* table_ctr, uint32_t n_desc,
                               uint32_t max_rules, unsigned long long* call_ctr, uint32_t n_slabs, bool clear,
                               uint32_t n_ctr, hipStream_t s);

struct TrafficDev {
    uint64_t seed;
    uint32_t pct_pod, pct_dst, pct_port, pct_icmp;
    const uint32_t* pods; uint32_t n_pods;
    const uint32_t* dst_addrs; const uint8_t* dst_lens; uint32_t n_dst;
    const uint16_t* ports; uint32_t n_ports;
};
hipError_t launch_gen4(const TrafficDev& t, uint64_t first, uint64_t n, uint32_t* src,
                       uint32_t* dst, uint16_t* sport, uint16_t* dport, uint8_t* proto,
                       hipStream_t s);

// 16-byte stream (contivcls.h cls_traffic_spec16); pools as (hi, lo) u64 pairs
struct TrafficDev16 {
    uint64_t seed;
    uint32_t pct_pod, pct_dst, pct_port, pct_icmp;
    const uint64_t* pods; uint32_t n_pods;
    const uint64_t* dst_addrs; const uint8_t* dst_lens; uint32_t n_dst;
    const uint16_t* ports; uint32_t n_ports;
};
hipError_t launch_gen16(const TrafficDev16& t, uint64_t first, uint64_t n, uint4* src, uint4* dst,
                        uint16_t* sport, uint16_t* dport, uint8_t* proto, hipStream_t s);

int max_lds_bytes();             // per-workgroup LDS the classify kernel may use
int cls_block();                 // classify workgroup size

}  // namespace cls
