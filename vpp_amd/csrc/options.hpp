// Tuning and diagnostic switches of the engine and the classifier compiler
// (tests and measurements: forced list modes, counter tiers, launch plans).
//
// The library never reads the process environment.  An engine's options
// start at these defaults and change only through cls_engine_set_option
// (include/contivcls.h); they are plain fields read by the calls that use
// them, so a launch pays no lookup.  The compiler entry points without an
// engine (cls_compile_v4 / v16) take theirs as an option string.  The
// compiler reads the options of the compile in progress through
// compile_opts(): table_compile and cls_compile_* install them for the
// duration of the compile (CompileScope), on the calling thread.
#pragma once
#include <cstdint>
#include <string>

namespace cls {

struct Opts {
    // ---- compiler (compile.cpp) -------------------------------------------
    int lds_budget = -1;        // LDS bytes for an image and its counters (-1: the kernel's budget)
    bool src_search = false;    // the interval search for sources, never the hash LPM
    bool phash_dense = true;    // false: at least 2 port-hash slots per port
    int list_mode_max = -1;     // cap on the list mode
    int list_mode = -1;         // exactly this list mode when the compiler has it
    int trie = -1;              // source trie: 0 never, 1 only (-1: when it fits best)
    int wide = -1;              // wide cells: 0 never, 1 first
    int v16_src_search = -1;    // 16-byte front end: 1 the interval search (no host hash, no trie)
    int v16_src_trie = -1;      // 16-byte front end: 1 the source trie, 0 never
    int orient = -1;            // 0 source-keyed, 1 destination-keyed (-1: the better one)
    bool debug_modes = false;   // stderr: why a list mode was refused
    bool pair4 = false;         // cls_compile_v4: the connection pair launch's four-cell image (tests)
    // ---- classify launches (engine.cpp) -----------------------------------
    uint32_t other_cap = 0;     // OTHER queue entries per workgroup (0: sized by the batch)
    int wg_per_cu = 0;          // classify workgroups per CU (0: by LDS)
    bool debug_floor = false;   // stderr: every stream shape's time
    bool fold_split = true;     // finish launch: a slot tile's rows over several blocks when tiles are few
    // ---- connection batches (engine.cpp) ----------------------------------
    bool conn_bitmap = true;    // bitmap form of linear IPv4 ACLs
    bool conn_pair = true;      // both tuples of a large ACL in one launch (classify4_pair)
    bool conn_pre_rules = true; // counting: the pair launch writes counter indices, not slots
    bool conn_pre_narrow = true;// u8 results / u16 words where they fit (else u32 words)
    uint32_t pair_qcap = 0;     // pair launch: OTHER queue entries per wave (0: sized by the batch)
    bool pair_qcap_set = false;
    bool pair_other_global = false;  // pair launch: the OTHER image read from global memory
    int pair_other_late = 1;    // pair launch: the OTHER image staged over the main one for the drain when
                                // it does not fit beside it (2: always -- tests; 0: never)
    bool pair_o4 = true;        // pair launch: the four-cell pair image where it fits (else the OTHER queue)
    bool pair_map_lds = true;   // pair image, counting: the slot -> rule map staged in LDS
    bool pair_class = true;     // pair launch: queued OTHER connections carry their source classes
    int pair_lq = -1;           // pair launch: cap on the OTHER queue entries per wave in LDS
    int conn_no_lds = 0;        // bit 0 rules, bit 1 counters, bit 2 descriptors from global memory
    int conn_wg_per_cu = 0;     // measurements: cap on the connection kernel's workgroups per CU (0: none)
    bool conn_jobs = true;      // the waves' LDS job lists (else owner search and shuffles)
    bool conn_wg768 = true;     // two 768-thread workgroups per CU where three 512-thread ones do not fit
    int conn_plan = -1;         // counting LDS plan 0..3 = 32j 16j 32s 16s (-1: scored)
    bool conn_flush_atomic = false;  // LDS counters flushed by device atomics, not per-workgroup rows
    bool debug_conn = false;    // stderr: a connection launch's LDS plan
    // ---- batches (fleet.cpp) ----------------------------------------------
    int batch_layout = 2;       // 0 packed, 1 one allocation per field, 2 staggered fields
};

// key = value (value NULL: the default).  Returns false with `why` for an
// unknown key or a malformed value.
bool opts_set(Opts& o, const char* key, const char* value, std::string& why);
// "key=value,key=value" (NULL or "": nothing)
bool opts_parse(Opts& o, const char* list, std::string& why);

// The options of the compile in progress on this thread (defaults outside one).
const Opts& compile_opts();
struct CompileScope {
    const Opts* prev;
    explicit CompileScope(const Opts& o);
    ~CompileScope();
    CompileScope(const CompileScope&) = delete;
    CompileScope& operator=(const CompileScope&) = delete;
};

}  // namespace cls
