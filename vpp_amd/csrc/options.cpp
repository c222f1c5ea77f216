// The options reader (options.hpp): option strings and
// cls_engine_set_option keys onto Opts fields.
#include "options.hpp"

#include <cstdlib>
#include <cstring>

namespace cls {

namespace {

thread_local const Opts* t_compile = nullptr;

bool num(const char* v, long long& out) {
    if (!v || !*v) return false;
    char* end = nullptr;
    out = std::strtoll(v, &end, 0);
    return end && *end == '\0';
}

}  // namespace

const Opts& compile_opts() {
    static const Opts defaults;
    return t_compile ? *t_compile : defaults;
}

CompileScope::CompileScope(const Opts& o) : prev(t_compile) { t_compile = &o; }
CompileScope::~CompileScope() { t_compile = prev; }

bool opts_set(Opts& o, const char* key, const char* value, std::string& why) {
    if (!key) {
        why = "option key is NULL";
        return false;
    }
    const Opts d;
    const std::string k(key);
    long long x = 0;
    const bool reset = value == nullptr;
    if (!reset && k != "orient" && k != "conn_plan" && !num(value, x)) {
        why = "option " + k + ": not a number: " + value;
        return false;
    }
    const bool b = x != 0;
    const int i = int(x);
    // one line per switch: key, field, value (reset: the default)
#define OPT(name, field, val)                         \
    if (k == name) {                                  \
        o.field = reset ? d.field : (val);            \
        return true;                                  \
    }
    OPT("lds_budget", lds_budget, i)
    OPT("src_search", src_search, b)
    OPT("phash_dense", phash_dense, b)
    OPT("list_mode_max", list_mode_max, i)
    OPT("list_mode", list_mode, i)
    OPT("trie", trie, i)
    OPT("wide", wide, i)
    OPT("v16_src_search", v16_src_search, i)
    OPT("v16_src_trie", v16_src_trie, i)
    OPT("debug_modes", debug_modes, b)
    OPT("pair4", pair4, b)
    OPT("other_cap", other_cap, uint32_t(x))
    OPT("wg_per_cu", wg_per_cu, i)
    OPT("debug_floor", debug_floor, b)
    OPT("fold_split", fold_split, b)
    OPT("conn_bitmap", conn_bitmap, b)
    OPT("conn_pair", conn_pair, b)
    OPT("conn_pre_rules", conn_pre_rules, b)
    OPT("conn_pre_narrow", conn_pre_narrow, b)
    OPT("pair_other_global", pair_other_global, b)
    OPT("pair_other_late", pair_other_late, i)
    OPT("pair_o4", pair_o4, b)
    OPT("pair_map_lds", pair_map_lds, b)
    OPT("pair_class", pair_class, b)
    OPT("pair_lq", pair_lq, i)
    OPT("conn_no_lds", conn_no_lds, i)
    OPT("conn_jobs", conn_jobs, b)
    OPT("conn_wg_per_cu", conn_wg_per_cu, i)
    OPT("conn_wg768", conn_wg768, b)
    OPT("conn_flush_atomic", conn_flush_atomic, b)
    OPT("debug_conn", debug_conn, b)
    OPT("batch_layout", batch_layout, i)
#undef OPT
    if (k == "pair_qcap") {
        o.pair_qcap = reset ? d.pair_qcap : uint32_t(x);
        o.pair_qcap_set = !reset;
        return true;
    }
    if (k == "orient") {
        const std::string v = reset ? "" : value;
        if (!reset && v != "src" && v != "dst") {
            why = "option orient: src or dst";
            return false;
        }
        o.orient = reset ? d.orient : v == "dst" ? 1 : 0;
        return true;
    }
    if (k == "conn_plan") {
        const std::string v = reset ? "" : value;
        const int p = v == "32j" ? 0 : v == "16j" ? 1 : v == "32s" ? 2 : v == "16s" ? 3 : -1;
        if (!reset && p < 0) {
            why = "option conn_plan: 32j, 16j, 32s or 16s";
            return false;
        }
        o.conn_plan = reset ? d.conn_plan : p;
        return true;
    }
    why = "unknown option " + k;
    return false;
}

bool opts_parse(Opts& o, const char* list, std::string& why) {
    if (!list) return true;
    const std::string s(list);
    size_t at = 0;
    while (at < s.size()) {
        size_t end = s.find(',', at);
        if (end == std::string::npos) end = s.size();
        const std::string kv = s.substr(at, end - at);
        at = end + 1;
        if (kv.empty()) continue;
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) {
            why = "option without a value: " + kv;
            return false;
        }
        if (!opts_set(o, kv.substr(0, eq).c_str(), kv.substr(eq + 1).c_str(), why)) return false;
    }
    return true;
}

}  // namespace cls
