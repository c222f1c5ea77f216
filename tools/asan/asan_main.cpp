// Host sanitizer run (ASan + UBSan) of the rule compiler (vpp_amd/csrc
// compile.cpp, the cls_compile_v4 / cls_compile_v16 entry points of
// engine.cpp) and of the CPU oracle (oracle/aclengine_ref.c), on the ACLs
// tools/asan/dump_acls.py writes: random adversarial ACLs (malformed CIDRs,
// nil sections, IPv6), the rendered config 2/3/5 tables and gen-policy lists.
// No GPU: the compiler and the oracle are host code.  For every ACL it
// compiles both layouts, then classifies random packets with the oracle's
// literal and pre-parsed evaluators and requires they agree.
// build + run: tools/asan/run.sh
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/contivcls.h"

extern "C" {
typedef struct orc_ctable orc_ctable;
int orc_classify_faithful(const cls_rule*, uint32_t, int, const void*, const void*, const uint16_t*,
                          const uint8_t*, uint64_t, uint8_t*, uint64_t*);
orc_ctable* orc_compile(const cls_rule*, uint32_t);
void orc_ctable_free(orc_ctable*);
int orc_classify_fast(const orc_ctable*, int, const void*, const void*, const uint16_t*, const uint8_t*, uint64_t,
                      uint8_t*, uint64_t*, int);
}

static int compile(int (*fn)(const cls_rule*, uint32_t, void*, uint64_t, uint64_t*), const std::vector<cls_rule>& r) {
    uint64_t need = 0;
    int rc = fn(r.data(), uint32_t(r.size()), nullptr, 0, &need);
    if (rc != CLS_OK) return rc;
    std::vector<uint8_t> blob(need);
    rc = fn(r.data(), uint32_t(r.size()), blob.data(), need, &need);
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "r");
    if (!f) return 2;
    std::mt19937_64 rng(7);
    std::vector<std::string> strs;
    char line[4096];
    int acls = 0, fails = 0;
    std::vector<cls_rule> rules;
    std::vector<std::string> nets;
    auto run = [&]() {
        // the networks' storage is stable now: point the rules at it
        for (size_t i = 0; i < rules.size(); ++i) {
            rules[i].src_network = nets[2 * i] == "-" ? nullptr : nets[2 * i].c_str();
            rules[i].dst_network = nets[2 * i + 1] == "-" ? nullptr : nets[2 * i + 1].c_str();
        }
        const int r4 = compile(cls_compile_v4, rules), r16 = compile(cls_compile_v16, rules);
        const size_t n = 3000;
        for (int af : {4, 16}) {
            std::vector<uint8_t> s(n * 16), d(n * 16), pr(n), v1(n), v2(n);
            std::vector<uint16_t> dp(n);
            for (size_t i = 0; i < n * 16; ++i) { s[i] = uint8_t(rng()); d[i] = uint8_t(rng()); }
            for (size_t i = 0; i < n; ++i) {
                pr[i] = uint8_t(rng() % 5);
                dp[i] = uint16_t(rng());
                if (af == 16 && (rng() & 1)) {        // IPv4-mapped
                    std::memset(&s[16 * i], 0, 10);
                    s[16 * i + 10] = s[16 * i + 11] = 0xFF;
                }
            }
            std::vector<uint64_t> c1(rules.size() + 1), c2(rules.size() + 1);
            orc_classify_faithful(rules.data(), uint32_t(rules.size()), af, s.data(), d.data(), dp.data(), pr.data(),
                                  n, v1.data(), c1.data());
            orc_ctable* t = orc_compile(rules.data(), uint32_t(rules.size()));
            if (t) {
                orc_classify_fast(t, af, s.data(), d.data(), dp.data(), pr.data(), n, v2.data(), c2.data(), 1);
                orc_ctable_free(t);
                if (v1 != v2 || c1 != c2) ++fails;
            }
        }
        std::printf("acl %d: %zu rules, compile v4 %d v16 %d\n", acls, rules.size(), r4, r16);
        ++acls;
        rules.clear();
        nets.clear();
    };
    while (std::fgets(line, sizeof line, f)) {
        if (line[0] == '=') {                       // end of an ACL
            run();
            continue;
        }
        cls_rule r;
        std::memset(&r, 0, sizeof r);
        char src[256], dst[256];
        unsigned v[14];
        int act;
        if (std::sscanf(line, "%u %d %255s %255s %u %u %u %u %u %u %u %u %u %u %u %u", &v[0], &act, src, dst, &v[1],
                        &v[2], &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12]) != 16)
            return 3;
        r.flags = v[0];
        r.acl_action = act;
        r.tcp_src_lo = v[1]; r.tcp_src_hi = v[2]; r.tcp_dst_lo = v[3]; r.tcp_dst_hi = v[4];
        r.udp_src_lo = v[5]; r.udp_src_hi = v[6]; r.udp_dst_lo = v[7]; r.udp_dst_hi = v[8];
        r.icmp_code_first = v[9]; r.icmp_code_last = v[10]; r.icmp_type_first = v[11]; r.icmp_type_last = v[12];
        rules.push_back(r);
        nets.push_back(src);
        nets.push_back(dst);
    }
    std::fclose(f);
    std::printf("%d ACLs, %d oracle disagreements\n", acls, fails);
    return fails ? 1 : 0;
}
