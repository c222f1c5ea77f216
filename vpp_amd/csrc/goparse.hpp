// Go 1.9 net.ParseCIDR / net.ParseIP semantics for the rule compiler.
//
// The engine receives the ACL's CIDR strings verbatim (include/contivcls.h
// cls_rule) and must reproduce what evalACL's net.ParseCIDR + IPNet.Contains
// do with them (mock/aclengine/aclengine_mock.go:500-520): which strings fail
// to parse (-> FAILURE verdict) and which addresses each network contains.
// Contains() reduces every network to an effective (family, prefix):
//   * a.b.c.d/n                     -> IPv4 /n
//   * IPv6 string whose masked IP is IPv4-mapped (::ffff:a.b.c.d/n, n >= 96)
//                                   -> IPv4 /(n-96)   (networkNumberAndMask)
//   * any other IPv6 string         -> IPv6 /n
// Packets are reduced with IP.To4() the same way, so an IPv4 packet only ever
// meets IPv4 prefixes and a native IPv6 packet only IPv6 prefixes.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>

namespace cls {

struct Prefix {
    int fam = 0;          // 4 or 16; 0 = parse error
    uint8_t addr[16] = {};  // masked network number (fam bytes used)
    int len = 0;          // prefix length within the family
};

namespace goparse {

constexpr int kBig = 0xFFFFFF;

// dtoi: decimal prefix of s; ok=false on empty or overflow
inline bool dtoi(const char* s, int n, int& val, int& used) {
    int v = 0, i = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; ++i) {
        v = v * 10 + (s[i] - '0');
        if (v >= kBig) { val = kBig; used = i; return false; }
    }
    val = v; used = i;
    return i != 0;
}

inline bool xtoi(const char* s, int n, int& val, int& used) {
    int v = 0, i = 0;
    for (; i < n; ++i) {
        char c = s[i];
        int d;
        if (c >= '0' && c <= '9') d = c - '0';
        else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
        else break;
        v = v * 16 + d;
        if (v >= kBig) { val = 0; used = i; return false; }
    }
    val = v; used = i;
    return i != 0;
}

// parseIPv4 -> 4 bytes
inline bool ipv4(const char* s, int n, uint8_t out[4]) {
    for (int i = 0; i < 4; ++i) {
        if (n == 0) return false;
        if (i > 0) {
            if (*s != '.') return false;
            ++s; --n;
        }
        int v, used;
        if (!dtoi(s, n, v, used) || v > 0xFF) return false;
        s += used; n -= used;
        out[i] = static_cast<uint8_t>(v);
    }
    return n == 0;
}

// parseIPv6 (no zone) -> 16 bytes
inline bool ipv6(const char* s, int n, uint8_t ip[16]) {
    std::memset(ip, 0, 16);
    int ellipsis = -1;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        s += 2; n -= 2;
        if (n == 0) return true;
    }
    int i = 0;
    while (i < 16) {
        int v, used;
        if (!xtoi(s, n, v, used) || v > 0xFFFF) return false;
        if (used < n && s[used] == '.') {
            if (ellipsis < 0 && i != 12) return false;
            if (i + 4 > 16) return false;
            uint8_t v4[4];
            if (!ipv4(s, n, v4)) return false;
            std::memcpy(ip + i, v4, 4);
            n = 0;
            i += 4;
            break;
        }
        ip[i] = static_cast<uint8_t>(v >> 8);
        ip[i + 1] = static_cast<uint8_t>(v);
        i += 2;
        s += used; n -= used;
        if (n == 0) break;
        if (*s != ':' || n == 1) return false;
        ++s; --n;
        if (*s == ':') {
            if (ellipsis >= 0) return false;
            ellipsis = i;
            ++s; --n;
            if (n == 0) break;
        }
    }
    if (n != 0) return false;
    if (i < 16) {
        if (ellipsis < 0) return false;
        int shift = 16 - i;
        for (int j = i - 1; j >= ellipsis; --j) ip[j + shift] = ip[j];
        for (int j = ellipsis + shift - 1; j >= ellipsis; --j) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return false;
    }
    return true;
}

inline bool is_v4_mapped(const uint8_t ip[16]) {
    static const uint8_t pfx[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};
    return std::memcmp(ip, pfx, 12) == 0;
}

}  // namespace goparse

// net.ParseCIDR + networkNumberAndMask, reduced to an effective Prefix.
// Returns fam = 0 when Go would return an error.
inline Prefix parse_cidr(const char* str) {
    Prefix p;
    int n = static_cast<int>(std::strlen(str));
    int slash = -1;
    for (int i = 0; i < n; ++i)
        if (str[i] == '/') { slash = i; break; }
    if (slash < 0) return p;
    uint8_t ip[16];
    int bits = 32;
    uint8_t v4[4];
    if (goparse::ipv4(str, slash, v4)) {
        std::memcpy(ip, v4, 4);
    } else {
        bits = 128;
        if (!goparse::ipv6(str, slash, ip)) return p;
    }
    int len, used;
    const char* m = str + slash + 1;
    int mn = n - slash - 1;
    if (!goparse::dtoi(m, mn, len, used) || used != mn || len < 0 || len > bits) return p;
    int nbytes = bits / 8;
    // ip.Mask(CIDRMask(len, bits))
    for (int b = 0; b < nbytes; ++b) {
        int ones = len - 8 * b;
        uint8_t mk = ones >= 8 ? 0xff : (ones <= 0 ? 0 : static_cast<uint8_t>(0xff << (8 - ones)));
        ip[b] &= mk;
    }
    if (bits == 32) {
        p.fam = 4; p.len = len;
        std::memcpy(p.addr, ip, 4);
    } else if (goparse::is_v4_mapped(ip)) {
        // networkNumberAndMask: To4() of the masked IP succeeds; the mask is
        // cut to its last 4 bytes.  A mapped IP survives masking only if
        // len >= 96 (bytes 10-11 keep 0xffff).
        p.fam = 4; p.len = len - 96;
        std::memcpy(p.addr, ip + 12, 4);
    } else {
        p.fam = 16; p.len = len;
        std::memcpy(p.addr, ip, 16);
    }
    return p;
}

// net.ParseIP reduced with To4(): fam 4 / 16, or 0 when nil.
inline Prefix parse_ip(const char* str) {
    Prefix p;
    int n = static_cast<int>(std::strlen(str));
    for (int i = 0; i < n; ++i) {
        if (str[i] == '.') {
            if (goparse::ipv4(str, n, p.addr)) { p.fam = 4; p.len = 32; }
            return p;
        }
        if (str[i] == ':') {
            uint8_t ip[16];
            if (!goparse::ipv6(str, n, ip)) return p;
            if (goparse::is_v4_mapped(ip)) { p.fam = 4; p.len = 32; std::memcpy(p.addr, ip + 12, 4); }
            else { p.fam = 16; p.len = 128; std::memcpy(p.addr, ip, 16); }
            return p;
        }
    }
    return p;
}

}  // namespace cls
