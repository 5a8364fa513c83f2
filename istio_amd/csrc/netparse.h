// netparse.h -- Go 1.9 net.ParseIP / ParseCIDR restated for host and device (src/net/ip.go:
// parseIPv4, parseIPv6, ParseIP, ParseCIDR, CIDRMask, IP.Mask, IPNet.Contains).  Used by the
// lowering/packing (host) and by the list-adapter kernels (device), so both parse identically.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define MXP_NHD __host__ __device__ inline
#else
#define MXP_NHD inline
#endif

namespace mxpnet {

constexpr int kBig = 0xFFFFFF;

// dtoi / xtoi (ip.go): digits from s, stopping at the first non-digit; fails on none or >= big
MXP_NHD bool dtoi(const uint8_t* s, uint32_t n, int* v, uint32_t* used) {
    int x = 0;
    uint32_t i = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        x = x * 10 + (s[i] - '0');
        if (x >= kBig) return false;
    }
    if (i == 0) return false;
    *v = x;
    *used = i;
    return true;
}

MXP_NHD int hexval(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

MXP_NHD bool xtoi(const uint8_t* s, uint32_t n, int* v, uint32_t* used) {
    int x = 0;
    uint32_t i = 0;
    for (; i < n; i++) {
        const int h = hexval(s[i]);
        if (h < 0) break;
        x = x * 16 + h;
        if (x >= kBig) return false;
    }
    if (i == 0) return false;
    *v = x;
    *used = i;
    return true;
}

// parseIPv4: dotted quad (leading zeros allowed in Go 1.9) -> 16-byte v4-in-v6 form
MXP_NHD bool parse_v4(const uint8_t* s, uint32_t n, uint8_t out[16]) {
    uint8_t q[4];
    for (int i = 0; i < 4; i++) {
        if (n == 0) return false;
        if (i) {
            if (*s != '.') return false;
            s++;
            n--;
        }
        int v;
        uint32_t c;
        if (!dtoi(s, n, &v, &c) || v > 255) return false;
        q[i] = (uint8_t)v;
        s += c;
        n -= c;
    }
    if (n) return false;
    for (int i = 0; i < 10; i++) out[i] = 0;
    out[10] = out[11] = 0xff;
    for (int i = 0; i < 4; i++) out[12 + i] = q[i];
    return true;
}

// parseIPv6 (zone not allowed), including the embedded-IPv4 tail and the `::` ellipsis
MXP_NHD bool parse_v6(const uint8_t* s, uint32_t n, uint8_t ip[16]) {
    for (int i = 0; i < 16; i++) ip[i] = 0;
    int ell = -1;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ell = 0;
        s += 2;
        n -= 2;
        if (!n) return true;
    }
    int i = 0;
    while (i < 16) {
        int v;
        uint32_t c;
        if (!xtoi(s, n, &v, &c) || v > 0xFFFF) return false;
        if (c < n && s[c] == '.') {
            if (ell < 0 && i != 12) return false;
            if (i + 4 > 16) return false;
            uint8_t t[16];
            if (!parse_v4(s, n, t)) return false;
            for (int k = 0; k < 4; k++) ip[i + k] = t[12 + k];
            n = 0;
            i += 4;
            break;
        }
        ip[i] = (uint8_t)(v >> 8);
        ip[i + 1] = (uint8_t)v;
        i += 2;
        s += c;
        n -= c;
        if (!n) break;
        if (*s != ':' || n == 1) return false;
        s++;
        n--;
        if (*s == ':') {
            if (ell >= 0) return false;
            ell = i;
            s++;
            n--;
            if (!n) break;
        }
    }
    if (n) return false;
    if (i < 16) {
        if (ell < 0) return false;
        const int k = 16 - i;
        for (int j = i - 1; j >= ell; j--) ip[j + k] = ip[j];
        for (int j = ell + k - 1; j >= ell; j--) ip[j] = 0;
    } else if (ell >= 0) {
        return false;
    }
    return true;
}

// ParseIP: the first '.' or ':' decides the family
MXP_NHD bool parse_ip(const uint8_t* s, uint32_t n, uint8_t out[16]) {
    for (uint32_t i = 0; i < n; i++) {
        if (s[i] == '.') return parse_v4(s, n, out);
        if (s[i] == ':') return parse_v6(s, n, out);
    }
    return false;
}

// 16-byte form holds an IPv4 address (IP.To4 != nil)
MXP_NHD bool is_v4(const uint8_t ip[16]) {
    for (int i = 0; i < 10; i++)
        if (ip[i]) return false;
    return ip[10] == 0xff && ip[11] == 0xff;
}

}  // namespace mxpnet
