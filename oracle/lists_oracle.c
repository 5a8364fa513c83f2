/*
 * ORACLE (test infrastructure only) -- C restatement of the list adapter's IP list.
 *
 * mixer/adapter/list/ipList.go: addEntry (:62-75) appends "/32" to entries without '/', then
 * net.ParseCIDR; checkList (:77-92) net.ParseIP's the symbol and scans every IPNet with Contains.
 * Go 1.9 src/net/ip.go (the reference's pinned toolchain, .circleci/config.yml): ParseCIDR, CIDRMask,
 * IP.Mask, networkNumberAndMask, IPNet.Contains -- restated below; parseIPv4 / parseIPv6 / dtoi
 * come from goval.c.  The scan stays linear like the reference (this is also the CPU baseline).
 */
#include <stdint.h>
#include <string.h>

#include "goval.h"

typedef struct {
    uint8_t ip[16];
    int iplen;
    uint8_t mask[16];
    int masklen;
} onet;

static const uint8_t v4pre[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};

/* net.ParseCIDR: returns 1 and the IPNet, or 0 (ParseError "invalid CIDR address") */
int oracle_parse_cidr(const uint8_t* s, size_t n, onet* out) {
    size_t i = 0;
    while (i < n && s[i] != '/') i++;
    if (i == n) return 0;
    uint8_t ip[16];
    int iplen = 4;
    if (!oracle_parse_ipv4(s, i, ip)) {
        iplen = 16;
        if (!oracle_parse_ipv6(s, i, ip)) return 0;
    }
    int bits;
    size_t used;
    const uint8_t* m = s + i + 1;
    size_t ml = n - i - 1;
    if (!oracle_dtoi(m, ml, &bits, &used) || used != ml || bits < 0 || bits > 8 * iplen) return 0;
    uint8_t mask[16] = {0};
    for (int k = 0, left = bits; k < iplen; k++, left -= 8) /* CIDRMask */
        mask[k] = left >= 8 ? 0xff : left <= 0 ? 0 : (uint8_t)(0xff00 >> left);
    /* IP.Mask(mask) */
    const uint8_t* src = ip;
    int srclen = 16;
    if (iplen == 4 && memcmp(ip, v4pre, 12) == 0) {
        src = ip + 12;
        srclen = 4;
    }
    if (srclen != iplen) return 0;
    memset(out, 0, sizeof *out);
    out->iplen = iplen;
    out->masklen = iplen;
    for (int k = 0; k < iplen; k++) {
        out->ip[k] = src[k] & mask[k];
        out->mask[k] = mask[k];
    }
    return 1;
}

/* IPNet.Contains(ip) with ip the 16-byte ParseIP result */
static int contains(const onet* n, const uint8_t ip16[16]) {
    /* networkNumberAndMask */
    const uint8_t* nn = n->ip;
    int nnlen = n->iplen;
    if (nnlen == 16 && memcmp(n->ip, v4pre, 12) == 0) {
        nn = n->ip + 12;
        nnlen = 4;
    }
    const uint8_t* m = n->mask;
    int mlen = n->masklen;
    if (mlen == 4) {
        if (nnlen != 4) return 0;
    } else if (mlen == 16) {
        if (nnlen == 4) {
            m = n->mask + 12;
            mlen = 4;
        }
    } else {
        return 0;
    }
    /* ip.To4() */
    const uint8_t* x = ip16;
    int xl = 16;
    if (memcmp(ip16, v4pre, 12) == 0) {
        x = ip16 + 12;
        xl = 4;
    }
    if (xl != nnlen) return 0;
    for (int i = 0; i < xl; i++)
        if ((nn[i] & m[i]) != (x[i] & m[i])) return 0;
    return 1;
}

/* checkList for n symbols: found[q] = 1 / 0, or -1 when the symbol is not an IP address */
void oracle_iplist_check(const onet* nets, size_t nn, const uint8_t* blob, const uint64_t* off, size_t n,
                         int8_t* found, int threads) {
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
    for (size_t q = 0; q < n; q++) {
        uint8_t ip[16];
        if (!oracle_parse_ip(blob + off[q], (size_t)(off[q + 1] - off[q]), ip)) {
            found[q] = -1;
            continue;
        }
        int8_t f = 0;
        for (size_t k = 0; k < nn && !f; k++) f = (int8_t)contains(&nets[k], ip);
        found[q] = f;
    }
}

size_t oracle_onet_size(void) { return sizeof(onet); }
