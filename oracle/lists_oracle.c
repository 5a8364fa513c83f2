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

/*
 * String lists (stringList.go:29-80): a set of the non-empty entries and overrides -- keyed by
 * strings.ToUpper for the case-insensitive kind -- and checkList = membership of the symbol (upper-
 * cased likewise).  Go's map is a hash table; so is this restatement (open addressing), used as the
 * compiled CPU baseline of the list bench and checked against lists.py's Python form.
 *
 * strings.ToUpper = strings.Map(unicode.ToUpper, s) (Go 1.9 src/strings/strings.go): runes decoded as
 * `for i, c := range s` does (invalid byte = U+FFFD, width 1), the input's own bytes until the first
 * rune whose upper case differs, utf8.EncodeRune of every rune from there on.  unicode.ToUpper above
 * ASCII: the sorted (rune, upper) pairs of oracle/unicode_upper.json, set by oracle_upper_table.
 */
#include <stdlib.h>

static uint32_t* g_upper = NULL; /* [2 n]: rune, upper */
static size_t g_nupper = 0;

void oracle_upper_table(const uint32_t* pairs, size_t n) {
    free(g_upper);
    g_upper = (uint32_t*)malloc(2 * n * sizeof(uint32_t) + 8);
    memcpy(g_upper, pairs, 2 * n * sizeof(uint32_t));
    g_nupper = n;
}

static uint32_t go_upper_rune(uint32_t r) {
    if (r < 0x80) return r >= 'a' && r <= 'z' ? r - 32 : r;
    size_t a = 0, b = g_nupper;
    while (a < b) {
        size_t m = (a + b) / 2;
        if (g_upper[2 * m] < r) a = m + 1;
        else b = m;
    }
    return a < g_nupper && g_upper[2 * a] == r ? g_upper[2 * a + 1] : r;
}

/* utf8.DecodeRuneInString (Go 1.9 src/unicode/utf8/utf8.go) */
static uint32_t go_decode(const uint8_t* s, size_t i, size_t n, size_t* w) {
    uint32_t c0 = s[i];
    *w = 1;
    if (c0 < 0x80) return c0;
    size_t left = n - i;
    if (c0 >= 0xC2 && c0 <= 0xDF) {
        if (left >= 2 && s[i + 1] >= 0x80 && s[i + 1] <= 0xBF) {
            *w = 2;
            return (c0 & 0x1F) << 6 | (s[i + 1] & 0x3F);
        }
    } else if (c0 >= 0xE0 && c0 <= 0xEF) {
        uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
        if (left >= 3 && s[i + 1] >= lo && s[i + 1] <= hi && s[i + 2] >= 0x80 && s[i + 2] <= 0xBF) {
            *w = 3;
            return (c0 & 0x0F) << 12 | (uint32_t)(s[i + 1] & 0x3F) << 6 | (s[i + 2] & 0x3F);
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4) {
        uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
        if (left >= 4 && s[i + 1] >= lo && s[i + 1] <= hi && s[i + 2] >= 0x80 && s[i + 2] <= 0xBF &&
            s[i + 3] >= 0x80 && s[i + 3] <= 0xBF) {
            *w = 4;
            return (c0 & 0x07) << 18 | (uint32_t)(s[i + 1] & 0x3F) << 12 | (uint32_t)(s[i + 2] & 0x3F) << 6 |
                   (s[i + 3] & 0x3F);
        }
    }
    return 0xFFFD;
}

static size_t go_encode(uint32_t r, uint8_t* o) {
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = 0xC0 | r >> 6; o[1] = 0x80 | (r & 0x3F); return 2; }
    if (r < 0x10000) { o[0] = 0xE0 | r >> 12; o[1] = 0x80 | ((r >> 6) & 0x3F); o[2] = 0x80 | (r & 0x3F); return 3; }
    o[0] = 0xF0 | r >> 18; o[1] = 0x80 | ((r >> 12) & 0x3F); o[2] = 0x80 | ((r >> 6) & 0x3F); o[3] = 0x80 | (r & 0x3F);
    return 4;
}

/* strings.ToUpper(s) into out (room for 3 n + 4 bytes); returns its length */
size_t oracle_go_to_upper(const uint8_t* s, size_t n, uint8_t* out) {
    size_t o = 0, i = 0;
    int changed = 0;
    while (i < n) {
        size_t w;
        uint32_t c = go_decode(s, i, n, &w);
        uint32_t r = go_upper_rune(c);
        if (!changed && r == c) {
            memcpy(out + o, s + i, w);
            o += w;
        } else {
            changed = 1;
            o += go_encode(r, out + o);
        }
        i += w;
    }
    return o;
}

typedef struct {
    uint8_t* keys;  /* blob of stored keys */
    uint64_t* off;  /* [n + 1] */
    uint64_t* slot; /* open addressing: entry + 1, 0 = empty */
    size_t n, cap;
    int upper;
} ostrlist;

static uint64_t fnv(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

static int strlist_find(const ostrlist* L, const uint8_t* k, size_t n) {
    for (size_t s = fnv(k, n) & (L->cap - 1);; s = (s + 1) & (L->cap - 1)) {
        uint64_t e = L->slot[s];
        if (!e) return 0;
        e--;
        if (L->off[e + 1] - L->off[e] == n && memcmp(L->keys + L->off[e], k, n) == 0) return 1;
    }
}

/* parse*StringList over entries (empty ones skipped) then overrides; returns the list */
void* oracle_strlist_new(const uint8_t* blob, const uint64_t* off, size_t n, int upper) {
    ostrlist* L = (ostrlist*)calloc(1, sizeof *L);
    L->upper = upper;
    size_t total = off[n] - off[0];
    L->keys = (uint8_t*)malloc(3 * total + 4 * n + 8);
    L->off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    L->cap = 16;
    while (L->cap < 2 * n + 2) L->cap <<= 1;
    L->slot = (uint64_t*)calloc(L->cap, sizeof(uint64_t));
    L->off[0] = 0;
    for (size_t i = 0; i < n; i++) {
        const uint8_t* s = blob + off[i];
        size_t len = off[i + 1] - off[i];
        if (!len) continue;
        uint8_t* dst = L->keys + L->off[L->n];
        size_t kl = upper ? oracle_go_to_upper(s, len, dst) : (memcpy(dst, s, len), len);
        if (strlist_find(L, dst, kl)) continue; /* a map: duplicates collapse */
        size_t sl = fnv(dst, kl) & (L->cap - 1);
        while (L->slot[sl]) sl = (sl + 1) & (L->cap - 1);
        L->slot[sl] = L->n + 1;
        L->off[L->n + 1] = L->off[L->n] + kl;
        L->n++;
    }
    return L;
}

size_t oracle_strlist_entries(const void* l) { return ((const ostrlist*)l)->n; }

void oracle_strlist_free(void* l) {
    ostrlist* L = (ostrlist*)l;
    if (!L) return;
    free(L->keys);
    free(L->off);
    free(L->slot);
    free(L);
}

/* checkList for n symbols: found[q] = 1 / 0 */
void oracle_strlist_found(const void* l, const uint8_t* blob, const uint64_t* off, size_t n, int8_t* found,
                          int threads) {
    const ostrlist* L = (const ostrlist*)l;
#pragma omp parallel num_threads(threads)
    {
        size_t cap = 256;
        uint8_t* buf = (uint8_t*)malloc(cap);
#pragma omp for schedule(dynamic, 256)
        for (size_t q = 0; q < n; q++) {
            const uint8_t* s = blob + off[q];
            size_t len = off[q + 1] - off[q];
            if (L->upper) {
                if (3 * len + 4 > cap) {
                    cap = 3 * len + 4;
                    buf = (uint8_t*)realloc(buf, cap);
                }
                len = oracle_go_to_upper(s, len, buf);
                s = buf;
            }
            found[q] = (int8_t)strlist_find(L, s, len);
        }
        free(buf);
    }
}
