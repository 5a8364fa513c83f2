// dfa_dev.h -- device layout of compiled regex DFAs (regex.h) and the gfx950 stepping loop, shared
// by the predicate VM (kernels.hip: `matches`) and the list kernel (lists.hip: REGEX lists).
#pragma once

#include <stdint.h>

typedef struct mxp_dfa_hdr {
    uint32_t ncls;      // rune classes + 1 (last column = END of text)
    uint32_t start;
    uint32_t trans;     // first transition (index into mxp_dfa_set.trans)
    uint32_t ascii;     // first ASCII class entry (128 per DFA, index into mxp_dfa_set.ascii)
    uint32_t hi;        // first non-ASCII range (index into hilo / hicls)
    uint32_t hi_n;
    uint32_t skip;      // subject bytes already consumed into `start` (a rule's literal prefix, verified
                        // by the prefix index); MXP_DFA_DECIDED: the prefix alone decides a match
    uint32_t pad;
} mxp_dfa_hdr;
#define MXP_DFA_DECIDED 0xFFFFFFFFu

typedef struct mxp_dfa_set {
    const mxp_dfa_hdr* hdr;
    const uint32_t* trans;   // next state | 0xFFFFFFFF accept | 0xFFFFFFFE reject
    const uint16_t* ascii;
    const uint32_t* hilo;    // ascending non-ASCII range starts
    const uint16_t* hicls;
} mxp_dfa_set;

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>

// 8 bytes at any address of a blob with >= 16 bytes of slack (two aligned loads + funnel shift)
__device__ __forceinline__ uint64_t mxp_ld8(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7) * 8u;
    const uint64_t lo = q[0];
    return sh == 0 ? lo : (lo >> sh) | (q[1] << (64u - sh));
}

// regexp.MatchString on one subject: decode runes the way Go's inputString does (utf8 rules; an
// invalid byte is U+FFFD of width 1), map each to its class, step; END column at the end.
__device__ __forceinline__ bool mxp_dfa_run(const mxp_dfa_set& S, uint32_t dfa, const uint8_t* s, uint32_t n) {
    const mxp_dfa_hdr H = S.hdr[dfa];
    const uint32_t* T = S.trans + H.trans;
    const uint16_t* asc = S.ascii + H.ascii;
    uint32_t st = H.start;
    uint32_t i = H.skip;
    if (i == MXP_DFA_DECIDED) return true;
    // ASCII bytes come out of the aligned 8-byte word that holds them: one subject load per 8 steps
    // (the pools and symbol blobs are readable to the aligned word past their end)
    uintptr_t wa = ((uintptr_t)(s + i)) & ~(uintptr_t)7;
    uint64_t win = *(const uint64_t*)wa;
    while (i < n) {
        const uintptr_t a = (uintptr_t)(s + i);
        if ((a & ~(uintptr_t)7) != wa) {
            wa = a & ~(uintptr_t)7;
            win = *(const uint64_t*)wa;
        }
        const uint32_t c0 = (uint32_t)(win >> ((a & 7u) * 8u)) & 0xFFu;
        uint32_t cls;
        if (c0 < 0x80) {
            cls = asc[c0];
            i++;
        } else {
            const uint64_t w = mxp_ld8(s + i);  // bytes i .. i+7 (only those < n are used)
            const uint32_t left = n - i;
            const uint32_t b1 = (uint32_t)(w >> 8) & 0xFF, b2 = (uint32_t)(w >> 16) & 0xFF, b3 = (uint32_t)(w >> 24) & 0xFF;
            uint32_t r = 0xFFFD, width = 1;
            if (c0 >= 0xC2 && c0 <= 0xDF) {
                if (left >= 2 && b1 >= 0x80 && b1 <= 0xBF) {
                    r = ((c0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
                    width = 2;
                }
            } else if (c0 >= 0xE0 && c0 <= 0xEF) {
                const uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
                if (left >= 3 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF) {
                    r = ((c0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
                    width = 3;
                }
            } else if (c0 >= 0xF0 && c0 <= 0xF4) {
                const uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
                if (left >= 4 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF && b3 >= 0x80 && b3 <= 0xBF) {
                    r = ((c0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
                    width = 4;
                }
            }
            i += width;
            // last range whose start <= r
            const uint32_t* lo = S.hilo + H.hi;
            int a = 0, b = (int)H.hi_n - 1, k = 0;
            while (a <= b) {
                const int m = (a + b) >> 1;
                if (lo[m] <= r) {
                    k = m;
                    a = m + 1;
                } else {
                    b = m - 1;
                }
            }
            cls = S.hicls[H.hi + k];
        }
        st = T[(uint64_t)st * H.ncls + cls];
        if (st == 0xFFFFFFFFu) return true;
    }
    return T[(uint64_t)st * H.ncls + H.ncls - 1] == 0xFFFFFFFFu;
}

#endif
