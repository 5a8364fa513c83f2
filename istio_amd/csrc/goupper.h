// goupper.h -- Go 1.9 strings.ToUpper for case-insensitive lists, host and device.
//
// The reference upper-cases list entries and every looked-up symbol with strings.ToUpper
// (mixer/adapter/list/stringList.go:59,66,79).  In Go 1.9 that is strings.Map(unicode.ToUpper, s):
//   * runes are read as `for i, c := range s` decodes them (an invalid byte is U+FFFD, width 1);
//   * while no rune has changed, the output is the input's bytes (an invalid byte stays as it is);
//   * from the first rune whose upper case differs, every rune is re-encoded with utf8.EncodeRune,
//     so an invalid byte after that point becomes U+FFFD's three bytes EF BF BD;
//   * unicode.ToUpper: 'a'..'z' for ASCII, above it the CaseRanges simple uppercase mapping of
//     Unicode 9.0.0 (upper_table.h, tools/gen_upper_table.py).
// The mapped string can be shorter or longer than the input, so it is produced as a byte stream and
// consumed 8 bytes at a time by the list hash and the entry compare (lists.hip) or collected into a
// string (lists.cpp).
#pragma once

#include <stdint.h>

#include "netparse.h"  // MXP_NHD
#include "upper_table.h"

// unicode.ToUpper(r) (Go 1.9 src/unicode/letter.go: ToUpper, to) over the rows {lo, hi, delta}
MXP_NHD uint32_t mxp_go_upper_rune(const uint32_t (*rows)[3], uint32_t r) {
    if (r < 0x80u) return r - 0x61u < 26u ? r - 32u : r;
    int a = 0, b = (int)MXP_UPPER_N - 1;
    while (a <= b) {
        const int m = (a + b) >> 1;
        if (rows[m][0] > r) {
            b = m - 1;
        } else if (rows[m][1] < r) {
            a = m + 1;
        } else {
            const uint32_t lo = rows[m][0], d = rows[m][2];
            return d == MXP_UPPER_ALT ? lo + ((r - lo) & ~1u) : r + d;
        }
    }
    return r;
}

// utf8.DecodeRuneInString at s[i] (Go 1.9 unicode/utf8 accept ranges): the rune and its width;
// an invalid or truncated sequence is U+FFFD of width 1
MXP_NHD uint32_t mxp_go_decode(const uint8_t* s, uint32_t i, uint32_t n, uint32_t* width) {
    const uint32_t c0 = s[i];
    *width = 1;
    if (c0 < 0x80u) return c0;
    const uint32_t left = n - i;
    if (c0 >= 0xC2u && c0 <= 0xDFu) {
        if (left >= 2) {
            const uint32_t b1 = s[i + 1];
            if (b1 >= 0x80u && b1 <= 0xBFu) {
                *width = 2;
                return ((c0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
            }
        }
    } else if (c0 >= 0xE0u && c0 <= 0xEFu) {
        if (left >= 3) {
            const uint32_t b1 = s[i + 1], b2 = s[i + 2];
            const uint32_t lo = c0 == 0xE0u ? 0xA0u : 0x80u, hi = c0 == 0xEDu ? 0x9Fu : 0xBFu;
            if (b1 >= lo && b1 <= hi && b2 >= 0x80u && b2 <= 0xBFu) {
                *width = 3;
                return ((c0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
            }
        }
    } else if (c0 >= 0xF0u && c0 <= 0xF4u) {
        if (left >= 4) {
            const uint32_t b1 = s[i + 1], b2 = s[i + 2], b3 = s[i + 3];
            const uint32_t lo = c0 == 0xF0u ? 0x90u : 0x80u, hi = c0 == 0xF4u ? 0x8Fu : 0xBFu;
            if (b1 >= lo && b1 <= hi && b2 >= 0x80u && b2 <= 0xBFu && b3 >= 0x80u && b3 <= 0xBFu) {
                *width = 4;
                return ((c0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
            }
        }
    }
    return 0xFFFDu;
}

// utf8.EncodeRune: the bytes of r, little-endian in a word, and their count
MXP_NHD uint32_t mxp_go_encode(uint32_t r, uint32_t* bytes) {
    if (r < 0x80u) {
        *bytes = r;
        return 1;
    }
    if (r < 0x800u) {
        *bytes = (0xC0u | (r >> 6)) | (0x80u | (r & 0x3Fu)) << 8;
        return 2;
    }
    if (r < 0x10000u) {
        *bytes = (0xE0u | (r >> 12)) | (0x80u | ((r >> 6) & 0x3Fu)) << 8 | (0x80u | (r & 0x3Fu)) << 16;
        return 3;
    }
    *bytes = (0xF0u | (r >> 18)) | (0x80u | ((r >> 12) & 0x3Fu)) << 8 | (0x80u | ((r >> 6) & 0x3Fu)) << 16 |
             (0x80u | (r & 0x3Fu)) << 24;
    return 4;
}

// strings.ToUpper(s) as a byte stream (Go 1.9 strings.Map with unicode.ToUpper).  The reference
// builds with Go 1.9 (bin/verify_go_version.sh:24-25, DOCKER_BUILDER istio/ci:go1.9 in
// bin/envsetup.sh:38).  Go 1.9's Map encodes every mapped rune after the first change with
// utf8.EncodeRune, so U+0080 stays C2 80 here.  The single-byte write of runes <= utf8.RuneSelf
// (which turned U+0080 into a lone 0x80 byte) arrived with the Go 1.10 rewrite of Map and was
// fixed again in Go 1.11; it is not the reference's behaviour.  Checked: U+0080 case.
struct MxpUpperStream {
    const uint8_t* s;
    uint32_t n, i;
    const uint32_t (*rows)[3];
    uint32_t pend, npend;  // bytes of the current rune not yet handed out (little-endian)
    bool changed;          // some rune has changed: re-encode from here on

    MXP_NHD MxpUpperStream(const uint8_t* s_, uint32_t n_, const uint32_t (*rows_)[3])
        : s(s_), n(n_), i(0), rows(rows_), pend(0), npend(0), changed(false) {}

    // refill pend from the next rune; false at the end of the input
    MXP_NHD bool refill() {
        if (i >= n) return false;
        uint32_t w;
        const uint32_t c = mxp_go_decode(s, i, n, &w);
        const uint32_t u = mxp_go_upper_rune(rows, c);
        if (!changed && u == c) {  // the input's own bytes (an invalid byte included)
            pend = 0;
            for (uint32_t k = 0; k < w; k++) pend |= (uint32_t)s[i + k] << (8u * k);
            npend = w;
        } else {
            changed = true;
            npend = mxp_go_encode(u, &pend);
        }
        i += w;
        return true;
    }

    // the next 8 output bytes, little-endian, zero past the end; returns how many are real
    MXP_NHD uint32_t next8(uint64_t* word) {
        uint64_t x = 0;
        uint32_t k = 0;
        while (k < 8u) {
            if (!npend && !refill()) break;
            x |= (uint64_t)(pend & 0xFFu) << (8u * k);
            pend >>= 8;
            npend--;
            k++;
        }
        *word = x;
        return k;
    }
};
