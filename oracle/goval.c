/*
 * ORACLE (test infrastructure only) -- Go 1.9 stdlib restatements for the interpreter oracle.
 * See goval.h.  Each function cites the Go source it restates.
 */
#include "goval.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- net.ParseIP (src/net/ip.go) */
#define IP_BIG 0xFFFFFF

static int dtoi(const uint8_t* s, size_t n, int* out, size_t* used) {
    int v = 0;
    size_t i = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        v = v * 10 + (s[i] - '0');
        if (v >= IP_BIG) { *out = IP_BIG; *used = i; return 0; }
    }
    if (i == 0) { *out = 0; *used = 0; return 0; }
    *out = v; *used = i; return 1;
}

static int xtoi(const uint8_t* s, size_t n, int* out, size_t* used) {
    int v = 0;
    size_t i = 0;
    for (; i < n; i++) {
        uint8_t c = s[i];
        if (c >= '0' && c <= '9') v = v * 16 + (c - '0');
        else if (c >= 'a' && c <= 'f') v = v * 16 + (c - 'a') + 10;
        else if (c >= 'A' && c <= 'F') v = v * 16 + (c - 'A') + 10;
        else break;
        if (v >= IP_BIG) { *out = 0; *used = i; return 0; }
    }
    if (i == 0) { *out = 0; *used = 0; return 0; }
    *out = v; *used = i; return 1;
}

static int parse_ipv4(const uint8_t* s, size_t n, uint8_t out[16]) {
    uint8_t p[4];
    for (int i = 0; i < 4; i++) {
        if (n == 0) return 0;
        if (i > 0) {
            if (s[0] != '.') return 0;
            s++; n--;
        }
        int v; size_t c;
        if (!dtoi(s, n, &v, &c) || v > 0xFF) return 0;
        s += c; n -= c;
        p[i] = (uint8_t)v;
    }
    if (n != 0) return 0;
    memset(out, 0, 10);
    out[10] = 0xff; out[11] = 0xff;
    memcpy(out + 12, p, 4);
    return 1;
}

static int parse_ipv6(const uint8_t* s, size_t n, uint8_t ip[16]) {
    memset(ip, 0, 16);
    int ellipsis = -1;
    if (n >= 2 && s[0] == ':' && s[1] == ':') {
        ellipsis = 0;
        s += 2; n -= 2;
        if (n == 0) return 1;
    }
    int i = 0;
    while (i < 16) {
        int v; size_t c;
        if (!xtoi(s, n, &v, &c) || v > 0xFFFF) return 0;
        if (c < n && s[c] == '.') {
            if (ellipsis < 0 && i != 16 - 4) return 0;
            if (i + 4 > 16) return 0;
            uint8_t ip4[16];
            if (!parse_ipv4(s, n, ip4)) return 0;
            ip[i] = ip4[12]; ip[i + 1] = ip4[13]; ip[i + 2] = ip4[14]; ip[i + 3] = ip4[15];
            n = 0;
            i += 4;
            break;
        }
        ip[i] = (uint8_t)(v >> 8);
        ip[i + 1] = (uint8_t)v;
        i += 2;
        s += c; n -= c;
        if (n == 0) break;
        if (s[0] != ':' || n == 1) return 0;
        s++; n--;
        if (s[0] == ':') {
            if (ellipsis >= 0) return 0;
            ellipsis = i;
            s++; n--;
            if (n == 0) break;
        }
    }
    if (n != 0) return 0;
    if (i < 16) {
        if (ellipsis < 0) return 0;
        int k = 16 - i;
        for (int j = i - 1; j >= ellipsis; j--) ip[j + k] = ip[j];
        for (int j = ellipsis + k - 1; j >= ellipsis; j--) ip[j] = 0;
    } else if (ellipsis >= 0) {
        return 0;
    }
    return 1;
}

int oracle_parse_ip(const uint8_t* s, size_t n, uint8_t out[16]) {
    for (size_t i = 0; i < n; i++) {
        if (s[i] == '.') return parse_ipv4(s, n, out) ? 16 : 0;
        if (s[i] == ':') return parse_ipv6(s, n, out) ? 16 : 0;
    }
    return 0;
}

static const uint8_t v4InV6Prefix[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff};

int oracle_parse_ipv4(const uint8_t* s, size_t n, uint8_t out[16]) { return parse_ipv4(s, n, out); }
int oracle_parse_ipv6(const uint8_t* s, size_t n, uint8_t out[16]) { return parse_ipv6(s, n, out); }
int oracle_dtoi(const uint8_t* s, size_t n, int* out, size_t* used) { return dtoi(s, n, out, used); }

int oracle_ip_equal(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
    if (na == nb) return na == 0 || memcmp(a, b, na) == 0;
    if (na == 4 && nb == 16) return memcmp(b, v4InV6Prefix, 12) == 0 && memcmp(a, b + 12, 4) == 0;
    if (na == 16 && nb == 4) return memcmp(a, v4InV6Prefix, 12) == 0 && memcmp(a + 12, b, 4) == 0;
    return 0;
}

/* ---------------------------------------------- time.Parse(RFC3339) (src/time/format.go, 1.9) */
static int is_digit_at(const uint8_t* s, size_t n, size_t i) { return i < n && s[i] >= '0' && s[i] <= '9'; }

/* time.leadingInt + time.atoi */
static int time_atoi(const uint8_t* s, size_t n, int64_t* out) {
    int neg = 0;
    if (n > 0 && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; s++; n--; }
    uint64_t x = 0;
    size_t i = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        if (x > (uint64_t)(INT64_MAX / 10)) return 0;
        x = x * 10 + (uint64_t)(s[i] - '0');
        if (x > (uint64_t)INT64_MAX) return 0;
    }
    if (i != n) return 0;
    *out = neg ? -(int64_t)x : (int64_t)x;
    return 1;
}

static int getnum(const uint8_t** s, size_t* n, int fixed, int* out) {
    if (!is_digit_at(*s, *n, 0)) return 0;
    if (!is_digit_at(*s, *n, 1)) {
        if (fixed) return 0;
        *out = (*s)[0] - '0';
        (*s)++; (*n)--;
        return 1;
    }
    *out = ((*s)[0] - '0') * 10 + ((*s)[1] - '0');
    (*s) += 2; (*n) -= 2;
    return 1;
}

static int is_leap(int64_t y) { return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0); }

static int days_in(int m, int64_t y) {
    static const int dm[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (m == 2 && is_leap(y)) return 29;
    return dm[m - 1];
}

/* days since 1970-01-01 of the civil date (proleptic Gregorian) */
static int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    int64_t era = (y >= 0 ? y : y - 399) / 400;
    int64_t yoe = y - era * 400;
    int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

int oracle_parse_rfc3339(const uint8_t* s, size_t n, int64_t* out_sec, int32_t* out_nsec) {
    int64_t year;
    int month, day, hour, minute, sec;
    int64_t nsec = 0;
    int64_t zone = 0;
    /* stdLongYear */
    if (n < 4 || !is_digit_at(s, n, 0)) return 0;
    if (!time_atoi(s, 4, &year)) return 0;
    s += 4; n -= 4;
    if (n < 1 || s[0] != '-') return 0;
    s++; n--;
    if (!getnum(&s, &n, 1, &month)) return 0;
    if (month <= 0 || 12 < month) return 0;
    if (n < 1 || s[0] != '-') return 0;
    s++; n--;
    if (!getnum(&s, &n, 1, &day)) return 0;
    if (n < 1 || s[0] != 'T') return 0;
    s++; n--;
    if (!getnum(&s, &n, 0, &hour)) return 0;
    if (hour < 0 || 24 <= hour) return 0;
    if (n < 1 || s[0] != ':') return 0;
    s++; n--;
    if (!getnum(&s, &n, 1, &minute)) return 0;
    if (minute < 0 || 60 <= minute) return 0;
    if (n < 1 || s[0] != ':') return 0;
    s++; n--;
    if (!getnum(&s, &n, 1, &sec)) return 0;
    if (sec < 0 || 60 <= sec) return 0;
    if (n >= 2 && s[0] == '.' && is_digit_at(s, n, 1)) {
        size_t k = 2;
        while (k < n && is_digit_at(s, n, k)) k++;
        int64_t ns;
        if (!time_atoi(s + 1, k - 1, &ns)) return 0;
        if (ns < 0 || ns >= 1000000000LL) return 0;
        for (int i = 0; i < 10 - (int)k; i++) ns *= 10;
        nsec = ns;
        s += k; n -= k;
    }
    /* stdISO8601ColonTZ */
    if (n >= 1 && s[0] == 'Z') {
        s++; n--;
    } else {
        if (n < 6) return 0;
        if (s[3] != ':') return 0;
        int64_t hr, mm;
        if (!time_atoi(s + 1, 2, &hr)) return 0;
        if (!time_atoi(s + 4, 2, &mm)) return 0;
        zone = (hr * 60 + mm) * 60;
        if (s[0] == '-') zone = -zone;
        else if (s[0] != '+') return 0;
        s += 6; n -= 6;
    }
    if (n != 0) return 0; /* extra text */
    if (day > days_in(month, year)) return 0;
    int64_t days = days_from_civil(year, month, 1) + (day - 1);
    *out_sec = days * 86400 + hour * 3600 + minute * 60 + sec - zone;
    *out_nsec = (int32_t)nsec;
    return 1;
}

/* ------------------------------------------------------------------------- fmt "%v" helpers */
static size_t put(char* buf, size_t cap, size_t w, const char* s, size_t n) {
    for (size_t i = 0; i < n && w + 1 < cap; i++) buf[w++] = s[i];
    if (w < cap) buf[w] = 0;
    return w;
}

/* strconv.FormatFloat(f, 'g', -1, 64) as used by fmt %v */
static size_t fmt_float(double d, char* buf, size_t cap) {
    char tmp[64];
    if (isnan(d)) return put(buf, cap, 0, "NaN", 3);
    if (isinf(d)) return put(buf, cap, 0, d > 0 ? "+Inf" : "-Inf", 4);
    if (d == 0) return put(buf, cap, 0, signbit(d) ? "-0" : "0", signbit(d) ? 2 : 1);
    int p;
    for (p = 0; p < 17; p++) {
        snprintf(tmp, sizeof tmp, "%.*e", p, d);
        if (strtod(tmp, NULL) == d) break;
    }
    /* tmp: [-]D[.DDD]e[+-]XX */
    char digs[32];
    int nd = 0, neg = 0;
    const char* q = tmp;
    if (*q == '-') { neg = 1; q++; }
    while (*q && *q != 'e') { if (*q != '.') digs[nd++] = *q; q++; }
    int exp = atoi(q + 1);
    while (nd > 1 && digs[nd - 1] == '0') nd--;
    size_t w = 0;
    if (neg) w = put(buf, cap, w, "-", 1);
    if (exp < -4 || exp >= 6) {
        w = put(buf, cap, w, digs, 1);
        if (nd > 1) { w = put(buf, cap, w, ".", 1); w = put(buf, cap, w, digs + 1, nd - 1); }
        char e[16];
        int ae = exp < 0 ? -exp : exp;
        int n = snprintf(e, sizeof e, "e%c%02d", exp < 0 ? '-' : '+', ae);
        return put(buf, cap, w, e, n);
    }
    int dp = exp + 1; /* digits before the decimal point */
    if (dp <= 0) {
        w = put(buf, cap, w, "0.", 2);
        for (int i = 0; i < -dp; i++) w = put(buf, cap, w, "0", 1);
        return put(buf, cap, w, digs, nd);
    }
    if (nd <= dp) {
        w = put(buf, cap, w, digs, nd);
        for (int i = nd; i < dp; i++) w = put(buf, cap, w, "0", 1);
        return w;
    }
    w = put(buf, cap, w, digs, dp);
    w = put(buf, cap, w, ".", 1);
    return put(buf, cap, w, digs + dp, nd - dp);
}

/* time.Duration.String() */
static size_t fmt_duration(int64_t d, char* out, size_t cap) {
    char buf[40];
    int w = sizeof buf;
    uint64_t u = (uint64_t)d;
    int neg = d < 0;
    if (neg) u = -u;
    if (u < 1000000000ULL) {
        int prec;
        buf[--w] = 's';
        w--;
        if (u == 0) return put(out, cap, 0, "0s", 2);
        if (u < 1000ULL) { prec = 0; buf[w] = 'n'; }
        else if (u < 1000000ULL) { prec = 3; w--; buf[w] = (char)0xC2; buf[w + 1] = (char)0xB5; }
        else { prec = 6; buf[w] = 'm'; }
        int print = 0;
        for (int i = 0; i < prec; i++) {
            int digit = (int)(u % 10);
            print = print || digit != 0;
            if (print) buf[--w] = (char)('0' + digit);
            u /= 10;
        }
        if (print) buf[--w] = '.';
        if (u == 0) buf[--w] = '0';
        while (u > 0) { buf[--w] = (char)('0' + u % 10); u /= 10; }
    } else {
        buf[--w] = 's';
        int print = 0;
        for (int i = 0; i < 9; i++) {
            int digit = (int)(u % 10);
            print = print || digit != 0;
            if (print) buf[--w] = (char)('0' + digit);
            u /= 10;
        }
        if (print) buf[--w] = '.';
        uint64_t v = u % 60;
        if (v == 0) buf[--w] = '0';
        while (v > 0) { buf[--w] = (char)('0' + v % 10); v /= 10; }
        u /= 60;
        if (u > 0) {
            buf[--w] = 'm';
            v = u % 60;
            if (v == 0) buf[--w] = '0';
            while (v > 0) { buf[--w] = (char)('0' + v % 10); v /= 10; }
            u /= 60;
            if (u > 0) {
                buf[--w] = 'h';
                while (u > 0) { buf[--w] = (char)('0' + u % 10); u /= 10; }
            }
        }
    }
    if (neg) buf[--w] = '-';
    return put(out, cap, 0, buf + w, sizeof buf - w);
}

static void civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
    z += 719468;
    int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    int64_t doe = z - era * 146097;
    int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t yy = yoe + era * 400;
    int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    int64_t mp = (5 * doy + 2) / 153;
    *d = (int)(doy - (153 * mp + 2) / 5 + 1);
    *m = (int)(mp < 10 ? mp + 3 : mp - 9);
    *y = yy + (*m <= 2);
}

size_t oracle_format_value(const gv* v, const mxp_bag_batch* b, char* buf, size_t cap) {
    char tmp[128];
    int n;
    switch (v->k) {
    case GV_STRING:
        return put(buf, cap, 0, (const char*)v->p, v->len);
    case GV_INT64:
        n = snprintf(tmp, sizeof tmp, "%lld", (long long)v->i);
        return put(buf, cap, 0, tmp, n);
    case GV_DOUBLE: {
        double d;
        memcpy(&d, &v->i, 8);
        return fmt_float(d, buf, cap);
    }
    case GV_BOOL:
        return put(buf, cap, 0, v->i ? "true" : "false", v->i ? 4 : 5);
    case GV_DURATION:
        return fmt_duration(v->i, buf, cap);
    case GV_TIME: {
        int64_t days = v->i >= 0 ? v->i / 86400 : -((-v->i + 86399) / 86400);
        int64_t rem = v->i - days * 86400;
        int64_t y;
        int m, d;
        civil_from_days(days, &y, &m, &d);
        n = snprintf(tmp, sizeof tmp, "%04lld-%02d-%02d %02d:%02d:%02d", (long long)y, m, d,
                     (int)(rem / 3600), (int)(rem / 60 % 60), (int)(rem % 60));
        size_t w = put(buf, cap, 0, tmp, n);
        if (v->ns) {
            char f[16];
            int k = snprintf(f, sizeof f, ".%09d", v->ns);
            while (k > 1 && f[k - 1] == '0') k--;
            w = put(buf, cap, w, f, k);
        }
        return put(buf, cap, w, " +0000 UTC", 10);
    }
    case GV_BYTES: {
        size_t w = put(buf, cap, 0, "[", 1);
        for (uint32_t i = 0; i < v->len; i++) {
            n = snprintf(tmp, sizeof tmp, i ? " %u" : "%u", v->p[i]);
            w = put(buf, cap, w, tmp, n);
        }
        return put(buf, cap, w, "]", 1);
    }
    case GV_MAP: {
        size_t w = put(buf, cap, 0, "map[", 4);
        if (b && v->i >= 0 && (uint64_t)v->i < b->n_maps) {
            for (uint64_t e = b->map_offsets[v->i]; e < b->map_offsets[v->i + 1]; e++) {
                uint32_t ks = b->map_keys[e], vs = b->map_values[e];
                if (e != b->map_offsets[v->i]) w = put(buf, cap, w, " ", 1);
                w = put(buf, cap, w, (const char*)b->str_bytes + b->str_offsets[ks],
                        b->str_offsets[ks + 1] - b->str_offsets[ks]);
                w = put(buf, cap, w, ":", 1);
                w = put(buf, cap, w, (const char*)b->str_bytes + b->str_offsets[vs],
                        b->str_offsets[vs + 1] - b->str_offsets[vs]);
            }
        }
        return put(buf, cap, w, "]", 1);
    }
    case GV_OTHER:
        if (b && v->i >= 0 && (uint64_t)v->i < b->n_strings)
            return put(buf, cap, 0, (const char*)b->str_bytes + b->str_offsets[v->i],
                       b->str_offsets[v->i + 1] - b->str_offsets[v->i]);
        return put(buf, cap, 0, "?", 1);
    default:
        return put(buf, cap, 0, "<nil>", 5);
    }
}
