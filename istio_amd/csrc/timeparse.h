// timeparse.h -- Go 1.9 time.Parse(time.RFC3339, s) restated for host and device (src/time/
// format.go: Parse with the RFC3339 layout "2006-01-02T15:04:05Z07:00": 4-digit year, 2-digit
// month / day / minute / second, 1-or-2-digit hour, optional fractional seconds, 'Z' or +hh:mm).
// The host's timestamp() pre-tables (goutil.cpp go_parse_rfc3339) and the device packer
// (pack.hip) parse through this one definition.
#pragma once

#include <stdint.h>

#include "netparse.h"  // MXP_NHD

namespace mxptime {

MXP_NHD bool digit(const uint8_t* s, uint64_t n, uint64_t i) { return i < n && s[i] >= '0' && s[i] <= '9'; }

// strconv.Atoi over exactly n bytes (optional sign), int64 range
MXP_NHD bool tatoi(const uint8_t* s, uint64_t n, int64_t* out) {
    bool neg = false;
    if (n && (s[0] == '-' || s[0] == '+')) {
        neg = s[0] == '-';
        s++;
        n--;
    }
    const uint64_t kMax = 0x7FFFFFFFFFFFFFFFull;
    uint64_t x = 0;
    uint64_t i = 0;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        if (x > kMax / 10) return false;
        x = x * 10 + (uint64_t)(s[i] - '0');
        if (x > kMax) return false;
    }
    if (i != n) return false;
    *out = neg ? -(int64_t)x : (int64_t)x;
    return true;
}

// getnum: two digits (fixed) or one or two
MXP_NHD bool num2(const uint8_t*& s, uint64_t& n, bool fixed, int* out) {
    if (!digit(s, n, 0)) return false;
    if (!digit(s, n, 1)) {
        if (fixed) return false;
        *out = s[0] - '0';
        s++;
        n--;
        return true;
    }
    *out = (s[0] - '0') * 10 + (s[1] - '0');
    s += 2;
    n -= 2;
    return true;
}

MXP_NHD bool lit(const uint8_t*& s, uint64_t& n, char c) {
    if (!n || s[0] != (uint8_t)c) return false;
    s++;
    n--;
    return true;
}

MXP_NHD int64_t civil_days(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    return era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
}

// -> true with Unix seconds and nanoseconds (UTC)
MXP_NHD bool parse_rfc3339(const uint8_t* s, uint64_t n, int64_t* sec_out, int32_t* nsec_out) {
    int64_t year;
    int mon, day, hh, mm, ss;
    int64_t nsec = 0, zone = 0;
    if (n < 4 || !digit(s, n, 0) || !tatoi(s, 4, &year)) return false;
    s += 4;
    n -= 4;
    if (!lit(s, n, '-') || !num2(s, n, true, &mon) || mon < 1 || mon > 12) return false;
    if (!lit(s, n, '-') || !num2(s, n, true, &day)) return false;
    if (!lit(s, n, 'T') || !num2(s, n, false, &hh) || hh >= 24) return false;
    if (!lit(s, n, ':') || !num2(s, n, true, &mm) || mm >= 60) return false;
    if (!lit(s, n, ':') || !num2(s, n, true, &ss) || ss >= 60) return false;
    if (n >= 2 && s[0] == '.' && digit(s, n, 1)) {
        uint64_t k = 2;
        while (digit(s, n, k)) k++;
        int64_t f;
        if (!tatoi(s + 1, k - 1, &f) || f < 0 || f >= 1000000000LL) return false;
        for (int i = 0; i < 10 - (int)k; i++) f *= 10;
        nsec = f;
        s += k;
        n -= k;
    }
    if (n && s[0] == 'Z') {
        s++;
        n--;
    } else {
        if (n < 6 || s[3] != ':') return false;
        int64_t zh, zm;
        if (!tatoi(s + 1, 2, &zh) || !tatoi(s + 4, 2, &zm)) return false;
        zone = (zh * 60 + zm) * 60;
        if (s[0] == '-') zone = -zone;
        else if (s[0] != '+') return false;
        s += 6;
        n -= 6;
    }
    if (n) return false;
    const int dim[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    const int maxd = dim[mon - 1] + (mon == 2 && (year % 4 == 0 && (year % 100 != 0 || year % 400 == 0)));
    if (day > maxd) return false;
    const int64_t days = civil_days(year, mon, 1) + (day - 1);
    *sec_out = days * 86400 + hh * 3600 + mm * 60 + ss - zone;
    *nsec_out = (int32_t)nsec;
    return true;
}

}  // namespace mxptime
