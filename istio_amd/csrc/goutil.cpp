// goutil.cpp -- see goutil.h.  Algorithms follow the Go 1.9 standard library sources named there.
#include "goutil.h"
#include "netparse.h"
#include "timeparse.h"

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace mxp {

static constexpr int64_t kMaxI64 = INT64_MAX;

bool go_parse_int10(const std::string& s, int64_t* out, std::string* err) {
    auto syntax = [&] {
        if (err) *err = "strconv.ParseInt: parsing \"" + s + "\": invalid syntax";
        return false;
    };
    if (s.empty()) return syntax();
    size_t i = 0;
    bool neg = false;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
    }
    if (i >= s.size()) return syntax();
    unsigned __int128 v = 0;
    for (; i < s.size(); i++) {
        if (s[i] < '0' || s[i] > '9') return syntax();
        v = v * 10 + (unsigned)(s[i] - '0');
        if (v > (unsigned __int128)kMaxI64 + 1) v = (unsigned __int128)kMaxI64 + 2;  // saturate
    }
    if ((!neg && v > (unsigned __int128)kMaxI64) || (neg && v > (unsigned __int128)kMaxI64 + 1)) {
        if (err) *err = "strconv.ParseInt: parsing \"" + s + "\": value out of range";
        return false;
    }
    *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
    return true;
}

bool go_parse_float(const std::string& s, double* out, std::string* err) {
    char* end = nullptr;
    errno = 0;
    double d = strtod(s.c_str(), &end);
    if (end == s.c_str() || *end != 0) {
        if (err) *err = "strconv.ParseFloat: parsing \"" + s + "\": invalid syntax";
        return false;
    }
    if (std::isinf(d)) {
        if (err) *err = "strconv.ParseFloat: parsing \"" + s + "\": value out of range";
        return false;
    }
    *out = d;
    return true;
}

static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static void put_utf8(std::string& o, uint32_t r) {
    if (r < 0x80) {
        o.push_back((char)r);
    } else if (r < 0x800) {
        o.push_back((char)(0xC0 | (r >> 6)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    } else if (r < 0x10000) {
        o.push_back((char)(0xE0 | (r >> 12)));
        o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    } else {
        o.push_back((char)(0xF0 | (r >> 18)));
        o.push_back((char)(0x80 | ((r >> 12) & 0x3F)));
        o.push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (r & 0x3F)));
    }
}

static size_t utf8_len_at(const std::string& s, size_t i) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) return 1;
    if ((c >> 5) == 6) return 2;
    if ((c >> 4) == 14) return 3;
    if ((c >> 3) == 30) return 4;
    return 1;
}

bool go_unquote(const std::string& lit, std::string* out) {
    size_t n = lit.size();
    if (n < 2) return false;
    char q = lit[0];
    if (q != lit[n - 1]) return false;
    std::string body = lit.substr(1, n - 2);
    if (q == '`') {
        if (body.find('`') != std::string::npos) return false;
        std::string o;
        for (char c : body)
            if (c != '\r') o.push_back(c);
        *out = o;
        return true;
    }
    if (q != '"' && q != '\'') return false;
    if (body.find('\n') != std::string::npos) return false;
    std::string o;
    size_t runes = 0;
    size_t i = 0;
    while (i < body.size()) {
        char c = body[i];
        if (c == q) return false;
        if (c != '\\') {
            size_t l = utf8_len_at(body, i);
            o.append(body, i, l);
            i += l;
            runes++;
        } else {
            if (i + 1 >= body.size()) return false;
            char e = body[i + 1];
            i += 2;
            switch (e) {
            case 'a': o.push_back('\a'); break;
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            case 'n': o.push_back('\n'); break;
            case 'r': o.push_back('\r'); break;
            case 't': o.push_back('\t'); break;
            case 'v': o.push_back('\v'); break;
            case '\\': o.push_back('\\'); break;
            case '\'': case '"':
                if (e != q) return false;
                o.push_back(e);
                break;
            case 'x': case 'u': case 'U': {
                int k = e == 'x' ? 2 : e == 'u' ? 4 : 8;
                if (i + k > body.size()) return false;
                uint32_t v = 0;
                for (int j = 0; j < k; j++) {
                    int h = hexval(body[i + j]);
                    if (h < 0) return false;
                    v = v * 16 + (uint32_t)h;
                }
                i += k;
                if (e == 'x') {
                    o.push_back((char)v);
                } else {
                    if (v > 0x10FFFF || (v >= 0xD800 && v < 0xE000)) return false;
                    put_utf8(o, v);
                }
                break;
            }
            default:
                if (e >= '0' && e <= '7') {
                    if (i + 2 > body.size()) return false;
                    uint32_t v = (uint32_t)(e - '0');
                    for (int j = 0; j < 2; j++) {
                        char d = body[i + j];
                        if (d < '0' || d > '7') return false;
                        v = v * 8 + (uint32_t)(d - '0');
                    }
                    if (v > 255) return false;
                    i += 2;
                    o.push_back((char)v);
                } else {
                    return false;
                }
            }
            runes++;
        }
        if (q == '\'' && runes > 1) return false;
    }
    if (q == '\'' && runes != 1) return false;
    *out = o;
    return true;
}

bool go_parse_duration(const std::string& orig, int64_t* out, std::string* err) {
    auto invalid = [&](const std::string& m) {
        if (err) *err = m;
        return false;
    };
    const std::string bad = "time: invalid duration " + orig;
    size_t p = 0, n = orig.size();
    bool neg = false;
    if (p < n && (orig[p] == '-' || orig[p] == '+')) {
        neg = orig[p] == '-';
        p++;
    }
    if (orig.compare(p, std::string::npos, "0") == 0) {
        *out = 0;
        return true;
    }
    if (p == n) return invalid(bad);
    int64_t d = 0;
    while (p < n) {
        char c = orig[p];
        if (!(c == '.' || (c >= '0' && c <= '9'))) return invalid(bad);
        size_t start = p;
        int64_t v = 0;
        while (p < n && orig[p] >= '0' && orig[p] <= '9') {
            if (v > kMaxI64 / 10) return invalid(bad);
            v = v * 10 + (orig[p] - '0');
            if (v < 0) return invalid(bad);
            p++;
        }
        bool pre = p != start;
        bool post = false;
        int64_t f = 0;
        double scale = 1;
        if (p < n && orig[p] == '.') {
            p++;
            size_t fs = p;
            bool overflow = false;
            while (p < n && orig[p] >= '0' && orig[p] <= '9') {
                if (!overflow) {
                    if (f > kMaxI64 / 10) {
                        overflow = true;
                    } else {
                        int64_t y = f * 10 + (orig[p] - '0');
                        if (y < 0) overflow = true;
                        else {
                            f = y;
                            scale *= 10;
                        }
                    }
                }
                p++;
            }
            post = p != fs;
        }
        if (!pre && !post) return invalid(bad);
        size_t us = p;
        while (p < n && !(orig[p] == '.' || (orig[p] >= '0' && orig[p] <= '9'))) p++;
        if (p == us) return invalid("time: missing unit in duration " + orig);
        std::string u = orig.substr(us, p - us);
        int64_t unit;
        if (u == "ns") unit = 1;
        else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000;
        else if (u == "ms") unit = 1000000;
        else if (u == "s") unit = 1000000000LL;
        else if (u == "m") unit = 60LL * 1000000000LL;
        else if (u == "h") unit = 3600LL * 1000000000LL;
        else return invalid("time: unknown unit " + u + " in duration " + orig);
        if (v > kMaxI64 / unit) return invalid(bad);
        v *= unit;
        if (f > 0) {
            v = (int64_t)((uint64_t)v + (uint64_t)(int64_t)((double)f * ((double)unit / scale)));
            if (v < 0) return invalid(bad);
        }
        d = (int64_t)((uint64_t)d + (uint64_t)v);
        if (d < 0) return invalid(bad);
    }
    *out = neg ? -d : d;
    return true;
}

// ------------------------------------------------------------------------------- net.ParseIP
bool go_parse_ip(const uint8_t* s, size_t n, uint8_t out[16]) {
    return n < (1u << 31) && mxpnet::parse_ip(s, (uint32_t)n, out);
}

std::string ip_canonical(const uint8_t* b, size_t n) {
    if (n == 4) {
        std::string o(12, '\0');
        o[10] = (char)0xff;
        o[11] = (char)0xff;
        o.append((const char*)b, 4);
        return o;
    }
    return std::string((const char*)b, n);
}

// ------------------------------------------------------------------------ time.Parse(RFC3339)
bool go_parse_rfc3339(const uint8_t* s, size_t n, int64_t* sec_out, int32_t* nsec_out) {
    return mxptime::parse_rfc3339(s, (uint64_t)n, sec_out, nsec_out);
}

// ---------------------------------------------------------------------------- formatting
std::string go_format_float(double d) {
    if (std::isnan(d)) return "NaN";
    if (std::isinf(d)) return d > 0 ? "+Inf" : "-Inf";
    if (d == 0) return std::signbit(d) ? "-0" : "0";
    char tmp[64];
    for (int p = 0; p < 17; p++) {
        snprintf(tmp, sizeof tmp, "%.*e", p, d);
        if (strtod(tmp, nullptr) == d) break;
    }
    std::string digs;
    bool neg = false;
    const char* q = tmp;
    if (*q == '-') {
        neg = true;
        q++;
    }
    for (; *q && *q != 'e'; q++)
        if (*q != '.') digs.push_back(*q);
    int exp = atoi(q + 1);
    while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
    std::string o = neg ? "-" : "";
    if (exp < -4 || exp >= 6) {
        o += digs[0];
        if (digs.size() > 1) o += "." + digs.substr(1);
        snprintf(tmp, sizeof tmp, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
        return o + tmp;
    }
    int dp = exp + 1;
    if (dp <= 0) return o + "0." + std::string(-dp, '0') + digs;
    if ((int)digs.size() <= dp) return o + digs + std::string(dp - digs.size(), '0');
    return o + digs.substr(0, dp) + "." + digs.substr(dp);
}

std::string go_format_duration(int64_t d) {
    uint64_t u = (uint64_t)d;
    bool neg = d < 0;
    if (neg) u = 0 - u;
    std::string tail;  // built in reverse
    auto frac = [&](int prec) {
        bool printed = false;
        for (int i = 0; i < prec; i++) {
            int dig = (int)(u % 10);
            printed = printed || dig != 0;
            if (printed) tail.push_back((char)('0' + dig));
            u /= 10;
        }
        if (printed) tail.push_back('.');
    };
    auto integer = [&](uint64_t v) {
        if (v == 0) tail.push_back('0');
        while (v) {
            tail.push_back((char)('0' + v % 10));
            v /= 10;
        }
    };
    if (u < 1000000000ULL) {
        if (u == 0) return "0s";
        tail.push_back('s');
        int prec;
        if (u < 1000ULL) {
            prec = 0;
            tail.push_back('n');
        } else if (u < 1000000ULL) {
            prec = 3;
            tail.push_back((char)0xB5);
            tail.push_back((char)0xC2);
        } else {
            prec = 6;
            tail.push_back('m');
        }
        frac(prec);
        integer(u);
    } else {
        tail.push_back('s');
        frac(9);
        integer(u % 60);
        u /= 60;
        if (u) {
            tail.push_back('m');
            integer(u % 60);
            u /= 60;
            if (u) {
                tail.push_back('h');
                integer(u);
            }
        }
    }
    if (neg) tail.push_back('-');
    return std::string(tail.rbegin(), tail.rend());
}

std::string go_format_time_utc(int64_t sec, int32_t nsec) {
    int64_t days = sec >= 0 ? sec / 86400 : -((-sec + 86399) / 86400);
    int64_t rem = sec - days * 86400;
    int64_t z = days + 719468;
    int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    int64_t doe = z - era * 146097;
    int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    int64_t mp = (5 * doy + 2) / 153;
    int d = (int)(doy - (153 * mp + 2) / 5 + 1);
    int m = (int)(mp < 10 ? mp + 3 : mp - 9);
    int64_t y = yoe + era * 400 + (m <= 2);
    char buf[96];
    int k = snprintf(buf, sizeof buf, "%04lld-%02d-%02d %02d:%02d:%02d", (long long)y, m, d, (int)(rem / 3600),
                     (int)(rem / 60 % 60), (int)(rem % 60));
    std::string o(buf, k);
    if (nsec) {
        k = snprintf(buf, sizeof buf, ".%09d", nsec);
        while (k > 1 && buf[k - 1] == '0') k--;
        o.append(buf, k);
    }
    return o + " +0000 UTC";
}

std::string go_format_bytes(const uint8_t* b, size_t n) {
    std::string o = "[";
    for (size_t i = 0; i < n; i++) {
        if (i) o += " ";
        o += std::to_string((unsigned)b[i]);
    }
    return o + "]";
}

}  // namespace mxp
