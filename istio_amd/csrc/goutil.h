// goutil.h -- Go 1.9 standard-library semantics the Mixer predicate path depends on, restated for
// the engine's host side (constant folding, batch pre-tables, error-message formatting).
//
//   strconv.ParseInt(s,10,64) / ParseFloat / Unquote   (used by expr.newConstant, expr.go:123-152)
//   time.ParseDuration                                (string literals -> DURATION, expr.go:143-146)
//   net.ParseIP, net.IP.Equal                         (externs.go:81-93)
//   time.Parse(time.RFC3339, s)                       (externs.go:95-102)
//   fmt "%v" of bag values                            (interpreterRun.go:469 error texts)
#pragma once

#include <cstdint>
#include <string>

namespace mxp {

bool go_parse_int10(const std::string& s, int64_t* out, std::string* err);
bool go_parse_float(const std::string& s, double* out, std::string* err);
// strconv.Unquote; returns false on "invalid syntax". Output is a Go byte string.
bool go_unquote(const std::string& lit, std::string* out);
bool go_parse_duration(const std::string& s, int64_t* out, std::string* err);

// net.ParseIP: true and the 16-byte form on success.
bool go_parse_ip(const uint8_t* s, size_t n, uint8_t out[16]);
// canonical form used for interning so that net.IP.Equal(a, b) <=> canon(a) == canon(b):
// 4-byte addresses become their 16-byte v4-in-v6 form; every other length is kept as is.
std::string ip_canonical(const uint8_t* b, size_t n);

bool go_parse_rfc3339(const uint8_t* s, size_t n, int64_t* sec, int32_t* nsec);

std::string go_format_float(double d);      // strconv.FormatFloat(d, 'g', -1, 64) == fmt %v
std::string go_format_duration(int64_t d);  // time.Duration.String()
std::string go_format_time_utc(int64_t sec, int32_t nsec);  // time.Time.String() in UTC
std::string go_format_bytes(const uint8_t* b, size_t n);    // fmt %v of []byte

}  // namespace mxp
