/*
 * ORACLE (test infrastructure only) -- Go value model and Go stdlib restatements used by the C
 * interpreter restatement in il_interp.c.  Never linked into the product (istio_amd/).
 *
 *   net.ParseIP / IP.Equal / IP.To4 (Go 1.9 src/net/ip.go)    -> oracle_parse_ip, oracle_ip_equal
 *   time.Parse(time.RFC3339, s) (Go 1.9 src/time/format.go)    -> oracle_parse_rfc3339
 *   fmt "%v" of the value kinds a bag can hold                  -> oracle_format_value
 */
#ifndef MXP_ORACLE_GOVAL_H
#define MXP_ORACLE_GOVAL_H

#include <stddef.h>
#include <stdint.h>

#include "../include/mxp_batch.h"

/* dynamic kinds of interpreter heap values (an interface{} in the reference) */
enum gv_kind {
    GV_NIL = 0,
    GV_STRING = 1,
    GV_INT64 = 2,
    GV_DOUBLE = 3,
    GV_BOOL = 4,
    GV_DURATION = 5,
    GV_TIME = 6,
    GV_BYTES = 7,
    GV_MAP = 8,
    GV_OTHER = 9
};

typedef struct gv {
    uint8_t k;
    uint8_t inl_used;
    uint32_t len;          /* string / bytes length                 */
    const uint8_t* p;      /* string / bytes data (may point at inl) */
    int64_t i;             /* int64, duration, bool, time sec, map id, other string id */
    int32_t ns;            /* time nanoseconds                       */
    uint8_t inl[16];       /* storage for ip() results               */
} gv;

/* net.ParseIP: returns 16 on success (16-byte form), 0 on failure. */
int oracle_parse_ip(const uint8_t* s, size_t n, uint8_t out[16]);
/* parseIPv4 / parseIPv6 (zone not allowed) / dtoi of src/net/ip.go, as ParseCIDR calls them */
int oracle_parse_ipv4(const uint8_t* s, size_t n, uint8_t out[16]);
int oracle_parse_ipv6(const uint8_t* s, size_t n, uint8_t out[16]);
int oracle_dtoi(const uint8_t* s, size_t n, int* out, size_t* used);
/* net.IP.Equal */
int oracle_ip_equal(const uint8_t* a, size_t na, const uint8_t* b, size_t nb);
/* time.Parse(time.RFC3339, s): returns 1 and the instant on success. */
int oracle_parse_rfc3339(const uint8_t* s, size_t n, int64_t* sec, int32_t* nsec);
/* fmt.Sprintf("%v", v) into buf (truncated to cap-1); returns length written. */
size_t oracle_format_value(const gv* v, const mxp_bag_batch* b, char* buf, size_t cap);

#endif
