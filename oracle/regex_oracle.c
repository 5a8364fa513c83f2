/*
 * ORACLE (test infrastructure only) -- placeholder for the Go regexp restatement.
 * Returns -2 ("unsupported") until the RE2-syntax engine lands; parity tests skip such pairs.
 */
#include "regex_oracle.h"

#include <stdio.h>

int oracle_regex_match(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap) {
    (void)pat; (void)npat; (void)s; (void)n;
    snprintf(err, errcap, "oracle: regexp not yet restated");
    return -2;
}
