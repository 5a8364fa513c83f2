/*
 * ORACLE (test infrastructure only) -- the `matches` extern's regexp.MatchString for the C
 * interpreter, delegated to the Go regexp restatement in oracle/goregex.py through a callback that
 * oracle.py installs (one restatement, not two).  Without the callback: -2 (unsupported).
 */
#include "regex_oracle.h"

#include <stdio.h>

typedef int (*regex_fn)(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap);
static regex_fn g_fn = 0;

void oracle_set_regex_fn(regex_fn fn) { g_fn = fn; }

int oracle_regex_match(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap) {
    if (g_fn) return g_fn(pat, npat, s, n, err, errcap);
    snprintf(err, errcap, "oracle: regexp restatement not installed");
    return -2;
}
