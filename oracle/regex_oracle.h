/*
 * ORACLE (test infrastructure only) -- Go `regexp` (RE2 syntax) restatement used by the
 * `matches` extern (mixer/pkg/il/runtime/externs.go:118-120) and the regex list checker
 * (mixer/adapter/list/regexList.go:26-33).
 */
#ifndef MXP_ORACLE_REGEX_H
#define MXP_ORACLE_REGEX_H
#include <stddef.h>
#include <stdint.h>

/* regexp.MatchString(pattern, s): 1 match, 0 no match, -1 compile error (message in err),
 * -2 pattern outside the restatement (message in err). */
int oracle_regex_match(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap);
/* installs the implementation (oracle.py: goregex.py via a ctypes callback) */
void oracle_set_regex_fn(int (*fn)(const uint8_t*, size_t, const uint8_t*, size_t, char*, size_t));

#endif
