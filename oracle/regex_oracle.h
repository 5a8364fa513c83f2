/*
 * ORACLE (test infrastructure only) -- Go `regexp` (RE2 syntax) restatement (oracle/goregex.c) used
 * by the `matches` extern (mixer/pkg/il/runtime/externs.go:118-120) and the regex list checker
 * (mixer/adapter/list/regexList.go:26-33).
 */
#ifndef MXP_ORACLE_REGEX_H
#define MXP_ORACLE_REGEX_H
#include <stddef.h>
#include <stdint.h>

typedef struct oracle_regex oracle_regex;

/* regexp.Compile: 0 ok, -1 syntax error (Go's "error parsing regexp: ..." text in err), -2 pattern
 * outside the restatement (Unicode classes, non-ASCII case folding; message in err). */
int oracle_regex_compile(const uint8_t* pat, size_t npat, oracle_regex** out, char* err, size_t errcap);
/* (*Regexp).MatchString on a compiled pattern: 1 match, 0 none */
int oracle_regex_exec(const oracle_regex* re, const uint8_t* s, size_t n);
void oracle_regex_free(oracle_regex* re);
/* regexp.MatchString(pattern, s): 1 match, 0 no match, -1 / -2 as oracle_regex_compile */
int oracle_regex_match(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap);
/* compiled-pattern cache of oracle_regex_match (default on); off = compile on every call, as
 * regexp.MatchString does (the CPU baseline) */
void oracle_regex_cache(int on);
/* regexList.checkList over n_sym symbols against n_pat patterns (blobs + offsets), OpenMP threads */
int oracle_regex_list_found(const uint8_t* pats, const uint64_t* pat_off, uint32_t n_pat, const uint8_t* syms,
                            const uint64_t* sym_off, uint32_t n_sym, int8_t* found, int threads, char* err,
                            size_t errcap);

#endif
