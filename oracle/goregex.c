/*
 * ORACLE (test infrastructure only) -- Go's regexp.MatchString (RE2 syntax) restated in C: the
 * `matches` extern (mixer/pkg/il/runtime/externs.go:118-120: regexp.MatchString(pattern, str) --
 * compile, then an unanchored search) and the regex list checker (mixer/adapter/list/regexList.go:
 * 26-65).  Function for function the C form of oracle/goregex.py (same parse.go semantics, error
 * codes and texts, Pike-VM match over Go's UTF-8 decoding and empty-width assertions), so the C
 * interpreter and the CPU baseline run a compiled regexp engine instead of calling back into Python.
 * tests/test_regex_oracle.py checks it against goregex.py (KATs, error texts, random patterns).
 *
 * Go 1.9 regexp/syntax is not vendored under /root/reference; PARITY UNPINNED beyond the
 * reference's own rows (tests.go:2064-2121, list_test.go:397-431).  Unicode classes (\p, \P) and
 * simple case folding read oracle/unicode_tables.h (tools/gen_unicode_tables.py, Unicode 13 where
 * Go 1.9 has Unicode 9).
 */
#include "regex_oracle.h"

#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "unicode_tables.h"

#define MAX_REPEAT 1000
#define MAX_RUNE 0x10FFFFu

/* empty-width assertions (syntax.EmptyOp) */
enum { BEGIN_LINE = 1, END_LINE = 2, BEGIN_TEXT = 4, END_TEXT = 8, WORD_B = 16, NO_WORD_B = 32 };

typedef struct {
    uint32_t lo, hi;
} rrange;

typedef struct {
    rrange* r;
    int n, cap;
} ranges;

/* ---------------------------------------------------------------------------- arena + errors */
typedef struct {
    void** blocks;
    int n, cap;
    jmp_buf jb;
    int code;           /* -1 syntax error, -2 unsupported */
    char msg[600];
} ctx;

static void* cx_alloc(ctx* c, size_t sz) {
    void* p = calloc(1, sz ? sz : 1);
    if (!p) abort();
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 64;
        c->blocks = (void**)realloc(c->blocks, c->cap * sizeof(void*));
    }
    c->blocks[c->n++] = p;
    return p;
}

static void cx_free(ctx* c) {
    for (int i = 0; i < c->n; i++) free(c->blocks[i]);
    free(c->blocks);
    c->blocks = NULL;
    c->n = c->cap = 0;
}

/* syntax.Error: "error parsing regexp: <code>: `<expr>`" */
static void fail_syntax(ctx* c, const char* code, const uint8_t* e, size_t n) {
    int k = snprintf(c->msg, sizeof c->msg, "error parsing regexp: %s: `", code);
    if (k < 0) k = 0;
    size_t room = sizeof c->msg - (size_t)k - 2;
    if (n > room) n = room;
    memcpy(c->msg + k, e, n);
    c->msg[k + n] = '`';
    c->msg[k + n + 1] = 0;
    c->code = -1;
    longjmp(c->jb, 1);
}

#define E_RANGE "invalid character class range"
#define E_ESCAPE "invalid escape sequence"
#define E_NAMED "invalid named capture"
#define E_PERL "invalid or unsupported Perl syntax"
#define E_REPEAT_OP "invalid nested repetition operator"
#define E_REPEAT_SIZE "invalid repeat count"
#define E_UTF8 "invalid UTF-8"
#define E_BRACKET "missing closing ]"
#define E_PAREN "missing closing )"
#define E_REPEAT_ARG "missing argument to repetition operator"
#define E_BACKSLASH "trailing backslash at end of expression"
#define E_UNEXPECTED_PAREN "unexpected )"

/* ---------------------------------------------------------------------------- runes */
/* utf8.DecodeRune: invalid -> (U+FFFD, 1) */
static uint32_t decode_rune(const uint8_t* b, size_t n, size_t i, int* w) {
    const uint32_t c = b[i];
    const size_t left = n - i;
    *w = 1;
    if (c < 0x80) return c;
    if (c >= 0xC2 && c <= 0xDF && left >= 2 && b[i + 1] >= 0x80 && b[i + 1] <= 0xBF) {
        *w = 2;
        return ((c & 0x1Fu) << 6) | (b[i + 1] & 0x3Fu);
    }
    if (c >= 0xE0 && c <= 0xEF && left >= 3) {
        const uint32_t lo = c == 0xE0 ? 0xA0 : 0x80, hi = c == 0xED ? 0x9F : 0xBF;
        if (b[i + 1] >= lo && b[i + 1] <= hi && b[i + 2] >= 0x80 && b[i + 2] <= 0xBF) {
            *w = 3;
            return ((c & 0x0Fu) << 12) | ((b[i + 1] & 0x3Fu) << 6) | (b[i + 2] & 0x3Fu);
        }
    }
    if (c >= 0xF0 && c <= 0xF4 && left >= 4) {
        const uint32_t lo = c == 0xF0 ? 0x90 : 0x80, hi = c == 0xF4 ? 0x8F : 0xBF;
        if (b[i + 1] >= lo && b[i + 1] <= hi && b[i + 2] >= 0x80 && b[i + 2] <= 0xBF && b[i + 3] >= 0x80 &&
            b[i + 3] <= 0xBF) {
            *w = 4;
            return ((c & 0x07u) << 18) | ((b[i + 1] & 0x3Fu) << 12) | ((b[i + 2] & 0x3Fu) << 6) | (b[i + 3] & 0x3Fu);
        }
    }
    return 0xFFFD;
}

static int is_word(int64_t r) {
    return r >= 0 && ((r >= 0x30 && r <= 0x39) || (r >= 0x41 && r <= 0x5A) || (r >= 0x61 && r <= 0x7A) || r == 0x5F);
}

/* ---------------------------------------------------------------------------- rune ranges */
static void rg_add(ctx* c, ranges* g, uint32_t lo, uint32_t hi) {
    if (g->n == g->cap) {
        int cap = g->cap ? 2 * g->cap : 8;
        rrange* r = (rrange*)cx_alloc(c, cap * sizeof(rrange));
        if (g->n) memcpy(r, g->r, g->n * sizeof(rrange));
        g->r = r;
        g->cap = cap;
    }
    g->r[g->n].lo = lo;
    g->r[g->n].hi = hi;
    g->n++;
}

static int rr_cmp(const void* a, const void* b) {
    const rrange *x = (const rrange*)a, *y = (const rrange*)b;
    if (x->lo != y->lo) return x->lo < y->lo ? -1 : 1;
    return x->hi < y->hi ? -1 : x->hi > y->hi;
}

/* norm: sorted, merged (adjacent ranges join) */
static ranges rg_norm(ctx* c, ranges g) {
    ranges out = {0};
    if (!g.n) return out;
    rrange* t = (rrange*)cx_alloc(c, g.n * sizeof(rrange));
    int k = 0;
    for (int i = 0; i < g.n; i++)
        if (g.r[i].lo <= g.r[i].hi) t[k++] = g.r[i];
    qsort(t, k, sizeof(rrange), rr_cmp);
    for (int i = 0; i < k; i++) {
        if (out.n && t[i].lo <= out.r[out.n - 1].hi + 1) {
            if (t[i].hi > out.r[out.n - 1].hi) out.r[out.n - 1].hi = t[i].hi;
        } else {
            rg_add(c, &out, t[i].lo, t[i].hi);
        }
    }
    return out;
}

static ranges rg_negate(ctx* c, ranges g) {
    ranges n = rg_norm(c, g), out = {0};
    uint32_t nxt = 0;
    for (int i = 0; i < n.n; i++) {
        if (n.r[i].lo > nxt) rg_add(c, &out, nxt, n.r[i].lo - 1);
        nxt = n.r[i].hi + 1;
    }
    if (nxt <= MAX_RUNE) rg_add(c, &out, nxt, MAX_RUNE);
    return out;
}

static void rg_extend(ctx* c, ranges* dst, ranges src) {
    for (int i = 0; i < src.n; i++) rg_add(c, dst, src.r[i].lo, src.r[i].hi);
}

/* unicode.SimpleFold over kUniFold: the next rune of r's orbit (r itself when r does not fold) */
static uint32_t simple_fold(uint32_t r) {
    int a = 0, b = (int)(sizeof kUniFold / sizeof kUniFold[0]) - 1;
    while (a <= b) {
        const int m = (a + b) / 2;
        if (kUniFold[m][0] == r) return kUniFold[m][1];
        if (kUniFold[m][0] < r) a = m + 1;
        else b = m - 1;
    }
    return r;
}

/* fold_orbit(r) -> number of runes written (r first) */
static int fold_orbit(uint32_t r, uint32_t out[8]) {
    int k = 0;
    out[k++] = r;
    for (uint32_t x = simple_fold(r); x != r && k < 8; x = simple_fold(x)) out[k++] = x;
    return k;
}

static int rg_contains(ranges g, uint32_t r) {  /* g normalised */
    int a = 0, b = g.n - 1;
    while (a <= b) {
        const int m = (a + b) / 2;
        if (r < g.r[m].lo) b = m - 1;
        else if (r > g.r[m].hi) a = m + 1;
        else return 1;
    }
    return 0;
}

/* appendFoldedRange over every range: the class closed under simple case folding */
static ranges fold_ranges(ctx* c, ranges g) {
    ranges n = rg_norm(c, g), out = {0};
    rg_extend(c, &out, n);
    for (size_t t = 0; t < sizeof kUniFold / sizeof kUniFold[0]; t++)
        if (rg_contains(n, kUniFold[t][0]))
            for (uint32_t x = kUniFold[t][1]; x != kUniFold[t][0]; x = simple_fold(x)) rg_add(c, &out, x, x);
    return rg_norm(c, out);
}

/* appendGroup: under (?i) a group is folded BEFORE it is negated */
static ranges group_ranges(int fi, ctx* c, ranges g, int negated) {
    if (fi) g = fold_ranges(c, g);
    return negated ? rg_negate(c, g) : rg_norm(c, g);
}

/* ---------------------------------------------------------------------------- AST */
enum { N_LIT, N_CLASS, N_ANY, N_ANYNL, N_EMPTY, N_CAT, N_ALT, N_STAR, N_PLUS, N_QUEST, N_REP, N_GROUP };

typedef struct node {
    int k;
    uint32_t rune;   /* N_LIT */
    int op;          /* N_EMPTY */
    ranges cls;      /* N_CLASS */
    struct node** sub; /* N_CAT / N_ALT */
    int nsub, capsub;
    struct node* a;  /* N_STAR / PLUS / QUEST / REP / GROUP */
    int lo, hi;      /* N_REP */
} node;

static node* mk(ctx* c, int k) {
    node* n = (node*)cx_alloc(c, sizeof(node));
    n->k = k;
    return n;
}

static void push(ctx* c, node* seq, node* x) {
    if (seq->nsub == seq->capsub) {
        int cap = seq->capsub ? 2 * seq->capsub : 8;
        node** s = (node**)cx_alloc(c, cap * sizeof(node*));
        if (seq->nsub) memcpy(s, seq->sub, seq->nsub * sizeof(node*));
        seq->sub = s;
        seq->capsub = cap;
    }
    seq->sub[seq->nsub++] = x;
}

typedef struct {
    ctx* c;
    const uint8_t* s;
    size_t n, i;
    int fi, fm, fs, fU;  /* flags i m s U */
} parser;

static int full_rune_ok(const uint8_t* b, size_t n, size_t i) {
    int w;
    const uint32_t r = decode_rune(b, n, i, &w);
    if (!(r == 0xFFFD && w == 1)) return 1;
    return n - i >= 3 && b[i] == 0xEF && b[i + 1] == 0xBF && b[i + 2] == 0xBD;
}

static uint32_t next_rune(parser* p) {
    if (!full_rune_ok(p->s, p->n, p->i)) fail_syntax(p->c, E_UTF8, p->s + p->i, p->n - p->i);
    int w;
    const uint32_t r = decode_rune(p->s, p->n, p->i, &w);
    p->i += w;
    return r;
}

static node* parse_alt(parser* p, int top);

static node* lit(parser* p, uint32_t r) {
    if (p->fi) {
        uint32_t orbit[8];
        const int k = fold_orbit(r, orbit);
        if (k > 1) {
            node* n = mk(p->c, N_CLASS);
            ranges g = {0};
            for (int j = 0; j < k; j++) rg_add(p->c, &g, orbit[j], orbit[j]);
            n->cls = rg_norm(p->c, g);
            return n;
        }
    }
    node* n = mk(p->c, N_LIT);
    n->rune = r;
    return n;
}

static int hexval(uint32_t d) {
    if (d >= '0' && d <= '9') return (int)(d - '0');
    if (d >= 'a' && d <= 'f') return (int)(d - 'a' + 10);
    if (d >= 'A' && d <= 'F') return (int)(d - 'A' + 10);
    return -1;
}

/* {n} {n,} {n,m} at p->i -> 1 with *lo, *hi (-1 = no max) and advance, else 0 (literal '{') */
static int num_at(parser* p, size_t j, int* v, size_t* end) {
    size_t k = j;
    while (k < p->n && p->s[k] >= '0' && p->s[k] <= '9') k++;
    if (k == j) return 0;
    if (k - j > 1 && p->s[j] == '0') return 0;  /* leading zeros */
    long x = 0;
    for (size_t t = j; t < k; t++) {
        x = x * 10 + (p->s[t] - '0');
        if (x > MAX_REPEAT + 1) x = MAX_REPEAT + 1;
    }
    *v = (int)x;
    *end = k;
    return 1;
}

static int try_repeat(parser* p, int* lo, int* hi) {
    size_t j = p->i + 1, e;
    if (!num_at(p, j, lo, &e)) return 0;
    j = e;
    if (j < p->n && p->s[j] == ',') {
        j++;
        if (j < p->n && p->s[j] == '}') {
            *hi = -1;
        } else {
            if (!num_at(p, j, hi, &e)) return 0;
            j = e;
        }
    } else {
        *hi = *lo;
    }
    if (j >= p->n || p->s[j] != '}') return 0;
    j++;
    const size_t start = p->i;
    p->i = j;
    if (*lo > MAX_REPEAT || *hi > MAX_REPEAT || (*hi >= 0 && *lo > *hi))
        fail_syntax(p->c, E_REPEAT_SIZE, p->s + start, j - start);
    return 1;
}

static void repeat(parser* p, node* seq, int op, size_t start, int lo, int hi) {
    if (seq->nsub == 0) fail_syntax(p->c, E_REPEAT_ARG, p->s + start, p->i - start);
    if (p->i < p->n && p->s[p->i] == '?') p->i++;  /* lazy form: irrelevant for a boolean match */
    if (p->i < p->n && (p->s[p->i] == '*' || p->s[p->i] == '+' || p->s[p->i] == '?'))
        fail_syntax(p->c, E_REPEAT_OP, p->s + start, p->i + 1 - start);
    if (p->i < p->n && p->s[p->i] == '{') {
        const size_t save = p->i;
        int a, b;
        if (try_repeat(p, &a, &b)) fail_syntax(p->c, E_REPEAT_OP, p->s + start, p->i - start);
        p->i = save;
    }
    node* prev = seq->sub[--seq->nsub];
    node* n = mk(p->c, op);
    n->a = prev;
    n->lo = lo;
    n->hi = hi;
    push(p->c, seq, n);
}

static ranges perl_class_ranges(ctx* c, char cl) {
    ranges g = {0};
    switch (cl) {
    case 'd': rg_add(c, &g, 0x30, 0x39); break;
    case 's': rg_add(c, &g, 0x09, 0x0A); rg_add(c, &g, 0x0C, 0x0D); rg_add(c, &g, 0x20, 0x20); break;
    default:  /* w */
        rg_add(c, &g, 0x30, 0x39); rg_add(c, &g, 0x41, 0x5A); rg_add(c, &g, 0x5F, 0x5F); rg_add(c, &g, 0x61, 0x7A);
        break;
    }
    return g;
}

static int valid_utf8(const uint8_t* b, size_t n) {  /* checkUTF8 */
    for (size_t i = 0; i < n;) {
        if (!full_rune_ok(b, n, i)) return 0;
        int w;
        decode_rune(b, n, i, &w);
        i += (size_t)w;
    }
    return 1;
}

/* unicodeTable (parse.go): "Any", unicode.Categories, unicode.Scripts -> 1 with *out, else 0 */
static int unicode_table(ctx* c, const uint8_t* name, size_t nl, ranges* out) {
    ranges g = {0};
    if (nl == 3 && memcmp(name, "Any", 3) == 0) {
        rg_add(c, &g, 0, MAX_RUNE);
        *out = g;
        return 1;
    }
    int a = 0, b = (int)(sizeof kUniClasses / sizeof kUniClasses[0]) - 1;
    while (a <= b) {
        const int m = (a + b) / 2;
        const char* k = kUniClasses[m].name;
        const size_t kl = strlen(k);
        int d = memcmp(k, name, kl < nl ? kl : nl);
        if (d == 0) d = kl < nl ? -1 : kl > nl;
        if (d == 0) {
            for (uint32_t t = 0; t < kUniClasses[m].n; t++)
                rg_add(c, &g, kUniRanges[kUniClasses[m].off + t][0], kUniRanges[kUniClasses[m].off + t][1]);
            *out = g;
            return 1;
        }
        if (d < 0) a = m + 1;
        else b = m - 1;
    }
    return 0;
}

/* parseUnicodeClass: \pN \p{Name} \P.. \p{^Name} at p->i ('\') -> the group's ranges */
static ranges unicode_class(parser* p) {
    const size_t start = p->i;
    int neg = p->s[p->i + 1] == 'P';
    p->i += 2;
    const uint8_t* name;
    size_t nl, seq_end;
    if (p->i < p->n && p->s[p->i] == '{') {
        size_t end = p->n;
        for (size_t k = p->i; k < p->n; k++)
            if (p->s[k] == '}') {
                end = k;
                break;
            }
        if (end == p->n) {
            if (!valid_utf8(p->s + start, p->n - start)) fail_syntax(p->c, E_UTF8, p->s + start, p->n - start);
            fail_syntax(p->c, E_RANGE, p->s + start, p->n - start);
        }
        name = p->s + p->i + 1;
        nl = end - (p->i + 1);
        if (!valid_utf8(name, nl)) fail_syntax(p->c, E_UTF8, name, nl);
        seq_end = end + 1;
    } else if (p->i < p->n) {
        if (!full_rune_ok(p->s, p->n, p->i)) fail_syntax(p->c, E_UTF8, p->s + p->i, p->n - p->i);
        int w;
        decode_rune(p->s, p->n, p->i, &w);
        name = p->s + p->i;
        nl = (size_t)w;
        seq_end = p->i + (size_t)w;
    } else {
        name = p->s + p->i;
        nl = 0;
        seq_end = p->i;
    }
    p->i = seq_end;
    if (nl && name[0] == '^') {
        neg = !neg;
        name++;
        nl--;
    }
    ranges tab;
    if (!nl || !unicode_table(p->c, name, nl, &tab)) fail_syntax(p->c, E_RANGE, p->s + start, seq_end - start);
    return group_ranges(p->fi, p->c, tab, neg);
}

/* parsePerlClassEscape (\d \s \w and negations) or parseUnicodeClass (\p \P) at p->i -> 1 with *out */
static int perl_class(parser* p, ranges* out) {
    if (p->i + 1 < p->n && p->s[p->i] == '\\') {
        const char c = (char)p->s[p->i + 1];
        if (c && strchr("dswDSW", c)) {
            p->i += 2;
            *out = group_ranges(p->fi, p->c, perl_class_ranges(p->c, (char)(c | 0x20)), c >= 'A' && c <= 'Z');
            return 1;
        }
        if (c == 'p' || c == 'P') {
            *out = unicode_class(p);
            return 1;
        }
    }
    return 0;
}

/* parseEscape: one escaped rune at p->i ('\') */
static uint32_t parse_escape(parser* p) {
    const size_t start = p->i;
    p->i++;
    if (p->i >= p->n) fail_syntax(p->c, E_BACKSLASH, (const uint8_t*)"", 0);
    const uint32_t c = next_rune(p);
#define FAIL_ESC() fail_syntax(p->c, E_ESCAPE, p->s + start, p->i - start)
    const int alnum = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
    if (c < 0x80 && !alnum) return c;
    if (c >= '1' && c <= '7') {
        if (p->i >= p->n || !(p->s[p->i] >= '0' && p->s[p->i] <= '7')) FAIL_ESC();
    }
    if (c >= '0' && c <= '7') {
        uint32_t r = c - '0';
        for (int t = 0; t < 2; t++)
            if (p->i < p->n && p->s[p->i] >= '0' && p->s[p->i] <= '7') {
                r = r * 8 + (p->s[p->i] - '0');
                p->i++;
            }
        return r;
    }
    if (c == 'x') {
        if (p->i >= p->n) FAIL_ESC();
        const uint32_t c2 = next_rune(p);
        if (c2 == '{') {
            int nhex = 0;
            uint32_t r = 0;
            for (;;) {
                if (p->i >= p->n) FAIL_ESC();
                const uint32_t d = next_rune(p);
                if (d == '}') break;
                const int v = d < 0x80 ? hexval(d) : -1;
                if (v < 0) FAIL_ESC();
                r = r * 16 + (uint32_t)v;
                if (r > MAX_RUNE) FAIL_ESC();
                nhex++;
            }
            if (nhex == 0) FAIL_ESC();
            return r;
        }
        const int x = c2 < 0x80 ? hexval(c2) : -1;
        const uint32_t c3 = p->i < p->n ? next_rune(p) : 0xFFFD;
        const int y = c3 < 0x80 ? hexval(c3) : -1;
        if (x < 0 || y < 0) FAIL_ESC();
        return (uint32_t)(x * 16 + y);
    }
    switch (c) {
    case 'a': return 7;
    case 'f': return 12;
    case 'n': return 10;
    case 'r': return 13;
    case 't': return 9;
    case 'v': return 11;
    default: break;
    }
    FAIL_ESC();
#undef FAIL_ESC
    return 0;
}

static uint32_t class_char(parser* p, size_t class_start) {
    if (p->i >= p->n) fail_syntax(p->c, E_BRACKET, p->s + class_start, p->n - class_start);
    if (p->s[p->i] == '\\') return parse_escape(p);
    return next_rune(p);
}

static const struct {
    const char* name;
    uint32_t r[4][2];
    int n;
} kPosix[] = {
    {"alnum", {{0x30, 0x39}, {0x41, 0x5A}, {0x61, 0x7A}}, 3},
    {"alpha", {{0x41, 0x5A}, {0x61, 0x7A}}, 2},
    {"ascii", {{0x00, 0x7F}}, 1},
    {"blank", {{0x09, 0x09}, {0x20, 0x20}}, 2},
    {"cntrl", {{0x00, 0x1F}, {0x7F, 0x7F}}, 2},
    {"digit", {{0x30, 0x39}}, 1},
    {"graph", {{0x21, 0x7E}}, 1},
    {"lower", {{0x61, 0x7A}}, 1},
    {"print", {{0x20, 0x7E}}, 1},
    {"punct", {{0x21, 0x2F}, {0x3A, 0x40}, {0x5B, 0x60}, {0x7B, 0x7E}}, 4},
    {"space", {{0x09, 0x0D}, {0x20, 0x20}}, 2},
    {"upper", {{0x41, 0x5A}}, 1},
    {"word", {{0x30, 0x39}, {0x41, 0x5A}, {0x5F, 0x5F}, {0x61, 0x7A}}, 4},
    {"xdigit", {{0x30, 0x39}, {0x41, 0x46}, {0x61, 0x66}}, 3},
};

static ranges parse_class(parser* p) {
    const size_t start = p->i;
    p->i++;
    int neg = 0;
    if (p->i < p->n && p->s[p->i] == '^') {
        neg = 1;
        p->i++;
    }
    ranges g = {0};
    int first = 1;
    for (;;) {
        if (p->i >= p->n) fail_syntax(p->c, E_BRACKET, p->s + start, p->n - start);
        const uint8_t c = p->s[p->i];
        if (c == ']' && !first) {
            p->i++;
            break;
        }
        if (c == '[' && p->i + 1 < p->n && p->s[p->i + 1] == ':') {  /* POSIX class */
            const uint8_t* end = NULL;
            for (size_t k = p->i + 2; k + 1 < p->n; k++)
                if (p->s[k] == ':' && p->s[k + 1] == ']') {
                    end = p->s + k;
                    break;
                }
            if (end) {
                const uint8_t* nm = p->s + p->i + 2;
                size_t nl = (size_t)(end - nm);
                int pneg = nl > 0 && nm[0] == '^';
                if (pneg) {
                    nm++;
                    nl--;
                }
                int found = -1;
                for (size_t t = 0; t < sizeof kPosix / sizeof kPosix[0]; t++)
                    if (strlen(kPosix[t].name) == nl && memcmp(kPosix[t].name, nm, nl) == 0) found = (int)t;
                if (found < 0) fail_syntax(p->c, E_RANGE, p->s + p->i, (size_t)(end + 2 - (p->s + p->i)));
                ranges pr = {0};
                for (int t = 0; t < kPosix[found].n; t++) rg_add(p->c, &pr, kPosix[found].r[t][0], kPosix[found].r[t][1]);
                rg_extend(p->c, &g, group_ranges(p->fi, p->c, pr, pneg));
                p->i = (size_t)(end + 2 - p->s);
                first = 0;
                continue;
            }
        }
        ranges pc;
        if (perl_class(p, &pc)) {
            rg_extend(p->c, &g, pc);
            first = 0;
            continue;
        }
        const size_t rstart = p->i;
        const uint32_t lo = class_char(p, start);
        if (p->i + 1 < p->n && p->s[p->i] == '-' && p->s[p->i + 1] != ']') {
            p->i++;
            const uint32_t hi = class_char(p, start);
            if (hi < lo) fail_syntax(p->c, E_RANGE, p->s + rstart, p->i - rstart);
            rg_add(p->c, &g, lo, hi);
        } else {
            rg_add(p->c, &g, lo, lo);
        }
        first = 0;
    }
    if (p->fi) g = fold_ranges(p->c, g);
    g = rg_norm(p->c, g);
    return neg ? rg_negate(p->c, g) : g;
}

static void parse_escape_atom(parser* p, node* seq) {
    if (p->i + 1 < p->n) {
        const uint8_t c = p->s[p->i + 1];
        if (c == 'A' || c == 'z' || c == 'b' || c == 'B') {
            p->i += 2;
            node* n = mk(p->c, N_EMPTY);
            n->op = c == 'A' ? BEGIN_TEXT : c == 'z' ? END_TEXT : c == 'b' ? WORD_B : NO_WORD_B;
            push(p->c, seq, n);
            return;
        }
        if (c == 'C') fail_syntax(p->c, E_ESCAPE, (const uint8_t*)"\\C", 2);
        if (c == 'Q') {
            p->i += 2;
            size_t end = p->n, stop;
            for (size_t k = p->i; k + 1 < p->n; k++)
                if (p->s[k] == '\\' && p->s[k + 1] == 'E') {
                    end = k;
                    break;
                }
            stop = end;
            while (p->i < stop) push(p->c, seq, lit(p, next_rune(p)));
            p->i = end == p->n ? p->n : end + 2;
            return;
        }
    }
    ranges g;
    if (perl_class(p, &g)) {
        node* n = mk(p->c, N_CLASS);
        n->cls = g;
        push(p->c, seq, n);
        return;
    }
    push(p->c, seq, lit(p, parse_escape(p)));
}

static void parse_group(parser* p, node* seq) {
    const size_t start = p->i;
    const uint8_t* s = p->s;
    if (p->i + 1 < p->n && s[p->i + 1] == '?') {
        if (p->i + 3 < p->n && s[p->i + 2] == 'P' && s[p->i + 3] == '<') {  /* (?P<name>re) */
            size_t end = p->n;
            for (size_t k = p->i + 4; k < p->n; k++)
                if (s[k] == '>') {
                    end = k;
                    break;
                }
            if (end == p->n) fail_syntax(p->c, E_NAMED, s + start, p->n - start);
            const size_t nl = end - (p->i + 4);
            int ok = nl > 0;
            for (size_t k = p->i + 4; k < end; k++) ok &= is_word(s[k]);
            if (!ok) fail_syntax(p->c, E_NAMED, s + start, end + 1 - start);
            p->i = end + 1;
            node* g = mk(p->c, N_GROUP);
            g->a = parse_alt(p, 0);
            push(p->c, seq, g);
            return;
        }
        size_t j = p->i + 2;
        int sign = 1, neg = 0, seen = 0;
        int nf[4] = {p->fi, p->fm, p->fs, p->fU};
        for (;;) {
            if (j >= p->n) fail_syntax(p->c, E_PERL, s + start, p->n - start);
            const uint8_t c = s[j++];
            if (c == 'i' || c == 'm' || c == 's' || c == 'U') {
                nf[c == 'i' ? 0 : c == 'm' ? 1 : c == 's' ? 2 : 3] = sign;
                seen = 1;
            } else if (c == '-') {
                if (neg) fail_syntax(p->c, E_PERL, s + start, j - start);
                neg = 1;
                sign = 0;
                seen = 0;
            } else if (c == ':' || c == ')') {
                if (neg && !seen) fail_syntax(p->c, E_PERL, s + start, j - start);
                if (c == ')') {  /* (?flags): the rest of the current group */
                    p->fi = nf[0];
                    p->fm = nf[1];
                    p->fs = nf[2];
                    p->fU = nf[3];
                    p->i = j;
                    return;
                }
                const int of[4] = {p->fi, p->fm, p->fs, p->fU};
                p->fi = nf[0];
                p->fm = nf[1];
                p->fs = nf[2];
                p->fU = nf[3];
                p->i = j;
                node* g = mk(p->c, N_GROUP);
                g->a = parse_alt(p, 0);
                push(p->c, seq, g);
                p->fi = of[0];
                p->fm = of[1];
                p->fs = of[2];
                p->fU = of[3];
                return;
            } else {
                fail_syntax(p->c, E_PERL, s + start, j - start);
            }
        }
    }
    p->i++;
    node* g = mk(p->c, N_GROUP);
    g->a = parse_alt(p, 0);
    push(p->c, seq, g);
}

static void parse_piece(parser* p, node* seq) {
    const size_t start = p->i;
    const uint8_t c = p->s[p->i];
    if (c == '*' || c == '+' || c == '?') {
        p->i++;
        repeat(p, seq, c == '*' ? N_STAR : c == '+' ? N_PLUS : N_QUEST, start, 0, 0);
        return;
    }
    if (c == '{') {
        int lo, hi;
        if (try_repeat(p, &lo, &hi)) {
            repeat(p, seq, N_REP, start, lo, hi);
            return;
        }
        p->i++;
        push(p->c, seq, lit(p, '{'));
        return;
    }
    if (c == '(') {
        parse_group(p, seq);
        return;
    }
    if (c == '[') {
        node* n = mk(p->c, N_CLASS);
        n->cls = parse_class(p);
        push(p->c, seq, n);
        return;
    }
    if (c == '.') {
        p->i++;
        push(p->c, seq, mk(p->c, p->fs ? N_ANY : N_ANYNL));
        return;
    }
    if (c == '^' || c == '$') {
        p->i++;
        node* n = mk(p->c, N_EMPTY);
        n->op = c == '^' ? (p->fm ? BEGIN_LINE : BEGIN_TEXT) : (p->fm ? END_LINE : END_TEXT);
        push(p->c, seq, n);
        return;
    }
    if (c == '\\') {
        parse_escape_atom(p, seq);
        return;
    }
    push(p->c, seq, lit(p, next_rune(p)));
}

static node* parse_alt(parser* p, int top) {
    node* alt = mk(p->c, N_ALT);
    node* cur = mk(p->c, N_CAT);
    push(p->c, alt, cur);
    const int saved[4] = {p->fi, p->fm, p->fs, p->fU};
    while (p->i < p->n) {
        const uint8_t c = p->s[p->i];
        if (c == '|') {
            p->i++;
            cur = mk(p->c, N_CAT);
            push(p->c, alt, cur);
            continue;
        }
        if (c == ')') {
            if (top) fail_syntax(p->c, E_UNEXPECTED_PAREN, p->s, p->n);
            break;
        }
        parse_piece(p, cur);
    }
    if (!top) {
        if (p->i >= p->n) fail_syntax(p->c, E_PAREN, p->s, p->n);
        p->i++;  /* ')' */
        p->fi = saved[0];
        p->fm = saved[1];
        p->fs = saved[2];
        p->fU = saved[3];
    }
    return alt->nsub == 1 ? alt->sub[0] : alt;
}

/* ---------------------------------------------------------------------------- program (Pike VM) */
enum { I_RUNE, I_SPLIT, I_EMPTY, I_MATCH };

typedef struct {
    int op;
    int x, y;       /* split: x, y; rune / empty: next = x */
    int arg;        /* empty: op */
    int r0, nr;     /* rune: ranges [r0, r0 + nr) of prog.rr */
} inst;

struct oracle_regex {
    inst* ins;
    int n, cap;
    rrange* rr;
    int nrr, caprr;
    int start;
};

static int emit(oracle_regex* p, inst x) {
    if (p->n == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 64;
        p->ins = (inst*)realloc(p->ins, p->cap * sizeof(inst));
    }
    p->ins[p->n] = x;
    return p->n++;
}

static int emit_rune(oracle_regex* p, const rrange* r, int nr, int next) {
    if (p->nrr + nr > p->caprr) {
        while (p->nrr + nr > p->caprr) p->caprr = p->caprr ? 2 * p->caprr : 64;
        p->rr = (rrange*)realloc(p->rr, p->caprr * sizeof(rrange));
    }
    memcpy(p->rr + p->nrr, r, nr * sizeof(rrange));
    inst x = {I_RUNE, next, 0, 0, p->nrr, nr};
    p->nrr += nr;
    return emit(p, x);
}

/* compile node n so that it continues at `nxt`; returns its entry pc */
static int compile_node(oracle_regex* p, const node* n, int nxt) {
    switch (n->k) {
    case N_LIT: {
        rrange r = {n->rune, n->rune};
        return emit_rune(p, &r, 1, nxt);
    }
    case N_CLASS: return emit_rune(p, n->cls.r, n->cls.n, nxt);
    case N_ANY: {
        rrange r = {0, MAX_RUNE};
        return emit_rune(p, &r, 1, nxt);
    }
    case N_ANYNL: {
        rrange r[2] = {{0, 9}, {11, MAX_RUNE}};
        return emit_rune(p, r, 2, nxt);
    }
    case N_EMPTY: {
        inst x = {I_EMPTY, nxt, 0, n->op, 0, 0};
        return emit(p, x);
    }
    case N_GROUP: return compile_node(p, n->a, nxt);
    case N_CAT: {
        int pc = nxt;
        for (int k = n->nsub - 1; k >= 0; k--) pc = compile_node(p, n->sub[k], pc);
        return pc;
    }
    case N_ALT: {
        int* e = (int*)malloc(n->nsub * sizeof(int));
        for (int k = 0; k < n->nsub; k++) e[k] = compile_node(p, n->sub[k], nxt);
        int pc = e[n->nsub - 1];
        for (int k = n->nsub - 2; k >= 0; k--) {
            inst x = {I_SPLIT, e[k], pc, 0, 0, 0};
            pc = emit(p, x);
        }
        free(e);
        return pc;
    }
    case N_QUEST: {
        const int body = compile_node(p, n->a, nxt);
        inst x = {I_SPLIT, body, nxt, 0, 0, 0};
        return emit(p, x);
    }
    case N_STAR: {
        inst x = {I_SPLIT, -1, nxt, 0, 0, 0};
        const int loop = emit(p, x);
        const int body = compile_node(p, n->a, loop);
        p->ins[loop].x = body;
        return loop;
    }
    case N_PLUS: {
        inst x = {I_SPLIT, -1, nxt, 0, 0, 0};
        const int loop = emit(p, x);
        const int body = compile_node(p, n->a, loop);
        p->ins[loop].x = body;
        return body;
    }
    case N_REP: {
        int pc = nxt;
        if (n->hi < 0) {
            node star = *n;
            star.k = N_STAR;
            pc = compile_node(p, &star, pc);
        } else {
            for (int t = 0; t < n->hi - n->lo; t++) {
                const int body = compile_node(p, n->a, pc);
                inst x = {I_SPLIT, body, pc, 0, 0, 0};
                pc = emit(p, x);
            }
        }
        for (int t = 0; t < n->lo; t++) pc = compile_node(p, n->a, pc);
        return pc;
    }
    default: return nxt;
    }
}

void oracle_regex_free(oracle_regex* r) {
    if (!r) return;
    free(r->ins);
    free(r->rr);
    free(r);
}

/* regexp.Compile: 0 ok (*out), -1 syntax error / -2 unsupported (message in err) */
int oracle_regex_compile(const uint8_t* pat, size_t npat, oracle_regex** out, char* err, size_t errcap) {
    ctx c;
    memset(&c, 0, sizeof c);
    oracle_regex* prog = (oracle_regex*)calloc(1, sizeof(oracle_regex));
    *out = NULL;
    if (setjmp(c.jb)) {
        if (err && errcap) {
            size_t k = strlen(c.msg);
            if (k > errcap - 1) k = errcap - 1;
            memcpy(err, c.msg, k);
            err[k] = 0;
        }
        const int code = c.code;
        cx_free(&c);
        oracle_regex_free(prog);
        return code;
    }
    parser p = {&c, pat ? pat : (const uint8_t*)"", pat ? npat : 0, 0, 0, 0, 0, 0};
    node* ast = parse_alt(&p, 1);
    inst m = {I_MATCH, 0, 0, 0, 0, 0};
    const int match = emit(prog, m);
    prog->start = compile_node(prog, ast, match);
    cx_free(&c);
    *out = prog;
    return 0;
}

static int empty_flags(int64_t prev, int64_t nxt) {
    int f = 0;
    if (prev < 0) f |= BEGIN_TEXT | BEGIN_LINE;
    else if (prev == 10) f |= BEGIN_LINE;
    if (nxt < 0) f |= END_TEXT | END_LINE;
    else if (nxt == 10) f |= END_LINE;
    f |= is_word(prev) != is_word(nxt) ? WORD_B : NO_WORD_B;
    return f;
}

typedef struct {
    int* dense;
    int* sparse;
    int n;
} sset;

static void add_thread(const oracle_regex* p, sset* cur, int pc, int flags, int* stack) {
    int sp = 0;
    stack[sp++] = pc;
    while (sp) {
        pc = stack[--sp];
        const unsigned k = (unsigned)cur->sparse[pc];
        if (k < (unsigned)cur->n && cur->dense[k] == pc) continue;  /* seen */
        cur->sparse[pc] = cur->n;
        cur->dense[cur->n++] = pc;
        const inst* x = &p->ins[pc];
        if (x->op == I_SPLIT) {
            stack[sp++] = x->y;
            stack[sp++] = x->x;
        } else if (x->op == I_EMPTY) {
            if ((x->arg & flags) == x->arg) stack[sp++] = x->x;
        }
    }
}

/* regexp.(*Regexp).MatchString: unanchored search, any match */
int oracle_regex_exec(const oracle_regex* p, const uint8_t* s, size_t n) {
    const int N = p->n;
    /* thread set (dense / sparse), the closure stack (a split pushes two: <= 2N + 1) and the list of
     * threads that consumed the current rune */
    int* mem = (int*)malloc(sizeof(int) * ((size_t)N * 5 + 16));
    sset a = {mem, mem + N, 0};
    int* stack = mem + 2 * N;
    int* clist = mem + 4 * N + 8;
    int nclist = 0;
    sset* cur = &a;
    size_t i = 0;
    int64_t prev = -1;
    int result = 0;
    for (;;) {
        int64_t nxt = -1;
        int w = 0;
        if (i < n) nxt = decode_rune(s, n, i, &w);
        const int flags = empty_flags(prev, nxt);
        cur->n = 0;
        for (int k = 0; k < nclist; k++) add_thread(p, cur, clist[k], flags, stack);
        add_thread(p, cur, p->start, flags, stack);
        for (int k = 0; k < cur->n; k++)
            if (p->ins[cur->dense[k]].op == I_MATCH) {
                result = 1;
                goto done;
            }
        if (nxt < 0) break;
        nclist = 0;
        for (int k = 0; k < cur->n; k++) {
            const inst* x = &p->ins[cur->dense[k]];
            if (x->op != I_RUNE) continue;
            for (int r = 0; r < x->nr; r++)
                if (p->rr[x->r0 + r].lo <= (uint32_t)nxt && (uint32_t)nxt <= p->rr[x->r0 + r].hi) {
                    clist[nclist++] = x->x;
                    break;
                }
        }
        prev = nxt;
        i += w;
    }
done:
    free(mem);
    return result;
}

/* ---------------------------------------------------------------------------- matches extern */
static int g_cache = 1;

void oracle_regex_cache(int on) { g_cache = on; }

/* compiled-pattern cache (per thread): the oracle's test runs evaluate the same rule's pattern for
 * many bags; the CPU baseline turns it off, so each call compiles as regexp.MatchString does */
#define RX_CACHE 64
typedef struct {
    uint8_t* pat;
    size_t n;
    oracle_regex* prog;
    int code;
    char err[256];
} rx_entry;
static __thread rx_entry t_cache[RX_CACHE];
static __thread unsigned t_next;

static uint64_t hash_bytes(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

int oracle_regex_match(const uint8_t* pat, size_t npat, const uint8_t* s, size_t n, char* err, size_t errcap) {
    if (!g_cache) {
        oracle_regex* prog;
        const int rc = oracle_regex_compile(pat, npat, &prog, err, errcap);
        if (rc) return rc;
        const int m = oracle_regex_exec(prog, s, n);
        oracle_regex_free(prog);
        return m;
    }
    const unsigned h = (unsigned)(hash_bytes(pat, npat) % RX_CACHE);
    rx_entry* e = &t_cache[h];
    if (!(e->pat && e->n == npat && memcmp(e->pat, pat, npat) == 0)) {
        free(e->pat);
        oracle_regex_free(e->prog);
        memset(e, 0, sizeof *e);
        e->pat = (uint8_t*)malloc(npat ? npat : 1);
        memcpy(e->pat, pat, npat);
        e->n = npat;
        e->code = oracle_regex_compile(pat, npat, &e->prog, e->err, sizeof e->err);
    }
    (void)t_next;
    if (e->code) {
        if (err && errcap) {
            size_t k = strlen(e->err);
            if (k > errcap - 1) k = errcap - 1;
            memcpy(err, e->err, k);
            err[k] = 0;
        }
        return e->code;
    }
    return oracle_regex_exec(e->prog, s, n);
}

/* regexList.checkList (regexList.go:26-33) for a batch of symbols: every pattern compiled once
 * (parseRegexList), a symbol is found when any pattern matches.  found[i] = 1 / 0; returns 0, or the
 * index + 1 of the first pattern that fails to compile (its error in err). */
int oracle_regex_list_found(const uint8_t* pats, const uint64_t* pat_off, uint32_t n_pat, const uint8_t* syms,
                            const uint64_t* sym_off, uint32_t n_sym, int8_t* found, int threads, char* err,
                            size_t errcap) {
    oracle_regex** progs = (oracle_regex**)calloc(n_pat ? n_pat : 1, sizeof(oracle_regex*));
    for (uint32_t k = 0; k < n_pat; k++) {
        if (oracle_regex_compile(pats + pat_off[k], pat_off[k + 1] - pat_off[k], &progs[k], err, errcap)) {
            for (uint32_t j = 0; j < k; j++) oracle_regex_free(progs[j]);
            free(progs);
            return (int)k + 1;
        }
    }
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads > 0 ? threads : 1)
    for (uint32_t i = 0; i < n_sym; i++) {
        int8_t f = 0;
        for (uint32_t k = 0; k < n_pat && !f; k++)
            f = (int8_t)oracle_regex_exec(progs[k], syms + sym_off[i], sym_off[i + 1] - sym_off[i]);
        found[i] = f;
    }
    for (uint32_t k = 0; k < n_pat; k++) oracle_regex_free(progs[k]);
    free(progs);
    return 0;
}
