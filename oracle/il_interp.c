/*
 * ORACLE (test infrastructure only) -- C restatement of the Mixer IL interpreter.
 *
 * Follows mixer/pkg/il/interpreter/interpreterRun.go:18-1163 opcode by opcode (stack of 64 uint32
 * words, 4 registers, 64-slot heap of interface{} values, 64 call frames; interpreter.go:39-44),
 * the extern calling convention of interpreter/extern.go:142-245 and the standard externs of
 * mixer/pkg/il/runtime/externs.go:81-128, plus the EvalPredicate wrapper
 * (mixer/pkg/il/evaluator/evaluator.go:75-83 -> interpreter/result.go:42-52).
 *
 * Bags come from the columnar batch of include/mxp_batch.h; `bag.Get(name)` resolves the name's
 * column and returns (value, found) exactly like FakeBag.Get (il/testing/fakebag.go:49-56).
 *
 * Used by tests/ (parity checker) and by bench.py's cpu_baseline leg (OpenMP over requests).
 * Never linked into the product.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "goval.h"
#include "regex_oracle.h"

enum {
    OP_Halt = 0, OP_Nop = 1, OP_Err = 2, OP_Errz = 3, OP_Errnz = 4,
    OP_PopS = 10, OP_PopB = 11, OP_PopI = 12, OP_PopD = 13,
    OP_DupS = 14, OP_DupB = 15, OP_DupI = 16, OP_DupD = 17,
    OP_RLoadS = 20, OP_RLoadB = 21, OP_RLoadI = 22, OP_RLoadD = 23,
    OP_ALoadS = 30, OP_ALoadB = 31, OP_ALoadI = 32, OP_ALoadD = 33,
    OP_APushS = 40, OP_APushB = 41, OP_APushI = 42, OP_APushD = 43,
    OP_RPushS = 50, OP_RPushB = 51, OP_RPushI = 52, OP_RPushD = 53,
    OP_EqS = 60, OP_EqB = 61, OP_EqI = 62, OP_EqD = 63,
    OP_AEqS = 70, OP_AEqB = 71, OP_AEqI = 72, OP_AEqD = 73,
    OP_Xor = 80, OP_And = 81, OP_Or = 82, OP_AXor = 83, OP_AAnd = 84, OP_AOr = 85, OP_Not = 86,
    OP_ResolveS = 90, OP_ResolveB = 91, OP_ResolveI = 92, OP_ResolveD = 93, OP_ResolveF = 94,
    OP_TResolveS = 100, OP_TResolveB = 101, OP_TResolveI = 102, OP_TResolveD = 103, OP_TResolveF = 104,
    OP_AddI = 110, OP_AddD = 111, OP_SubI = 112, OP_SubD = 113,
    OP_AAddI = 114, OP_AAddD = 115, OP_ASubI = 116, OP_ASubD = 117,
    OP_Jmp = 200, OP_Jz = 201, OP_Jnz = 202, OP_Call = 203, OP_Ret = 204,
    OP_Lookup = 210, OP_TLookup = 211, OP_ALookup = 212, OP_NLookup = 213, OP_ANLookup = 214
};

/* il.Type */
enum { T_Unknown = 0, T_Void, T_String, T_Integer, T_Double, T_Bool, T_Duration, T_Interface };

enum { EXT_NONE = 0, EXT_IP, EXT_IP_EQUAL, EXT_TIMESTAMP, EXT_TIMESTAMP_EQUAL, EXT_MATCH,
       EXT_MATCHES, EXT_STARTSWITH, EXT_ENDSWITH };

#define STACK_SIZE 64
#define HEAP_SIZE 64
#define FRAMES 64
#define REGS 4

typedef struct oracle_prog {
    uint32_t* code;
    uint32_t ncode;
    uint8_t* str_bytes;
    uint64_t* str_off;
    uint32_t nstr;
    /* function table indexed by the string id of the function name */
    uint8_t* fn_kind;      /* 0 none, 1 IL function, 2 extern */
    uint32_t* fn_addr;
    uint8_t* fn_ret;
    uint32_t* fn_param_off;
    uint8_t* fn_nparams;
    uint8_t* fn_params;
    uint8_t* fn_ext;       /* EXT_* for externs */
} oracle_prog;

typedef struct oracle_result {
    int32_t status;        /* 0 ok, 1 error, 2 panic */
    int32_t rtype;         /* il.Type */
    uint32_t v1, v2;
    gv val;                /* string / interface result */
    char msg[512];
} oracle_result;

static uint32_t str_len(const oracle_prog* p, uint32_t id) { return (uint32_t)(p->str_off[id + 1] - p->str_off[id]); }
static const uint8_t* str_ptr(const oracle_prog* p, uint32_t id) { return p->str_bytes + p->str_off[id]; }

static int streq_lit(const oracle_prog* p, uint32_t id, const char* lit) {
    size_t n = strlen(lit);
    return str_len(p, id) == n && memcmp(str_ptr(p, id), lit, n) == 0;
}

void* oracle_prog_new(const uint32_t* code, uint32_t ncode, const uint8_t* str_bytes,
                      const uint64_t* str_off, uint32_t nstr, const uint8_t* fn_kind,
                      const uint32_t* fn_addr, const uint8_t* fn_ret, const uint32_t* fn_param_off,
                      const uint8_t* fn_nparams, const uint8_t* fn_params, uint32_t nparams_total) {
    oracle_prog* p = (oracle_prog*)calloc(1, sizeof *p);
    p->ncode = ncode;
    p->code = (uint32_t*)malloc(sizeof(uint32_t) * (ncode + 4));
    memcpy(p->code, code, sizeof(uint32_t) * ncode);
    memset(p->code + ncode, 0, sizeof(uint32_t) * 4);
    p->nstr = nstr;
    p->str_off = (uint64_t*)malloc(sizeof(uint64_t) * (nstr + 1));
    memcpy(p->str_off, str_off, sizeof(uint64_t) * (nstr + 1));
    p->str_bytes = (uint8_t*)malloc(str_off[nstr] + 1);
    memcpy(p->str_bytes, str_bytes, str_off[nstr]);
    p->fn_kind = (uint8_t*)malloc(nstr);
    memcpy(p->fn_kind, fn_kind, nstr);
    p->fn_addr = (uint32_t*)malloc(sizeof(uint32_t) * nstr);
    memcpy(p->fn_addr, fn_addr, sizeof(uint32_t) * nstr);
    p->fn_ret = (uint8_t*)malloc(nstr);
    memcpy(p->fn_ret, fn_ret, nstr);
    p->fn_param_off = (uint32_t*)malloc(sizeof(uint32_t) * nstr);
    memcpy(p->fn_param_off, fn_param_off, sizeof(uint32_t) * nstr);
    p->fn_nparams = (uint8_t*)malloc(nstr);
    memcpy(p->fn_nparams, fn_nparams, nstr);
    p->fn_params = (uint8_t*)malloc(nparams_total + 1);
    memcpy(p->fn_params, fn_params, nparams_total);
    p->fn_ext = (uint8_t*)calloc(nstr, 1);
    for (uint32_t i = 0; i < nstr; i++) {
        if (p->fn_kind[i] != 2) continue;
        if (streq_lit(p, i, "ip")) p->fn_ext[i] = EXT_IP;
        else if (streq_lit(p, i, "ip_equal")) p->fn_ext[i] = EXT_IP_EQUAL;
        else if (streq_lit(p, i, "timestamp")) p->fn_ext[i] = EXT_TIMESTAMP;
        else if (streq_lit(p, i, "timestamp_equal")) p->fn_ext[i] = EXT_TIMESTAMP_EQUAL;
        else if (streq_lit(p, i, "match")) p->fn_ext[i] = EXT_MATCH;
        else if (streq_lit(p, i, "matches")) p->fn_ext[i] = EXT_MATCHES;
        else if (streq_lit(p, i, "startsWith")) p->fn_ext[i] = EXT_STARTSWITH;
        else if (streq_lit(p, i, "endsWith")) p->fn_ext[i] = EXT_ENDSWITH;
    }
    return p;
}

void oracle_prog_free(void* vp) {
    oracle_prog* p = (oracle_prog*)vp;
    if (!p) return;
    free(p->code); free(p->str_off); free(p->str_bytes); free(p->fn_kind); free(p->fn_addr);
    free(p->fn_ret); free(p->fn_param_off); free(p->fn_nparams); free(p->fn_params); free(p->fn_ext);
    free(p);
}

static uint32_t alloc_size(uint8_t t) {
    switch (t) {
    case T_String: case T_Bool: case T_Interface: return 1;
    case T_Integer: case T_Duration: case T_Double: return 2;
    default: return 0;
    }
}

/* ---------------------------------------------------------------------------- bag access */
/* Referenced-attribute tracking (il/testing/fakebag.go:54-60,102-115): every Get(name) records
 * `name`, every StringMap.Get(key) records `name[key]`, found or not. */
typedef struct ref_ent {
    const uint8_t* name;
    uint32_t nlen;
    int32_t klen;            /* -1: attribute reference, else map key length */
    const uint8_t* key;
} ref_ent;
typedef struct ref_track {
    ref_ent* e;
    uint32_t n, cap;
} ref_track;

static void track_push(ref_track* t, const uint8_t* name, uint32_t nlen, const uint8_t* key, int32_t klen) {
    if (!t) return;
    if (t->n == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->e = (ref_ent*)realloc(t->e, sizeof(ref_ent) * t->cap);
    }
    t->e[t->n].name = name;
    t->e[t->n].nlen = nlen;
    t->e[t->n].key = key;
    t->e[t->n].klen = klen;
    t->n++;
}

typedef struct bagctx {
    const mxp_bag_batch* b;
    const int32_t* col_of_sid;  /* program string id -> batch column, -1 when absent */
    uint32_t req;
    const struct oracle_prog* prog;
    ref_track* track;           /* NULL: no tracking */
} bagctx;

static gv gv_string(const uint8_t* p, uint32_t n) {
    gv v;
    memset(&v, 0, sizeof v);
    v.k = GV_STRING; v.p = p; v.len = n;
    return v;
}

static gv batch_str(const mxp_bag_batch* b, uint32_t sid, uint8_t kind) {
    gv v;
    memset(&v, 0, sizeof v);
    v.k = kind;
    v.p = b->str_bytes + b->str_offsets[sid];
    v.len = (uint32_t)(b->str_offsets[sid + 1] - b->str_offsets[sid]);
    return v;
}

/* attribute.Bag.Get(name) for the program string `sid` */
static int bag_get(const bagctx* c, uint32_t sid, gv* out) {
    if (c->track) track_push(c->track, str_ptr(c->prog, sid), str_len(c->prog, sid), NULL, -1);
    int32_t col = c->col_of_sid[sid];
    if (col < 0) return 0;
    const mxp_bag_batch* b = c->b;
    uint8_t k = b->kinds[col][c->req];
    uint64_t v = b->values[col][c->req];
    memset(out, 0, sizeof *out);
    switch (k) {
    case MXP_ABSENT: return 0;
    case MXP_STRING: *out = batch_str(b, (uint32_t)v, GV_STRING); return 1;
    case MXP_BYTES: *out = batch_str(b, (uint32_t)v, GV_BYTES); return 1;
    case MXP_INT64: out->k = GV_INT64; out->i = (int64_t)v; return 1;
    case MXP_DOUBLE: out->k = GV_DOUBLE; out->i = (int64_t)v; return 1;
    case MXP_BOOL: out->k = GV_BOOL; out->i = v ? 1 : 0; return 1;
    case MXP_DURATION: out->k = GV_DURATION; out->i = (int64_t)v; return 1;
    case MXP_TIMESTAMP: out->k = GV_TIME; out->i = b->time_sec[v]; out->ns = b->time_nsec[v]; return 1;
    case MXP_STRING_MAP:  /* the map remembers its attribute name (p / len) for StringMap.Get tracking */
        out->k = GV_MAP; out->i = (int64_t)v;
        out->p = str_ptr(c->prog, sid); out->len = str_len(c->prog, sid);
        return 1;
    case MXP_OTHER: out->k = GV_OTHER; out->i = (int64_t)v; return 1;
    default: return 0;
    }
}

/* il.MapGet (il/types.go:88-98); returns -1 when the value is not a map (Go panics). */
static int map_get(const bagctx* c, const gv* m, const uint8_t* key, uint32_t klen, gv* out) {
    const mxp_bag_batch* b = c->b;
    if (m->k != GV_MAP) return -1;
    if (c->track) track_push(c->track, m->p, m->len, key, (int32_t)klen);
    for (uint64_t e = b->map_offsets[m->i]; e < b->map_offsets[m->i + 1]; e++) {
        uint32_t ks = b->map_keys[e];
        uint32_t n = (uint32_t)(b->str_offsets[ks + 1] - b->str_offsets[ks]);
        if (n == klen && memcmp(b->str_bytes + b->str_offsets[ks], key, n) == 0) {
            *out = batch_str(b, b->map_values[e], GV_STRING);
            return 1;
        }
    }
    return 0;
}

static int gv_str_eq(const gv* a, const gv* b) {
    return a->len == b->len && (a->len == 0 || memcmp(a->p, b->p, a->len) == 0);
}

/* ------------------------------------------------------------------------------ run */
static void set_msg(oracle_result* r, int status, const char* fmt, const char* a, uint32_t alen) {
    r->status = status;
    char tmp[400];
    uint32_t n = alen < sizeof tmp - 1 ? alen : (uint32_t)sizeof tmp - 1;
    if (a) memcpy(tmp, a, n);
    tmp[a ? n : 0] = 0;
    snprintf(r->msg, sizeof r->msg, fmt, tmp);
}

#define PANIC(text) do { r->status = 2; snprintf(r->msg, sizeof r->msg, "%s", text); return 2; } while (0)
#define FAIL(text) do { r->status = 1; snprintf(r->msg, sizeof r->msg, "%s", text); return 1; } while (0)

static int conv_err(oracle_result* r, const char* what, const gv* v, const mxp_bag_batch* b) {
    char val[256];
    oracle_format_value(v, b, val, sizeof val);
    r->status = 1;
    snprintf(r->msg, sizeof r->msg, "error converting value to %s: '%s'", what, val);
    return 1;
}

static int run(const oracle_prog* p, uint32_t fn_sid, const bagctx* bc, oracle_result* r) {
    uint32_t registers[REGS] = {0};
    uint32_t sp = 0, ip, fp = 0;
    uint32_t opstack[STACK_SIZE + 4];
    struct { uint32_t regs[REGS]; uint32_t sp, ip, fn; } frames[FRAMES];
    gv heap[HEAP_SIZE + 1];
    uint32_t hp = 0;
    const mxp_bag_batch* b = bc->b;
    uint32_t t1, t2, t3;
    gv tv;
    uint32_t fn = fn_sid;

    /* The reference zero-initialises its stack, frames and heap per call (interpreterRun.go:49-51).
     * Only never-written heap slots and frame registers are observable (as nil / 0): heap reads at
     * or above hp yield nil below, and frames are zeroed on first use. */
    int frames_zeroed = 0;
    r->status = 0;
    r->v1 = r->v2 = 0;
    r->msg[0] = 0;
    memset(&r->val, 0, sizeof r->val);
    r->rtype = p->fn_ret[fn];
    ip = p->fn_addr[fn];
    if (p->fn_nparams[fn] != 0) FAIL("init function must have 0 args");

#define STR(id) ((const char*)str_ptr(p, (id))), str_len(p, (id))
#define UNDERFLOW do { FAIL("stack underflow"); } while (0)
#define OVERFLOW do { FAIL("stack overflow"); } while (0)
#define HEAPOVF do { FAIL("heap overflow"); } while (0)
    /* hp can reach 64 only through an extern's unchecked push (extern.go:212,235); the next
     * checked push then writes heap[64]: Go's index panic */
#define BADHEAP do { FAIL("invalid heap access"); } while (0)

    for (;;) {
        if (ip >= p->ncode) PANIC("runtime error: index out of range");
        uint32_t code = p->code[ip++];
        switch (code) {
        case OP_Halt: FAIL("catching fire as instructed");
        case OP_Nop: break;
        case OP_Err:
            t1 = p->code[ip++];
            set_msg(r, 1, "%s", STR(t1));
            return 1;
        case OP_Errz: case OP_Errnz:
            if (sp < 1) UNDERFLOW;
            t1 = p->code[ip++];
            sp--;
            t2 = opstack[sp];
            if ((code == OP_Errz && t2 == 0) || (code == OP_Errnz && t2 != 0)) {
                set_msg(r, 1, "%s", STR(t1));
                return 1;
            }
            break;
        case OP_PopS: case OP_PopB:
            if (sp < 1) UNDERFLOW;
            sp--;
            break;
        case OP_PopI: case OP_PopD:
            if (sp < 2) UNDERFLOW;
            sp -= 2;
            break;
        case OP_DupS: case OP_DupB:
            if (sp < 1) UNDERFLOW;
            if (sp > STACK_SIZE - 1) OVERFLOW;
            opstack[sp] = opstack[sp - 1];
            sp++;
            break;
        case OP_DupI: case OP_DupD:
            if (sp < 2) UNDERFLOW;
            if (sp > STACK_SIZE - 2) OVERFLOW;
            opstack[sp] = opstack[sp - 2];
            opstack[sp + 1] = opstack[sp - 1];
            sp += 2;
            break;
        case OP_RLoadS: case OP_RLoadB:
            if (sp < 1) UNDERFLOW;
            t1 = p->code[ip++];
            if (t1 >= REGS) PANIC("runtime error: index out of range");
            sp--;
            registers[t1] = opstack[sp];
            break;
        case OP_RLoadI: case OP_RLoadD:
            if (sp < 2) UNDERFLOW;
            t1 = p->code[ip++];
            if (t1 + 1 >= REGS) PANIC("runtime error: index out of range");
            registers[t1] = opstack[sp - 1];
            registers[t1 + 1] = opstack[sp - 2];
            sp -= 2;
            break;
        case OP_ALoadS:
            t1 = p->code[ip++];
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            if (t1 >= REGS) PANIC("runtime error: index out of range");
            t2 = hp;
            heap[hp++] = gv_string(str_ptr(p, t1), str_len(p, t1));
            registers[t1] = t2;
            break;
        case OP_ALoadB:
            t1 = p->code[ip++];
            if (t1 >= REGS) PANIC("runtime error: index out of range");
            registers[t1] = p->code[ip++];
            break;
        case OP_ALoadI: case OP_ALoadD:
            t1 = p->code[ip++];
            if (t1 + 1 >= REGS) PANIC("runtime error: index out of range");
            registers[t1] = p->code[ip];
            registers[t1 + 1] = p->code[ip + 1];
            ip += 2;
            break;
        case OP_RPushS: case OP_RPushB:
            t1 = p->code[ip++];
            if (sp > STACK_SIZE - 1) OVERFLOW;
            if (t1 >= REGS) PANIC("runtime error: index out of range");
            opstack[sp++] = registers[t1];
            break;
        case OP_RPushI: case OP_RPushD:
            t1 = p->code[ip++];
            if (sp > STACK_SIZE - 1) OVERFLOW;
            if (t1 + 1 >= REGS) PANIC("runtime error: index out of range");
            opstack[sp] = registers[t1 + 1];
            opstack[sp + 1] = registers[t1];
            sp += 2;
            break;
        case OP_APushS:
            t1 = p->code[ip++];
            if (sp > STACK_SIZE - 1) OVERFLOW;
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            t2 = hp;
            heap[hp++] = gv_string(str_ptr(p, t1), str_len(p, t1));
            opstack[sp++] = t2;
            break;
        case OP_APushB:
            t1 = p->code[ip++];
            if (sp > STACK_SIZE - 1) OVERFLOW;
            opstack[sp++] = t1;
            break;
        case OP_APushI: case OP_APushD:
            t1 = p->code[ip];
            t2 = p->code[ip + 1];
            ip += 2;
            if (sp > STACK_SIZE - 2) OVERFLOW;
            opstack[sp] = t2;
            opstack[sp + 1] = t1;
            sp += 2;
            break;
        case OP_EqS:
            if (sp < 2) UNDERFLOW;
            t1 = opstack[sp - 1];
            t2 = opstack[sp - 2];
            sp -= 2;
            if (t1 >= hp) BADHEAP;
            if (heap[t1].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
            if (t2 >= hp) BADHEAP;
            if (heap[t2].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
            opstack[sp++] = gv_str_eq(&heap[t1], &heap[t2]) ? 1 : 0;
            break;
        case OP_EqB:
            if (sp < 2) UNDERFLOW;
            t1 = opstack[sp - 1];
            t2 = opstack[sp - 2];
            sp -= 2;
            opstack[sp++] = t1 == t2 ? 1 : 0;
            break;
        case OP_EqI: case OP_EqD:
            if (sp < 4) UNDERFLOW;
            t3 = (opstack[sp - 1] == opstack[sp - 3] && opstack[sp - 2] == opstack[sp - 4]) ? 1 : 0;
            sp -= 4;
            opstack[sp++] = t3;
            break;
        case OP_AEqS: {
            t1 = p->code[ip++];
            if (sp < 1) UNDERFLOW;
            sp--;
            t2 = opstack[sp];
            if (t2 >= hp) BADHEAP;
            if (heap[t2].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
            gv c = gv_string(str_ptr(p, t1), str_len(p, t1));
            opstack[sp++] = gv_str_eq(&c, &heap[t2]) ? 1 : 0;
            break;
        }
        case OP_AEqB:
            t1 = p->code[ip++];
            if (sp < 1) UNDERFLOW;
            sp--;
            t2 = opstack[sp];
            opstack[sp++] = t1 == t2 ? 1 : 0;
            break;
        case OP_AEqI: case OP_AEqD:
            t1 = p->code[ip];
            t2 = p->code[ip + 1];
            ip += 2;
            if (sp < 2) UNDERFLOW;
            t3 = (opstack[sp - 1] == t1 && opstack[sp - 2] == t2) ? 1 : 0;
            sp -= 2;
            opstack[sp++] = t3;
            break;
        case OP_Xor: case OP_And: case OP_Or:
            if (sp < 2) UNDERFLOW;
            t1 = opstack[sp - 1];
            t2 = opstack[sp - 2];
            sp -= 2;
            if (code == OP_Xor) opstack[sp++] = ((t1 == 0 && t2 == 0) || (t1 != 0 && t2 != 0)) ? 0 : 1;
            else if (code == OP_And) opstack[sp++] = (t1 != 0 && t2 != 0) ? 1 : 0;
            else opstack[sp++] = (t1 == 0 && t2 == 0) ? 0 : 1;
            break;
        case OP_AXor: case OP_AAnd: case OP_AOr:
            t1 = p->code[ip++];
            if (sp < 1) UNDERFLOW;
            sp--;
            t2 = opstack[sp];
            if (code == OP_AXor) opstack[sp++] = ((t1 == 0 && t2 == 0) || (t1 != 0 && t2 != 0)) ? 0 : 1;
            else if (code == OP_AAnd) opstack[sp++] = (t1 != 0 && t2 != 0) ? 1 : 0;
            else opstack[sp++] = (t1 == 0 && t2 == 0) ? 0 : 1;
            break;
        case OP_Not:
            if (sp < 1) UNDERFLOW;
            opstack[sp - 1] = opstack[sp - 1] == 0 ? 1 : 0;
            break;

        case OP_ResolveS: case OP_TResolveS:
            if (sp > STACK_SIZE - (code == OP_ResolveS ? 1u : 2u)) OVERFLOW;
            t1 = p->code[ip++];
            if (!bag_get(bc, t1, &tv)) {
                if (code == OP_TResolveS) { opstack[sp++] = 0; break; }
                set_msg(r, 1, "lookup failed: '%s'", STR(t1));
                return 1;
            }
            if (tv.k != GV_STRING) return conv_err(r, "string", &tv, b);
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            t2 = hp;
            heap[hp++] = tv;
            opstack[sp++] = t2;
            if (code == OP_TResolveS) opstack[sp++] = 1;
            break;
        case OP_ResolveB: case OP_TResolveB:
            if (sp > STACK_SIZE - (code == OP_ResolveB ? 1u : 2u)) OVERFLOW;
            t1 = p->code[ip++];
            if (!bag_get(bc, t1, &tv)) {
                if (code == OP_TResolveB) { opstack[sp++] = 0; break; }
                set_msg(r, 1, "lookup failed: '%s'", STR(t1));
                return 1;
            }
            if (tv.k != GV_BOOL) return conv_err(r, "bool", &tv, b);
            opstack[sp++] = tv.i ? 1 : 0;
            if (code == OP_TResolveB) opstack[sp++] = 1;
            break;
        case OP_ResolveI: case OP_TResolveI:
            if (sp > STACK_SIZE - (code == OP_ResolveI ? 2u : 3u)) OVERFLOW;
            t1 = p->code[ip++];
            if (!bag_get(bc, t1, &tv)) {
                if (code == OP_TResolveI) { opstack[sp++] = 0; break; }
                set_msg(r, 1, "lookup failed: '%s'", STR(t1));
                return 1;
            }
            if (tv.k != GV_INT64 && tv.k != GV_DURATION) return conv_err(r, "integer or duration", &tv, b);
            opstack[sp] = (uint32_t)((uint64_t)tv.i >> 32);
            opstack[sp + 1] = (uint32_t)((uint64_t)tv.i & 0xFFFFFFFFu);
            sp += 2;
            if (code == OP_TResolveI) opstack[sp++] = 1;
            break;
        case OP_ResolveD: case OP_TResolveD:
            if (sp > STACK_SIZE - (code == OP_ResolveD ? 2u : 3u)) OVERFLOW;
            t1 = p->code[ip++];
            if (!bag_get(bc, t1, &tv)) {
                if (code == OP_TResolveD) { opstack[sp++] = 0; break; }
                set_msg(r, 1, "lookup failed: '%s'", STR(t1));
                return 1;
            }
            if (tv.k != GV_DOUBLE) return conv_err(r, "double", &tv, b);
            opstack[sp] = (uint32_t)((uint64_t)tv.i >> 32);
            opstack[sp + 1] = (uint32_t)((uint64_t)tv.i & 0xFFFFFFFFu);
            sp += 2;
            if (code == OP_TResolveD) opstack[sp++] = 1;
            break;
        case OP_ResolveF: case OP_TResolveF:
            if (sp > STACK_SIZE - 2) OVERFLOW;
            t1 = p->code[ip++];
            if (!bag_get(bc, t1, &tv)) {
                if (code == OP_TResolveF) { opstack[sp++] = 0; break; }
                set_msg(r, 1, "lookup failed: '%s'", STR(t1));
                return 1;
            }
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            t2 = hp;
            heap[hp++] = tv;
            opstack[sp++] = t2;
            if (code == OP_TResolveF) opstack[sp++] = 1;
            break;

        case OP_AddI: case OP_SubI: {
            if (sp < 4) UNDERFLOW;
            t1 = opstack[sp - 1]; t2 = opstack[sp - 2]; sp -= 2;
            uint64_t a = (uint64_t)t1 + ((uint64_t)t2 << 32);
            if (code == OP_SubI) a = (uint64_t)(-(int64_t)a);
            t1 = opstack[sp - 1]; t2 = opstack[sp - 2]; sp -= 2;
            a += (uint64_t)t1 + ((uint64_t)t2 << 32);
            opstack[sp] = (uint32_t)(a >> 32);
            opstack[sp + 1] = (uint32_t)a;
            sp += 2;
            break;
        }
        case OP_AAddI: case OP_ASubI: {
            if (sp < 2) UNDERFLOW;
            t1 = p->code[ip]; t2 = p->code[ip + 1]; ip += 2;
            uint64_t a = (uint64_t)t1 + ((uint64_t)t2 << 32);
            if (code == OP_ASubI) a = (uint64_t)(-(int64_t)a);
            t1 = opstack[sp - 1]; t2 = opstack[sp - 2]; sp -= 2;
            a += (uint64_t)t1 + ((uint64_t)t2 << 32);
            opstack[sp] = (uint32_t)(a >> 32);
            opstack[sp + 1] = (uint32_t)a;
            sp += 2;
            break;
        }
        case OP_AddD: case OP_SubD: case OP_AAddD: case OP_ASubD: {
            uint64_t u;
            double d, e;
            if (code == OP_AddD || code == OP_SubD) {
                if (sp < 4) UNDERFLOW;
                t1 = opstack[sp - 1]; t2 = opstack[sp - 2]; sp -= 2;
            } else {
                if (sp < 2) UNDERFLOW;
                t1 = p->code[ip]; t2 = p->code[ip + 1]; ip += 2;
            }
            u = (uint64_t)t1 + ((uint64_t)t2 << 32);
            memcpy(&d, &u, 8);
            if (code == OP_SubD || code == OP_ASubD) d *= -1;
            t1 = opstack[sp - 1]; t2 = opstack[sp - 2]; sp -= 2;
            u = (uint64_t)t1 + ((uint64_t)t2 << 32);
            memcpy(&e, &u, 8);
            d += e;
            memcpy(&u, &d, 8);
            opstack[sp] = (uint32_t)(u >> 32);
            opstack[sp + 1] = (uint32_t)u;
            sp += 2;
            break;
        }

        case OP_Jmp:
            t1 = p->code[ip++];
            ip = t1;
            break;
        case OP_Jz: case OP_Jnz:
            if (sp < 1) UNDERFLOW;
            t1 = p->code[ip++];
            sp--;
            t2 = opstack[sp];
            if ((code == OP_Jz && t2 == 0) || (code == OP_Jnz && t2 != 0)) ip = t1;
            break;

        case OP_Call: {
            t1 = p->code[ip++];
            if (fp >= FRAMES) PANIC("runtime error: index out of range");
            if (!frames_zeroed) {
                memset(frames, 0, sizeof frames);
                frames_zeroed = 1;
            }
            /* stackFrame.save copies the frame's registers over the live ones (stackFrame.go:28-33) */
            uint32_t nps = 0;
            for (uint32_t k = 0; k < p->fn_nparams[fn]; k++) nps += alloc_size(p->fn_params[p->fn_param_off[fn] + k]);
            memcpy(registers, frames[fp].regs, sizeof registers);
            frames[fp].sp = sp - nps;
            frames[fp].ip = ip;
            frames[fp].fn = fn;
            fp++;
            if (t1 >= p->nstr || p->fn_kind[t1] == 0) {
                set_msg(r, 1, "function not found: '%s'", STR(t1));
                return 1;
            }
            if (p->fn_kind[t1] == 2) {
                fp--;
                uint32_t psz = 0;
                for (uint32_t k = 0; k < p->fn_nparams[t1]; k++) psz += alloc_size(p->fn_params[p->fn_param_off[t1] + k]);
                if (sp < psz) UNDERFLOW;
                uint32_t ap = sp - psz;
                uint32_t ro1 = 0, ro2 = 0;
                gv args[2];
                int ext = p->fn_ext[t1];
                if (ext == EXT_NONE) PANIC("extern not bound");
                for (uint32_t k = 0; k < p->fn_nparams[t1] && k < 2; k++) {
                    uint32_t hi = opstack[ap];
                    if (hi >= HEAP_SIZE) PANIC("runtime error: index out of range");
                    if (hi < hp) args[k] = heap[hi];
                    else memset(&args[k], 0, sizeof args[k]);  /* never-written slot: nil */
                    ap += 1;
                }
                switch (ext) {
                case EXT_IP: {
                    if (args[0].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
                    uint8_t out[16];
                    if (!oracle_parse_ip(args[0].p, args[0].len, out)) {
                        set_msg(r, 1, "could not convert %s to IP_ADDRESS", (const char*)args[0].p, args[0].len);
                        return 1;
                    }
                    gv res;
                    memset(&res, 0, sizeof res);
                    res.k = GV_BYTES; res.len = 16; res.inl_used = 1;
                    memcpy(res.inl, out, 16);
                    if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range");
                    heap[hp] = res;
                    heap[hp].p = heap[hp].inl;
                    hp++;
                    ro1 = hp - 1;
                    break;
                }
                case EXT_IP_EQUAL:
                    if (args[0].k != GV_BYTES || args[1].k != GV_BYTES) PANIC("reflect: Call using value as type []uint8");
                    ro1 = (uint32_t)oracle_ip_equal(args[0].p, args[0].len, args[1].p, args[1].len);
                    break;
                case EXT_TIMESTAMP: {
                    if (args[0].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
                    int64_t s; int32_t ns;
                    if (!oracle_parse_rfc3339(args[0].p, args[0].len, &s, &ns)) {
                        char tmp[300];
                        uint32_t n = args[0].len < 250 ? args[0].len : 250;
                        memcpy(tmp, args[0].p, n);
                        tmp[n] = 0;
                        r->status = 1;
                        snprintf(r->msg, sizeof r->msg,
                                 "could not convert '%s' to TIMESTAMP. expected format: '2006-01-02T15:04:05Z07:00'", tmp);
                        return 1;
                    }
                    gv res;
                    memset(&res, 0, sizeof res);
                    res.k = GV_TIME; res.i = s; res.ns = ns;
                    if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range");
                    heap[hp++] = res;
                    ro1 = hp - 1;
                    break;
                }
                case EXT_TIMESTAMP_EQUAL:
                    if (args[0].k != GV_TIME || args[1].k != GV_TIME) PANIC("reflect: Call using value as type time.Time");
                    ro1 = (args[0].i == args[1].i && args[0].ns == args[1].ns) ? 1 : 0;
                    break;
                case EXT_MATCH: case EXT_MATCHES: case EXT_STARTSWITH: case EXT_ENDSWITH: {
                    if (args[0].k != GV_STRING || args[1].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
                    const gv* s = &args[0];
                    const gv* pt = &args[1];
                    if (ext == EXT_MATCH) {
                        /* externs.go:108-116 */
                        if (pt->len > 0 && pt->p[pt->len - 1] == '*')
                            ro1 = s->len >= pt->len - 1 && memcmp(s->p, pt->p, pt->len - 1) == 0;
                        else if (pt->len > 0 && pt->p[0] == '*')
                            ro1 = s->len >= pt->len - 1 && memcmp(s->p + s->len - (pt->len - 1), pt->p + 1, pt->len - 1) == 0;
                        else
                            ro1 = gv_str_eq(s, pt);
                    } else if (ext == EXT_STARTSWITH) {
                        ro1 = s->len >= pt->len && memcmp(s->p, pt->p, pt->len) == 0;
                    } else if (ext == EXT_ENDSWITH) {
                        ro1 = s->len >= pt->len && memcmp(s->p + s->len - pt->len, pt->p, pt->len) == 0;
                    } else {
                        /* externMatches(pattern, str): target (1st arg) is the pattern */
                        char err[256];
                        int m = oracle_regex_match(args[0].p, args[0].len, args[1].p, args[1].len, err, sizeof err);
                        if (m < 0) {
                            r->status = 1;
                            snprintf(r->msg, sizeof r->msg, "%s", err);
                            return 1;
                        }
                        ro1 = (uint32_t)m;
                    }
                    break;
                }
                default:
                    PANIC("unknown extern");
                }
                uint32_t rsz = alloc_size(p->fn_ret[t1]);
                /* interpreterRun.go:899-900 store two words; at sp - psz + 1 == 64 the second one is
                 * past the 64-word opstack: Go's index panic */
                if (sp - psz + 1 >= STACK_SIZE) PANIC("runtime error: index out of range");
                opstack[sp - psz] = ro1;
                opstack[sp - psz + 1] = ro2;
                sp -= psz - rsz;
                break;
            }
            fn = t1;
            ip = p->fn_addr[t1];
            break;
        }

        case OP_Ret:
            if (fp == 0) {
                uint8_t rt = p->fn_ret[fn];
                r->rtype = rt;
                switch (rt) {
                case T_Void: break;
                case T_Integer: case T_Double: case T_Bool: case T_Duration:
                    if (alloc_size(rt) == 1) {
                        if (sp < 1) UNDERFLOW;
                        r->v1 = opstack[sp - 1];
                    } else {
                        if (sp < 2) UNDERFLOW;
                        r->v1 = opstack[sp - 1];
                        r->v2 = opstack[sp - 2];
                    }
                    break;
                case T_String:
                    if (sp < 1) UNDERFLOW;
                    r->v1 = opstack[sp - 1];
                    if (r->v1 >= hp) BADHEAP;
                    if (heap[r->v1].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
                    r->val = heap[r->v1];
                    break;
                case T_Interface:
                    if (sp < 1) UNDERFLOW;
                    r->v1 = opstack[sp - 1];
                    if (r->v1 >= HEAP_SIZE) PANIC("runtime error: index out of range");
                    if (r->v1 < hp) r->val = heap[r->v1];
                    if (r->val.inl_used) r->val.p = r->val.inl; /* ip() bytes travel with the result */
                    break;
                default:
                    PANIC("interpreter.run: unhandled return type");
                }
                r->status = 0;
                return 0;
            }
            {
                t1 = alloc_size(p->fn_ret[fn]);
                t2 = sp;
                fp--;
                memcpy(frames[fp].regs, registers, sizeof registers);  /* restore() copies live -> frame */
                sp = frames[fp].sp;
                ip = frames[fp].ip;
                fn = frames[fp].fn;
                for (t3 = 0; t3 < t1; t3++) opstack[sp + t3] = opstack[t2 - t1 + t3];
                sp += t1;
            }
            break;

        case OP_TLookup: case OP_Lookup: case OP_NLookup: {
            if (sp < 2) UNDERFLOW;
            t1 = opstack[sp - 1];
            t2 = opstack[sp - 2];
            sp -= 2;
            if (t1 >= hp) BADHEAP;
            if (heap[t1].k != GV_STRING) PANIC("interface conversion: interface {} is not string");
            gv key = heap[t1];
            if (t2 >= hp) BADHEAP;
            gv m = heap[t2];
            int f = map_get(bc, &m, key.p, key.len, &tv);
            if (f < 0) PANIC("Unknown map type");
            if (code == OP_TLookup) {
                if (f) {
                    if (hp == HEAP_SIZE - 1) HEAPOVF;
                    if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
                    t3 = hp;
                    heap[hp++] = tv;
                    opstack[sp] = t3;
                    opstack[sp + 1] = 1;
                    sp += 2;
                } else {
                    opstack[sp++] = 0;
                }
                break;
            }
            if (!f) {
                if (code == OP_Lookup) {
                    set_msg(r, 1, "member lookup failed: '%s'", (const char*)key.p, key.len);
                    return 1;
                }
                tv = gv_string((const uint8_t*)"", 0);
            }
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            t3 = hp;
            heap[hp++] = tv;
            opstack[sp++] = t3;
            break;
        }
        case OP_ALookup: case OP_ANLookup: {
            if (sp < 1) UNDERFLOW;
            t1 = p->code[ip++];
            sp--;
            t2 = opstack[sp];
            if (t2 >= hp) BADHEAP;
            gv m = heap[t2];
            int f = map_get(bc, &m, str_ptr(p, t1), str_len(p, t1), &tv);
            if (f < 0) PANIC("Unknown map type");
            if (!f) {
                if (code == OP_ALookup) {
                    set_msg(r, 1, "member lookup failed: '%s'", STR(t1));
                    return 1;
                }
                tv = gv_string((const uint8_t*)"", 0);
            }
            if (hp == HEAP_SIZE - 1) HEAPOVF;
            if (hp >= HEAP_SIZE) PANIC("runtime error: index out of range"); /* heap[64] after an extern push */
            t3 = hp;
            heap[hp++] = tv;
            opstack[sp++] = t3;
            break;
        }
        default: {
            char tmp[64];
            snprintf(tmp, sizeof tmp, "invalid opcode: '%u'", code);
            FAIL(tmp);
        }
        }
    }
}

/* ------------------------------------------------------------------------------ API */

static int32_t* build_colmap(const oracle_prog* p, const mxp_bag_batch* b) {
    int32_t* m = (int32_t*)malloc(sizeof(int32_t) * (p->nstr ? p->nstr : 1));
    for (uint32_t s = 0; s < p->nstr; s++) {
        m[s] = -1;
        uint32_t n = str_len(p, s);
        for (uint32_t c = 0; c < b->n_columns; c++) {
            const char* name = b->column_names[c];
            if (strlen(name) == n && memcmp(name, str_ptr(p, s), n) == 0) { m[s] = (int32_t)c; break; }
        }
    }
    return m;
}

/* Interpreter.Eval(fnName) for one request of the batch. Returns status. */
int oracle_eval(void* vp, uint32_t fn_sid, const mxp_bag_batch* b, uint32_t req, oracle_result* out) {
    oracle_prog* p = (oracle_prog*)vp;
    int32_t* cm = build_colmap(p, b);
    bagctx bc = {b, cm, req, p, NULL};
    run(p, fn_sid, &bc, out);
    free(cm);
    return out->status;
}

/*
 * EvalPredicate over a request x rule matrix: codes[req * nprogs + rule] =
 *   0 false, 1 true, 2 error (evaluation error), 3 panic (Go runtime panic, incl. AsBool on a
 *   non-bool result).  fn_sids[rule] is the id of "eval" in program `rule`.
 */
void oracle_eval_matrix(void** progs, const uint32_t* fn_sids, uint32_t nprogs, const mxp_bag_batch* b,
                        uint32_t req_begin, uint32_t req_end, uint8_t* codes, int nthreads) {
    int32_t** cms = (int32_t**)malloc(sizeof(int32_t*) * (nprogs ? nprogs : 1));
    for (uint32_t k = 0; k < nprogs; k++) cms[k] = build_colmap((oracle_prog*)progs[k], b);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t rq = (int64_t)req_begin; rq < (int64_t)req_end; rq++) {
        oracle_result r;
        for (uint32_t k = 0; k < nprogs; k++) {
            const oracle_prog* p = (const oracle_prog*)progs[k];
            bagctx bc = {b, cms[k], (uint32_t)rq, p, NULL};
            run(p, fn_sids[k], &bc, &r);
            uint8_t c;
            if (r.status == 1) c = 2;
            else if (r.status == 2) c = 3;
            else if (r.rtype != T_Bool) c = 3;
            else c = r.v1 ? 1 : 0;
            codes[(uint64_t)(rq - req_begin) * nprogs + k] = c;
        }
    }
    (void)nthreads;
    for (uint32_t k = 0; k < nprogs; k++) free(cms[k]);
    free(cms);
}

/* Error text of one pair (for comparing error messages). Returns status. */
int oracle_eval_msg(void* vp, uint32_t fn_sid, const mxp_bag_batch* b, uint32_t req, char* msg, uint32_t cap) {
    oracle_result r;
    oracle_eval(vp, fn_sid, b, req, &r);
    snprintf(msg, cap, "%s", r.msg);
    return r.status;
}

size_t oracle_result_size(void) { return sizeof(oracle_result); }

/* ------------------------------------------------------------------ referenced attributes */
static int ref_cmp_str(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
    int c = memcmp(a, b, na < nb ? na : nb);
    return c ? c : (na < nb ? -1 : na > nb ? 1 : 0);
}
typedef struct ref_str {
    char* s;
    size_t n;
} ref_str;
static int ref_str_cmp(const void* x, const void* y) {
    const ref_str* a = (const ref_str*)x;
    const ref_str* b = (const ref_str*)y;
    return ref_cmp_str((const uint8_t*)a->s, a->n, (const uint8_t*)b->s, b->n);
}

/*
 * FakeBag.ReferencedList (il/testing/fakebag.go:75-89) of one request after EvalPredicate of every
 * program in order: the sorted, distinct "name" / "name[key]" strings, each followed by '\n', into
 * out.  Returns the length written, or -(length needed) when cap is too small.
 */
int64_t oracle_referenced(void** progs, const uint32_t* fn_sids, uint32_t nprogs, const mxp_bag_batch* b,
                          uint32_t req, char* out, uint64_t cap) {
    ref_track t = {NULL, 0, 0};
    for (uint32_t k = 0; k < nprogs; k++) {
        const oracle_prog* p = (const oracle_prog*)progs[k];
        int32_t* cm = build_colmap(p, b);
        bagctx bc = {b, cm, req, p, &t};
        oracle_result r;
        run(p, fn_sids[k], &bc, &r);
        /* names point into the program: copy before the next program runs */
        free(cm);
        for (uint32_t i = 0; i < t.n; i++) {
            if (t.e[i].klen == -2) continue;
            size_t n = t.e[i].nlen + (t.e[i].klen >= 0 ? (size_t)t.e[i].klen + 2 : 0);
            char* s = (char*)malloc(n + 1);
            memcpy(s, t.e[i].name, t.e[i].nlen);
            if (t.e[i].klen >= 0) {
                s[t.e[i].nlen] = '[';
                memcpy(s + t.e[i].nlen + 1, t.e[i].key, (size_t)t.e[i].klen);
                s[n - 1] = ']';
            }
            s[n] = 0;
            t.e[i].name = (const uint8_t*)s;
            t.e[i].nlen = (uint32_t)n;
            t.e[i].klen = -2;  /* materialised */
        }
    }
    ref_str* v = (ref_str*)malloc(sizeof(ref_str) * (t.n ? t.n : 1));
    for (uint32_t i = 0; i < t.n; i++) {
        v[i].s = (char*)t.e[i].name;
        v[i].n = t.e[i].nlen;
    }
    qsort(v, t.n, sizeof(ref_str), ref_str_cmp);
    uint64_t len = 0;
    for (uint32_t i = 0; i < t.n; i++) {
        if (i && ref_str_cmp(&v[i], &v[i - 1]) == 0) continue;
        if (len + v[i].n + 1 <= cap) {
            memcpy(out + len, v[i].s, v[i].n);
            out[len + v[i].n] = '\n';
        }
        len += v[i].n + 1;
    }
    for (uint32_t i = 0; i < t.n; i++) free(v[i].s);
    free(v);
    free(t.e);
    return len <= cap ? (int64_t)len : -(int64_t)len;
}
