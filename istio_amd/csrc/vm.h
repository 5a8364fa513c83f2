// vm.h -- the engine's GPU predicate bytecode ("MXP VM"), shared by the host lowering (lower.cpp)
// and the gfx950 kernels (kernels.hip).
//
// A rule's reference IL (mixer/pkg/il, produced by compile_rule) is lowered to a flat, wave-uniform
// program: every stack slot of the reference VM (interpreterRun.go, 64 x u32 words) becomes a
// statically numbered 64-bit register, `tresolve_x; jnz` / `tlookup; jnz` pairs fuse into one op,
// `resolve_f m; anlookup "k"` fuses into a virtual-column load, constant `ip("...")` /
// `timestamp("...")` / string-pattern externs fold or specialise.  One wavefront runs one rule over
// 64 requests (one request per lane); jumps are forward-only and become per-lane wait targets.
#pragma once

#include <stdint.h>

#define MXP_VM_MAXREG 8      // registers (reference stack slots) per rule in the hot kernels
#define MXP_VM_DEEPREG 64    // ... in the deep-rule VM kernels (rules with more values live at once)
#define MXP_VM_WAKE 0x80u    // op flag: some jump lands on this instruction
#define MXP_VM_DONE 0xFFFFFFFFu

enum mxp_vm_op {
    VM_NOP = 0,
    VM_RES = 1,      // d <- column x (want class y); missing -> ERR_LOOKUP(z = attr id), wrong kind -> ERR_CONV
    VM_TRES = 2,     // tresolve+jnz: present -> d <- column x, jump z; absent -> fall through
    VM_VCOL = 3,     // d <- virtual column x (map attr [const key]); z = attr id
    VM_CONST = 4,    // d <- y | z << 32
    VM_EQ = 5,       // d <- r[a] == r[b]
    VM_EQK = 6,      // d <- r[a] == (y | z << 32)
    VM_NOT = 7,      // d <- r[a] == 0
    VM_JZ = 8,       // r[a] == 0 -> jump z
    VM_JNZ = 9,      // r[a] != 0 -> jump z
    VM_JMP = 10,     // jump z
    VM_RET = 11,     // result r[a]; y = 1 when the function returns bool (else EvalPredicate panics)
    VM_LOOKUP = 12,  // map r[a], key r[b]; y = mode (LK_*); d <- value; z = jump target (LK_TRY)
    VM_LOOKUPK = 13, // map r[a], key string x; y = mode; d <- value; z = jump target (LK_TRY)
    VM_STRFN = 14,   // d <- fn y (SF_*) (r[a], r[b])
    VM_STRFNK = 15,  // d <- fn y (r[a], const string x)        (x = pattern / prefix / suffix id)
    VM_IPOF = 16,    // d <- ip(r[a])          (per-string pre-table; error if unparsable)
    VM_TSOF = 17,    // d <- timestamp(r[a])   (per-string pre-table)
    VM_IPEQ = 18,    // d <- ip_equal(r[a], r[b])
    VM_TSEQ = 19,    // d <- timestamp_equal(r[a], r[b])
    VM_ERR = 20,     // raise error y with aux z
    VM_LOGIC = 21,   // d <- r[a] (y: 0 and, 1 or, 2 xor) r[b]
    VM_LOGICK = 22,  // d <- r[a] (y) const x
    VM_FTOS = 23,    // d <- r[a] as string: interface value must hold a string (Go `.(string)`), else panic
    VM_STOF = 24,    // d <- interface handle of string r[a]
    VM_JZRET = 25,   // r[a] == 0 -> finish with bool result y
    VM_JNZRET = 26,  // r[a] != 0 -> finish with bool result y
    VM_RETK = 27,    // finish with bool result y
    VM_MOV = 28,     // d <- r[a]                 (templates: hoisted CONST)
    VM_REGEX = 29,   // d <- regexp.MatchString(<rule-set DFA x>, string r[a])
    VM_REGEXD = 30,  // d <- regexp.MatchString(string r[a], string r[b]): pattern DFA from the batch's rxof table
    VM_REGEXR = 31,  // d <- regexp.MatchString(<rule-set DFA r[b]>, string r[a])   (templates: hoisted REGEX)
    VM_HEAP = 32,    // reference heap count r[d] (rules that can reach slot 63, lower.cpp): y = 1 checked
                     // allocation (r[d] == 63 -> "heap overflow"); r[d] >= 64 -> index panic; else r[d]++
};

// Leading-atom guard of a rule (vmopt.cpp): the rule's program starts with
//   RES col (want S/B/I/D) | VCOL col ; EQK K ; [NOT]
// followed by a decision.  The kernel evaluates the guards of a whole 32-rule group with vector
// compares and runs the VM (from `cont`) only for lanes the guard leaves undecided.
enum mxp_guard_mode {
    GM_NONE = 0,  // run the whole program
    GM_AND = 1,   // atom false -> result false; atom true -> continue at cont
    GM_ONLY = 2,  // result = atom
    GM_OR = 3,    // atom true -> result true; atom false -> continue at cont
};
#define GK_VCOL 5  // guard kind: virtual map[key] column (else a want class W_S..W_D)
#define GT_PREFIX (1u << 9)  // mxp_guard.mode flag: the atom is `column startsWith K` (K = string id)

typedef struct mxp_guard {
    uint32_t col;    // column index (resolve or virtual); bits 24..31: kind (W_* or GK_VCOL)
    uint32_t mode;   // bits 0..7 mode, bit 8 negate, bit 9 GT_PREFIX, 16..31 continuation pc
    uint32_t klo;    // constant (register value) compared against
    uint32_t khi;
} mxp_guard;

// Per 32-rule group: the guard masks the kernel's phase 1 works with (bit k = rule 32 g + k), and
// the group's guarded rules split into column segments (the rules whose guard reads the same
// column with the same want class), so each segment loads its column once per request and compares
// its rules' constants (kargs.gk[32 g + k]) against it.
typedef struct mxp_rgroup {
    uint32_t all;      // rules present in the group
    uint32_t guarded;  // mode != GM_NONE
    uint32_t only;     // GM_ONLY
    uint32_t orm;      // GM_OR  (GM_AND = guarded & ~only & ~orm)
    uint32_t neg;      // negated atoms
    uint32_t indexed;  // rules whose continuing pairs come from the guard index (mxp_index_kernel)
    uint32_t seg0;     // segments 1 .. nseg-1 are kargs.segs[seg0 .. seg0 + nseg - 2]
    uint32_t nseg;
    uint32_t s_col;    // segment 0, inline (mxp_seg fields)
    uint32_t s_okset;
    uint32_t s_rules;
    uint32_t s_cmp;
    uint32_t id;       // group index g (rules 32 g .. 32 g + 31)
    uint32_t vm;       // 1: some rule can leave phase 1 with continuing lanes (mxp_eval_kernel)
    uint32_t pad[2];
} mxp_rgroup;           // 64 B: fetched four at a time by one wavefront-wide load

typedef struct mxp_seg {
    uint32_t col;      // column read by the guards of the segment
    uint32_t okset;    // bits 0..15: kinds that pass the want class; bits 24..31: want class / GK_VCOL
    uint32_t rules;    // rules of the group in this segment (all need the column's type check)
    uint32_t cmp;      // the subset whose atom phase 1 computes (indexed rules need no compare)
} mxp_seg;

// Guard index: for `attr == K && <continuation>` rules (GM_AND, not negated, templated), the pairs
// that continue are exactly the requests whose column value equals K.  Per (column, want class) an
// open-addressing hash table maps a value K to the rules guarded by it (a range of kargs.postings,
// sorted by template), so each request enumerates its own surviving rules instead of comparing
// against all of them.
typedef struct mxp_index {
    uint32_t col;
    uint32_t okset;    // as mxp_seg.okset (bits 0..15)
    uint32_t hmask;    // table size - 1 (power of two)
    uint32_t hoff;     // first entry in kargs.hents.  Prefix tables: pairs of entries {key bytes 0..3 |
                       // key string id, tag, start, len | min(|K|, 255) << 24}, {key bytes 4..19}: keys
                       // of <= 20 bytes inline
    uint32_t prefix;   // MXP_IX_EQ / MXP_IX_PREFIX / MXP_IX_COMPOSITE
    uint32_t plen0;    // prefix / composite: distinct key lengths kargs.plens[plen0 .. plen0 + nplen), ascending
    uint32_t nplen;
    uint32_t col2;     // composite: the prefix column (string want class)
    uint32_t okset2;
    uint32_t hmask2;   // composite table: pairs of entries {K2 word 0 | K2 string id, tag, start,
                       // len | min(|K2|, 255) << 24}, {K1 lo, K1 hi, K2 words 1, 2}: keys of <= 12 bytes inline
    uint32_t hoff2;
    uint32_t hslot;    // prefix / composite: the probed column's row in kargs.heads (MXP_VM_DONE: none)
    uint32_t tailk;    // prefix: some postings are `.*$` tail keys (code 508): the probe finds the
                       // subject's last '\n'
    uint32_t boff;     // prefix / composite: the pair table's occupancy bitmap at kargs.hbits[boff ..]
                       // (bit s: slot s holds a key), read before an entry pair
    uint32_t pad[2];
} mxp_index;           // 64 B

// index kinds.  Composite: rules `A == K1 && B.startsWith(K2) && ...` (vmopt.h SecondAtom), keyed by
// (K1, K2): a request probes its A value with B's leading bytes at every K2 length and resumes the
// rules it finds after both atoms (kargs.rule_tmpl2).  Requests whose B fails the string type check
// use the composite's equality table over K1 instead (hmask / hoff) and run the continuation after
// the first atom (kargs.rule_tmpl), which raises the reference's error.
#define MXP_IX_EQ 0u
#define MXP_IX_PREFIX 1u
#define MXP_IX_COMPOSITE 2u

typedef struct mxp_hent {
    uint32_t klo, khi; // equality: the key (column value register); prefix: string id of the key, hash tag
    uint32_t start;    // postings [start, start + len); len == 0: empty slot
    uint32_t len;
} mxp_hent;

// A chunk of consecutive lean groups whose rules are all served by guard indexes and whose guards all
// read one column: in phase 1 their words depend only on that column's kind (match 0, error where
// the guard's type check fails), so mxp_fill_kernel computes them once per request and streams the
// stores.  Groups g0 .. g0 + n - 1 (n <= MXP_FILL_CHUNK), `all` = rules present in every group but
// the last, `last` = those of the last.
#define MXP_FILL_CHUNK 16u
// columns < MXP_CC have LDS column-cache slots in the lean guard kernels (kargs.lean_cols)
#define MXP_CC 8u
typedef struct mxp_fill {
    uint32_t col;
    uint32_t okset;    // bits 0..15: kinds that pass; bits 24..31: want class / GK_VCOL (0xFFFF: every kind)
    uint32_t g0;
    uint32_t n;
    uint32_t moff;     // kargs.fill_masks[moff + i]: rules of group g0 + i this chunk writes
    uint32_t vt;       // 1: some group has value-class merge entries (mxp_vtfill_kernel)
    uint32_t pad[2];
} mxp_fill;

// Value classes (kernels.hip mxp_vt_*): at most MXP_VT_MAX columns per batch; per active slot a
// kargs.vt_meta[a * 8 + MXP_VTM_*]
#define MXP_VT_MAX 8
#define MXP_VTM_COL 0    // column
#define MXP_VTM_CAP 1    // class table capacity (power of two >= 64): classes are its slots
#define MXP_VTM_TBASE 2  // first (match, error) word pair in kargs.vt_tm: word j of class k at tbase + j * cap + k
#define MXP_VTM_KBASE 3  // first entry in kargs.vt_keys / vt_rep
#define MXP_VTM_NW 4     // bitmap words holding the slot's rules
#define MXP_VTM_WOFF 5   // first (group, rule mask) pair in kargs.vt_words
#define MXP_VT_EMPTY 0xFFFFFFFFFFFFFFFFull

// dense-rule injection slots (mxp_inject_kernel): 16 dwords = dense-id mask (2), bitmap word,
// entry count, up to 12 entries (bit | dense id << 5); a word with more entries takes several slots
#define MXP_INJ_SLOT 16u

// kargs.rule_tmpl value of indexed rules whose atom IS the result (`col.startsWith(K)` alone): a
// posting is a true pair, no continuation to run
#define MXP_TMPL_DIRECT 0xFFFFFFFEu
// ... a code-509 posting (a literal-key regexp rule's exact key) whose subject does not end there
#define MXP_TMPL_SKIP 0xFFFFFFFDu

#if defined(__HIPCC__)
#define MXP_HD __host__ __device__
#else
#define MXP_HD
#endif
// word-at-a-time byte-string hash (little-endian 8-byte words, zero beyond the end), shared by the
// prefix index builder (host) and the index kernel, which hashes a request's leading bytes
static inline MXP_HD uint64_t mxp_str_step(uint64_t h, uint64_t w) {
    h ^= w;
    h *= 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 31);
}
static inline MXP_HD uint64_t mxp_str_final(uint64_t h, uint64_t len) {
    h ^= len * 0xC2B2AE3D27D4EB4Full;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}
// composite keys: the hash of K2's bytes seeded with the A value (K1)
static inline MXP_HD uint64_t mxp_composite_seed(uint64_t k1) { return mxp_str_step(0x2545F4914F6CDD1Dull, k1); }
static inline uint64_t mxp_str_hash_seeded(uint64_t h, const uint8_t* p, uint64_t n) {
    for (uint64_t i = 0; i < n; i += 8) {
        uint64_t w = 0;
        for (uint64_t k = 0; k < 8 && i + k < n; k++) w |= (uint64_t)p[i + k] << (8 * k);
        h = mxp_str_step(h, w);
    }
    return mxp_str_final(h, n);
}
static inline uint64_t mxp_str_hash(const uint8_t* p, uint64_t n) { return mxp_str_hash_seeded(0, p, n); }

static inline MXP_HD uint32_t mxp_hash64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// class key of a column value: the value itself matters only for kind 1 (MXP_STRING / VC_VALUE,
// a string id); every other kind is one class per kind
static inline MXP_HD uint64_t mxp_vt_key(uint32_t kind, uint64_t v) {
    return kind == 1u ? ((1ull << 32) | (uint32_t)v) : ((uint64_t)kind << 32);
}

// Continuation templates: the continuations (code from the guard's cont pc) of many rules differ
// only in constants (C2: the path prefix and the ip literal).  Hoisting every constant operand
// into a register (EQK -> EQ, STRFNK -> STRFN, LOOKUPK -> LOOKUP, LOGICK -> LOGIC, CONST -> MOV)
// makes them byte-identical; such rules share one template program and keep only a per-rule
// constant vector, so survivors of DIFFERENT rules can run side by side in one wavefront.
typedef struct mxp_tmpl {
    uint32_t off;      // template code: prog[off - pc0 + pc] for pc >= pc0 (jump targets unchanged)
    uint32_t pc0;      // continuation start
    uint32_t len;      // program length (pcs < len)
    uint32_t nconst;   // constants per rule, loaded into registers creg0 .. creg0 + nconst - 1
    uint32_t creg0;
    uint32_t pad[3];
} mxp_tmpl;

// want classes for VM_RES / VM_TRES
enum mxp_vm_want { W_S = 0, W_B = 1, W_I = 2, W_D = 3, W_F = 4 };

// lookup modes
enum mxp_vm_lk { LK_N = 0 /* missing -> "" */, LK_TRY = 1 /* tlookup+jnz */, LK_ERR = 2 /* missing -> error */ };

// string functions (mixer/pkg/il/runtime/externs.go:108-128)
enum mxp_vm_sf { SF_MATCH = 0, SF_STARTS = 1, SF_ENDS = 2, SF_REGEX = 3 };

// per-pair result codes
enum mxp_pair_code { PC_FALSE = 0, PC_TRUE = 1, PC_ERROR = 2, PC_PANIC = 3 };

// error / panic codes recorded for error pairs (host formats the reference's text)
enum mxp_err_code {
    ERR_NONE = 0,
    ERR_LOOKUP = 1,      // "lookup failed: '%v'"                       aux = attr string id
    ERR_CONV_S = 2,      // "error converting value to string: '%v'"   aux = column
    ERR_CONV_B = 3,
    ERR_CONV_I = 4,
    ERR_CONV_D = 5,
    ERR_IP = 6,          // "could not convert %s to IP_ADDRESS"        aux = string id
    ERR_TS = 7,          // "could not convert '%s' to TIMESTAMP..."    aux = string id
    ERR_MEMBER = 8,      // "member lookup failed: '%v'"               aux = key string id
    ERR_REGEX = 9,       // regexp compile error ("error parsing regexp: ...")   aux = pattern string id
    ERR_STATIC = 10,     // rule failed to compile: every evaluation errors   aux = rule
    ERR_UNSUPPORTED = 11,// construct not lowered by this engine build   aux = rule
    ERR_UNDERFLOW = 12,  // "stack underflow" (interpreterRun.go:1148) -- reachable from OR chains
    ERR_REGEX_UNSUPPORTED = 13,  // batch pattern this engine cannot compile (Unicode classes / folding)   aux = pattern string id
    ERR_OVERFLOW = 14,   // "stack overflow" (interpreterRun.go:1145-1147)
    ERR_HEAP = 15,       // "heap overflow" (interpreterRun.go:1154-1156)
    PANIC_MAPTYPE = 32,  // il.MapGet on a non-map value ("Unknown map type")
    PANIC_EXTARG = 33,   // reflect.Call with a wrong dynamic type (ip_equal / timestamp_equal)
    PANIC_NOTBOOL = 34,  // Result.AsBool on a non-bool result
    PANIC_STATIC = 35,   // compile-time panic in the reference
    PANIC_CONV = 36,     // interface conversion: heap value is not a string
    PANIC_INDEX = 37,    // Go "index out of range": heap slot 64 (after an extern's unchecked allocation)
                         // or a result word past the 64-word stack (interpreterRun.go:899-900)
};

// 16-byte instruction; loaded with one scalar s_load_dwordx4 per step.
typedef struct mxp_vm_ins {
    uint8_t op;   // mxp_vm_op | MXP_VM_WAKE
    uint8_t d;
    uint8_t a;
    uint8_t b;
    uint32_t x;
    uint32_t y;
    uint32_t z;
} mxp_vm_ins;

// F-handle (interface{} register value): kind (mxp_kind) in bits 56..63, id in bits 0..55.
#define MXP_FH(kind, id) ((((uint64_t)(kind)) << 56) | ((uint64_t)(id) & 0x00FFFFFFFFFFFFFFull))
#define MXP_FH_KIND(h) ((uint32_t)((h) >> 56))
#define MXP_FH_ID(h) ((h) & 0x00FFFFFFFFFFFFFFull)
// []byte ids: canonical (net.IP.Equal) class in bits 28..55, exact bytes in bits 0..27
#define MXP_BYTES_CANON(id) ((id) >> 28)
#define MXP_BYTES_RAW(id) ((id) & 0x0FFFFFFFull)
#define MXP_BYTES_ID(canon, raw) ((((uint64_t)(canon)) << 28) | (uint64_t)(raw))

// virtual-column kinds (VM_VCOL)
enum mxp_vcol_kind { VC_ABSENT = 0, VC_VALUE = 1, VC_NOTMAP = 3 };

// referenced-attribute record (mxp_eval_refs): an attribute read by the VM for (req, rule).
// slot: a column index (VM_RES / VM_TRES / VM_VCOL; key = MXP_VM_DONE), or MXP_REF_LOOKUP | found |
// batch map id for a map lookup (VM_LOOKUP[K]; key = the key's string id)
#define MXP_REF_LOOKUP 0x80000000u
#define MXP_REF_FOUND 0x40000000u
#define MXP_REF_MAPID 0x3FFFFFFFu
typedef struct mxp_ref_rec {
    uint32_t req;
    uint32_t rule;
    uint32_t slot;
    uint32_t key;
} mxp_ref_rec;

// error log record (one per error pair, capacity-bounded)
typedef struct mxp_err_rec {
    uint32_t req;
    uint32_t rule;
    uint32_t code;
    uint32_t aux;
} mxp_err_rec;
