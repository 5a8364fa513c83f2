// kernels.hip -- gfx950 kernels of the MXP predicate engine.
//
// mxp_eval_kernel: the batched replacement of the reference's per-(bag, rule) evaluation loop
//   resolver.filterActions (mixer/pkg/runtime/resolver.go:202-238)
//     -> evaluator.IL.EvalPredicate (mixer/pkg/il/evaluator/evaluator.go:75)
//       -> interpreter.run (mixer/pkg/il/interpreter/interpreterRun.go:18-1163)
// executed as a wave-uniform bytecode VM (vm.h):
//   * a workgroup owns a tile of 64 requests (one per lane) and its 4 wavefronts sweep disjoint
//     32-rule groups, so every wave runs ONE rule's program at a time: the opcode stream is scalar
//     (s_load_dwordx4 per step) and only operand data is per-lane;
//   * short-circuit jumps are forward-only: a lane that jumps parks with a wait target, and the
//     wave skips straight to min(wait) once no lane is live;
//   * the reference's stack slots live in an LDS register file regs[reg][thread] (8-byte stride per
//     lane -> conflict-free ds_read_b64 / ds_write_b64);
//   * results are accumulated per lane into 32-rule words and written rule-word-major
//     (out[word * N + request]) so every store is a coalesced 256-byte wave store.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mxp_batch.h"
#include "kargs.h"
#include "pack_args.h"
#include "vm.h"

namespace {

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return uni(v);
}

struct StrRef {
    const uint8_t* p;
    uint32_t n;
};

__device__ __forceinline__ StrRef str_of(const mxp_kargs& A, uint64_t id) {
    const bool g = id < A.n_gstr;
    const uint64_t d = g ? A.gstr_off[id] : A.bstr_off[id - A.n_gstr];
    StrRef r;
    r.p = (g ? A.gstr : A.bstr) + (d >> 24);
    r.n = (uint32_t)(d & 0xFFFFFFu);
    return r;
}

// 8 bytes at any address of a string pool (pools are 8-aligned with 16 bytes of tail slack)
__device__ __forceinline__ uint64_t ld8(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7) * 8u;
    const uint64_t lo = q[0];
    return sh == 0 ? lo : (lo >> sh) | (q[1] << (64u - sh));
}

// 8 bytes at an 8-aligned address (string starts in the pools, and whole words after them)
__device__ __forceinline__ uint64_t ld8a(const uint8_t* p) { return *(const uint64_t*)p; }

// equality of n bytes at two 8-aligned addresses
__device__ __forceinline__ bool bytes_eq_a(const uint8_t* a, const uint8_t* b, uint32_t n) {
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8)
        if (ld8a(a + i) != ld8a(b + i)) return false;
    if (i == n) return true;
    const uint64_t mask = (1ull << ((n - i) * 8u)) - 1ull;
    return ((ld8a(a + i) ^ ld8a(b + i)) & mask) == 0;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8)
        if (ld8(a + i) != ld8(b + i)) return false;
    if (i == n) return true;
    const uint64_t mask = (1ull << ((n - i) * 8u)) - 1ull;
    return ((ld8(a + i) ^ ld8(b + i)) & mask) == 0;
}

// match / startsWith / endsWith (mixer/pkg/il/runtime/externs.go:108-128)
__device__ bool strfn(uint32_t fn, StrRef s, StrRef p) {
    if (fn == SF_STARTS) return s.n >= p.n && bytes_eq(s.p, p.p, p.n);
    if (fn == SF_ENDS) return s.n >= p.n && bytes_eq(s.p + (s.n - p.n), p.p, p.n);
    // SF_MATCH: trailing '*' -> prefix, else leading '*' -> suffix, else equality
    if (p.n > 0 && p.p[p.n - 1] == '*') return s.n >= p.n - 1 && bytes_eq(s.p, p.p, p.n - 1);
    if (p.n > 0 && p.p[0] == '*') return s.n >= p.n - 1 && bytes_eq(s.p + (s.n - (p.n - 1)), p.p + 1, p.n - 1);
    return s.n == p.n && bytes_eq(s.p, p.p, p.n);
}

__device__ __forceinline__ void log_err(const mxp_kargs& A, uint32_t req, uint32_t rule, uint32_t code, uint32_t aux) {
    if (!A.errlog) return;
    // (errcount[3]: some record is a conversion error, whose text prints the caller's value -- the
    // host then collects the records at once instead of when a text is asked for)
    if (code >= ERR_CONV_S && code <= ERR_CONV_D) atomicOr(A.errcount + 3, 1u);
    uint32_t slot = atomicAdd(A.errcount, 1u);
    if (slot < A.errcap) {
        mxp_err_rec r;
        r.req = req;
        r.rule = rule;
        r.code = code;
        r.aux = aux;
        A.errlog[slot] = r;
    }
}

// a true pair found after phase 1 (guard-index kernel): OR its match bit in and, when the caller
// asked for fused hit counters, count it.  Each (rule, request) pair is produced once per
// evaluation (a rule sits in one index under one key; the composite and its equality fallback serve
// disjoint lanes; aliases are distinct rules), so neither atomic needs its return value: no
// round trip per true pair.
// fused hit counters on for this evaluation (kargs.hits_gate: a uniform scalar load)
__device__ __forceinline__ bool counting(const mxp_kargs& A) {
    return A.hits && (!A.hits_gate || *A.hits_gate != 0u);
}

// Deferred pairs (kargs.dtp_ent): the index kernel runs before the value-class fill, so a true or
// error pair is recorded in its wave's list (LDS counter; the wave of request q is q / 64, and every
// pair of q is produced by that wave) and OR-ed in by the fill as it streams the words out.  Pairs
// past a wave's dtp_cap go to the overflow list (OR-ed in after the fill by the gated index launch);
// past that list's capacity a flag re-runs the index kernel with plain OR-s after the fill.
__shared__ uint32_t g_dtpn[4];  // entries per wave of the index kernel's workgroup
__device__ __forceinline__ void dtp_push(const mxp_kargs& A, uint32_t rule, uint32_t req, uint32_t plane) {
    const uint32_t slot = atomicAdd(&g_dtpn[threadIdx.x >> 6], 1u);
    if (slot < A.dtp_cap) {
        A.dtp_ent[(uint64_t)(req >> 6) * A.dtp_cap + slot] = rule | (plane << 23) | ((req & 63u) << 24);
        return;  // (a true pair in a wave list is counted by mxp_dtp_sort_kernel)
    }
    // past the wave list (histogram counting): counted here, the sort kernel never sees it
    if (plane == 0u && A.dtp_part && counting(A))
        __hip_atomic_fetch_add(A.hits + rule, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t o = atomicAdd(&A.dtp_ovf_n[0], 1u);
    if (o < A.dtp_ovf_cap) {
        A.dtp_ovf[2ull * o] = req;
        A.dtp_ovf[2ull * o + 1] = rule | (plane << 31);
    } else {
        __hip_atomic_store(&A.dtp_ovf_n[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <bool kDtp = false>
__device__ __forceinline__ void set_true1(const mxp_kargs& A, uint32_t rule, uint32_t req) {
    const uint32_t bit = 1u << (rule & 31u);
    if (kDtp) {
        dtp_push(A, rule, req, 0u);
        // counted per pair here, or where the pair is filed (kargs.dtp_part: mxp_dtp_sort_kernel's
        // histogram, dtp_push past the wave list)
        if (!A.dtp_part && counting(A)) __hip_atomic_fetch_add(A.hits + rule, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __hip_atomic_fetch_or(A.out_match + (uint64_t)(rule >> 5) * A.n + req, bit, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    if (counting(A)) __hip_atomic_fetch_add(A.hits + rule, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ... and the same for the rule's aliases (indexed duplicates of its program, kargs.alias_off)
// returns the number of pairs set
template <bool kDtp = false>
__device__ __forceinline__ uint32_t set_true(const mxp_kargs& A, uint32_t rule, uint32_t req) {
    if (!A.out_match) return 0;
    set_true1<kDtp>(A, rule, req);
    uint32_t c = 1;
    if (A.alias_off)
        for (uint32_t j = A.alias_off[rule]; j < A.alias_off[rule + 1]; j++, c++) set_true1<kDtp>(A, A.aliases[j], req);
    return c;
}

// an error pair found by the guard-index kernel, with its aliases
__shared__ uint8_t g_rerr[4][64];  // deferred-pair index kernel: its tile's request error flags (kargs.req_err_init)
template <bool kDtp = false>
__device__ __forceinline__ void set_error(const mxp_kargs& A, uint32_t rule, uint32_t req) {
    if (A.req_err) {
        if constexpr (kDtp) {
            if (A.req_err_init) g_rerr[threadIdx.x >> 6][req & 63u] = 1;  // (the wave's own tile)
            else A.req_err[req] = 1;
        } else {
            A.req_err[req] = 1;
        }
    }
    if (!A.out_err) return;
    if (kDtp) {
        dtp_push(A, rule, req, 1u);
        if (A.alias_off)
            for (uint32_t j = A.alias_off[rule]; j < A.alias_off[rule + 1]; j++) dtp_push(A, A.aliases[j], req, 1u);
        return;
    }
    atomicOr(A.out_err + (uint64_t)(rule >> 5) * A.n + req, 1u << (rule & 31u));
    if (A.alias_off)
        for (uint32_t j = A.alias_off[rule]; j < A.alias_off[rule + 1]; j++) {
            const uint32_t r = A.aliases[j];
            atomicOr(A.out_err + (uint64_t)(r >> 5) * A.n + req, 1u << (r & 31u));
        }
}

// constant-address-space views: uniform loads through them become scalar s_load_dwordxN
typedef __attribute__((address_space(4))) const uint32_t cuint32;

// Referenced-attribute tracking (mxp_eval_refs): one record per attribute read the VM performs
// (VM_RES / VM_TRES / VM_VCOL: slot = column; VM_LOOKUP[K]: the map key), appended with one atomic
// per wavefront.  Records past refcap are counted, not stored (the host re-runs with more room).
__device__ __forceinline__ void ref_rec(const mxp_kargs& A, bool on, uint32_t req, uint32_t rule, uint32_t slot,
                                        uint32_t key) {
    const uint64_t m = __ballot(on);
    if (!m) return;
    const uint32_t lane = __lane_id();
    const uint32_t first = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(A.refcount, (uint32_t)__builtin_popcountll(m));
    base = __builtin_amdgcn_readlane(base, first);
    if (on) {
        const uint32_t i = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (i < A.refcap) A.refs[i] = mxp_ref_rec{req, rule, slot, key};
    }
}

// Runs one program from `pc0` for the lanes in `live` (the others keep their phase-1 result) and
// returns the pair code of every lane that ran.  The program is wave-uniform: instruction pc is
// P[pc] (pc in [pc0, len)), fetched with one scalar s_load_dwordx4 per step.  `rule` may differ
// per lane (template batches of the guard-index kernel); it only names the pair in error records and
// Eval results.  The register file is regs[reg][thread] in LDS.
// kLite: the continuation-template instantiation for rule sets whose index templates hold no map
// lookups, virtual columns or regexps (Plan::tmpl_lite) -- without those cases the index kernel
// needs far fewer registers
template <bool kRefs, bool kNfa = kRefs, bool kLite = false>
__device__ uint32_t run_rule(const mxp_kargs& A, cuint32* P, uint32_t len, uint32_t pc0, bool live, uint32_t rule,
                             uint32_t req, uint64_t (*regs)[256], uint32_t tid, bool fan = false) {
#define REG(i) regs[i][tid]
    const uint64_t N = A.n;
    uint32_t wait = live ? pc0 : MXP_VM_DONE;
    uint32_t res = PC_FALSE;
    uint32_t ecode = ERR_NONE, eaux = 0;  // the lane's error (logged once, after the loop)
    uint32_t pc = pc0;

#define FAIL(code_, aux_)                                   \
    do {                                                    \
        res = ((code_) >= 32u) ? PC_PANIC : PC_ERROR;       \
        ecode = (code_);                                    \
        eaux = (aux_);                                      \
        live = false;                                       \
        wait = MXP_VM_DONE;                                 \
    } while (0)
#define JUMP(t_)             \
    do {                     \
        live = false;        \
        wait = (t_);         \
    } while (0)
#define FINISH(code_)         \
    do {                      \
        res = (code_);        \
        live = false;         \
        wait = MXP_VM_DONE;   \
    } while (0)
#define FINISHV(code_)                                                              \
    do {                                                                            \
        if (A.out_vals) A.out_vals[(uint64_t)req * A.n_rules + rule] = (code_);     \
        FINISH(code_);                                                              \
    } while (0)

    while (pc < len) {
        cuint32* ip = P + (uint64_t)pc * 4u;
        const uint32_t w0 = uni(ip[0]);
        const uint32_t x = uni(ip[1]), y = uni(ip[2]), z = uni(ip[3]);
        const uint32_t op = w0 & 0x7Fu;
        const uint32_t d = (w0 >> 8) & 0xFFu, a = (w0 >> 16) & 0xFFu, b = w0 >> 24;
        if (w0 & MXP_VM_WAKE) live = live || (wait == pc);
        if (__ballot(live) == 0) {
            pc = wave_min(wait);
            if (pc == MXP_VM_DONE) break;
            continue;
        }
        switch (op) {
        case VM_RES:
        case VM_TRES: {
            if constexpr (kRefs) ref_rec(A, live, req, rule, x, MXP_VM_DONE);
            if (live) {
                const uint64_t at = (uint64_t)x * N + req;
                const uint32_t k = A.kinds[at];
                uint64_t v = A.vals[at];
                bool ok;
                switch (y) {
                case W_S: ok = k == MXP_STRING; break;
                case W_B: ok = k == MXP_BOOL; break;
                case W_I: ok = k == MXP_INT64 || k == MXP_DURATION; break;
                case W_D: ok = k == MXP_DOUBLE; break;
                default: ok = k != MXP_ABSENT; v = MXP_FH(k, v); break;
                }
                if (k == MXP_ABSENT) {
                    if (op == VM_RES) FAIL(ERR_LOOKUP, z);
                } else if (!ok) {
                    FAIL(ERR_CONV_S + y, x);
                } else {
                    REG(d) = v;
                    if (op == VM_TRES) JUMP(z);
                }
            }
            break;
        }
        case VM_VCOL: {
            if constexpr (kLite) break;
            if constexpr (kRefs) ref_rec(A, live, req, rule, x, MXP_VM_DONE);
            if (live) {
                const uint64_t at = (uint64_t)x * N + req;
                const uint32_t k = A.kinds[at];
                if (k == VC_VALUE) REG(d) = A.vals[at];
                else if (k == VC_ABSENT) FAIL(ERR_LOOKUP, z);
                else FAIL(PANIC_MAPTYPE, 0);
            }
            break;
        }
        case VM_CONST:
            if (live) REG(d) = (uint64_t)y | ((uint64_t)z << 32);
            break;
        case VM_EQ:
            if (live) REG(d) = REG(a) == REG(b) ? 1u : 0u;
            break;
        case VM_EQK:
            if (live) REG(d) = REG(a) == ((uint64_t)y | ((uint64_t)z << 32)) ? 1u : 0u;
            break;
        case VM_NOT:
            if (live) REG(d) = REG(a) == 0 ? 1u : 0u;
            break;
        case VM_LOGIC:
        case VM_LOGICK:
            if (live) {
                const uint64_t p = REG(a);
                const uint64_t q = op == VM_LOGIC ? REG(b) : (uint64_t)x;
                // interpreterRun.go:352-443 operate on u32 words
                const bool pb = (uint32_t)p != 0, qb = (uint32_t)q != 0;
                REG(d) = (y == 0 ? (pb && qb) : y == 1 ? (pb || qb) : (pb != qb)) ? 1u : 0u;
            }
            break;
        case VM_JZ:
            if (live && (uint32_t)REG(a) == 0) JUMP(z);
            break;
        case VM_JNZ:
            if (live && (uint32_t)REG(a) != 0) JUMP(z);
            break;
        // folded bool results (vmopt.cpp): y is PC_FALSE / PC_TRUE, i.e. also the value 0 / 1
        case VM_JZRET:
            if (live && (uint32_t)REG(a) == 0) FINISHV(y);
            break;
        case VM_JNZRET:
            if (live && (uint32_t)REG(a) != 0) FINISHV(y);
            break;
        case VM_RETK:
            if (live) FINISHV(y);
            break;
        case VM_JMP:
            if (live) JUMP(z);
            break;
        case VM_RET:
            if (live) {
                const uint64_t v = REG(a);
                if (A.out_vals) A.out_vals[(uint64_t)req * A.n_rules + rule] = v;
                if (y == 1) {
                    FINISH((uint32_t)v != 0 ? PC_TRUE : PC_FALSE);
                } else if (A.out_vals) {
                    FINISH(PC_FALSE);  // Eval: a non-bool result is just a value
                } else {
                    FAIL(PANIC_NOTBOOL, 0);  // EvalPredicate: Result.AsBool panics (result.go:42-52)
                }
            }
            break;
        case VM_LOOKUP:
        case VM_LOOKUPK: {
            if constexpr (kLite) break;
            bool rec = false;
            uint32_t rslot = 0, rkey = 0;
            if (live) {
                const uint64_t h = REG(a);
                const uint32_t key = op == VM_LOOKUP ? (uint32_t)REG(b) : x;
                if (MXP_FH_KIND(h) != MXP_STRING_MAP) {
                    FAIL(PANIC_MAPTYPE, 0);
                } else {
                    const uint32_t m = (uint32_t)MXP_FH_ID(h);
                    const uint32_t e0 = A.map_off[m], e1 = A.map_off[m + 1];
                    uint32_t found = MXP_VM_DONE;
                    for (uint32_t e = e0; e < e1; e++)
                        if (A.map_keys[e] == key) {
                            found = A.map_vals[e];
                            break;
                        }
                    rec = true;
                    rslot = MXP_REF_LOOKUP | (found != MXP_VM_DONE ? MXP_REF_FOUND : 0u) | (m & MXP_REF_MAPID);
                    rkey = key;
                    if (found != MXP_VM_DONE) {
                        REG(d) = found;
                        if (y == LK_TRY) JUMP(z);
                    } else if (y == LK_N) {
                        REG(d) = A.empty_sid;
                    } else if (y == LK_ERR) {
                        FAIL(ERR_MEMBER, key);
                    }
                }
            }
            if constexpr (kRefs) ref_rec(A, rec, req, rule, rslot, rkey);
            break;
        }
        case VM_STRFN:
        case VM_STRFNK:
            if (live) {
                const StrRef s = str_of(A, REG(a));
                const StrRef p = str_of(A, op == VM_STRFN ? REG(b) : (uint64_t)x);
                REG(d) = strfn(y, s, p) ? 1u : 0u;
            }
            break;
        case VM_IPOF:
        case VM_TSOF:
            if (live) {
                const uint64_t sid = REG(a);
                const uint64_t h = (op == VM_IPOF ? A.ipof : A.tsof)[sid];
                if (h == ~0ull) FAIL(op == VM_IPOF ? ERR_IP : ERR_TS, (uint32_t)sid);
                else REG(d) = h;
            }
            break;
        case VM_IPEQ:
        case VM_TSEQ:
            if (live) {
                const uint64_t p = REG(a), q = REG(b);
                const uint32_t want = op == VM_IPEQ ? MXP_BYTES : MXP_TIMESTAMP;
                if (MXP_FH_KIND(p) != want || MXP_FH_KIND(q) != want) FAIL(PANIC_EXTARG, 0);
                else if (op == VM_IPEQ)  // net.IP.Equal: same canonical class
                    REG(d) = MXP_BYTES_CANON(MXP_FH_ID(p)) == MXP_BYTES_CANON(MXP_FH_ID(q)) ? 1u : 0u;
                else  // time.Time.Equal: same instant
                    REG(d) = MXP_FH_ID(p) == MXP_FH_ID(q) ? 1u : 0u;
            }
            break;
        case VM_ERR:
            if (live) FAIL(y, z);
            break;
        case VM_FTOS:
            if (live) {
                const uint64_t h = REG(a);
                if (MXP_FH_KIND(h) != MXP_STRING) FAIL(PANIC_CONV, 0);
                else REG(d) = MXP_FH_ID(h);
            }
            break;
        case VM_STOF:
            if (live) REG(d) = MXP_FH(MXP_STRING, REG(a));
            break;
        case VM_MOV:
            if (live) REG(d) = REG(a);
            break;
        case VM_HEAP:  // reference heap count (only rules that can reach slot 63 carry it)
            if (live) {
                const uint64_t h = REG(d);
                if (y != 0u && h == 63u) FAIL(ERR_HEAP, 0);
                else if (h >= 64u) FAIL(PANIC_INDEX, 0);
                else REG(d) = h + 1u;
            }
            break;
        case VM_REGEX:
        case VM_REGEXR:
        case VM_REGEXD:
            if (kLite) break;
            if (live) {
                // one stepping loop for the three forms (a single inlined copy of the DFA walk)
                // the set is chosen by value (a pointer into the by-value kernarg block would spill
                // the whole block to scratch)
                const bool bat = op == VM_REGEXD;
                const mxp_dfa_set S{bat ? A.rx_batch.hdr : A.rx.hdr, bat ? A.rx_batch.trans : A.rx.trans,
                                    bat ? A.rx_batch.ascii : A.rx.ascii, bat ? A.rx_batch.hilo : A.rx.hilo,
                                    bat ? A.rx_batch.hicls : A.rx.hicls, A.rx.nfa_scratch, A.rx.nfa_busy,
                                    A.rx.nfa_nslots, A.rx.nfa_wmax};
                uint32_t dfa = x;
                uint64_t subj = REG(a);
                bool run = true;
                if (op == VM_REGEXR) {
                    dfa = (uint32_t)REG(b);
                } else if (op == VM_REGEXD) {
                    const uint64_t psid = REG(a);
                    dfa = A.rxof[psid];
                    subj = REG(b);
                    if (dfa == MXP_RXOF_SYNTAX || dfa == MXP_RXOF_UNSUPPORTED) {
                        FAIL(dfa == MXP_RXOF_SYNTAX ? ERR_REGEX : ERR_REGEX_UNSUPPORTED, (uint32_t)psid);
                        run = false;
                    }
                }
                if (run) {
                    const StrRef sub = str_of(A, subj);
                    // (over-budget patterns run the bit-parallel NFA: only the kNfa instantiations,
                    // launched for rule sets and batches that have one, carry its registers)
                    if constexpr (kNfa)
                        REG(d) = mxp_rx_run(S, dfa, sub.p, sub.n) ? 1u : 0u;
                    else
                        REG(d) = mxp_dfa_run(S, dfa, sub.p, sub.n) ? 1u : 0u;
                }
            }
            break;
        default:
            break;
        }
        pc++;
    }
#undef FAIL
#undef JUMP
#undef FINISH
#undef FINISHV
#undef REG
    if (ecode != ERR_NONE && A.errlog) {
        log_err(A, req, rule, ecode, eaux);
        if (fan && A.alias_off)
            for (uint32_t j = A.alias_off[rule]; j < A.alias_off[rule + 1]; j++) log_err(A, req, A.aliases[j], ecode, eaux);
    }
    return res;
}

}  // namespace

// Phase 1 (guards) + phase 2 (VM for undecided lanes) over 32-rule groups.
namespace {

typedef __attribute__((address_space(4))) const uint64_t cuint64;

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off, 64);
    return uni(v);
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, off, 64);
        if (lane >= (uint32_t)off) v += t;
    }
    return v;
}

// Bits k of `rules` whose guard constant K[k] equals this lane's column value.  Wide segments
// compare against all 32 constants (scalar-loaded, one v_cmp_eq_u64 + select each); narrow ones
// walk their rule bits.
__device__ __forceinline__ uint32_t seg_eq(cuint64* K, uint32_t rules, uint64_t cv) {
    uint32_t eq = 0;
    if (__builtin_popcount(rules) >= 8) {
        for (int c = 0; c < 32; c += 8) {
            if (((rules >> c) & 0xFFu) == 0) continue;
#pragma unroll
            for (int k = 0; k < 8; k++) eq |= (cv == K[c + k]) ? (1u << (c + k)) : 0u;
        }
        return eq & rules;
    }
    for (uint32_t r = rules; r; r &= r - 1) {
        const uint32_t k = __builtin_ctz(r);
        eq |= (cv == K[k]) ? (1u << k) : 0u;
    }
    return eq;
}

// Error records of the rules whose guard column failed for this lane (missing attribute, wrong
// dynamic type, map attribute that is not a map): the same codes the VM's RES / VCOL raise.
__device__ __forceinline__ void log_guard_errors(const mxp_kargs& A, uint32_t e, uint32_t r0, uint32_t req) {
    for (uint32_t bits = e; bits; bits &= bits - 1) {
        const uint32_t r = r0 + __builtin_ctz(bits);
        const mxp_guard G = A.guards[r];
        const uint32_t col = G.col & 0xFFFFFFu, gk = G.col >> 24;
        const uint32_t ck = A.kinds[(uint64_t)col * A.n + req];
        uint32_t code, aux;
        if (gk == GK_VCOL) {
            code = ck == VC_ABSENT ? ERR_LOOKUP : PANIC_MAPTYPE;
            aux = 0;
        } else {
            code = ck == MXP_ABSENT ? ERR_LOOKUP : ERR_CONV_S + gk;
            aux = col;
        }
        if (code == ERR_LOOKUP) aux = A.prog[A.rule_off[r]].z;
        log_err(A, req, r, code, aux);
    }
}

// Value classes: the words of group g's class-served rules for one request -- per merge entry
// (active slot a, word position j) the class word of the request's class in that slot.
__device__ __forceinline__ void vt_words_of(const mxp_kargs& A, uint32_t g, uint32_t req, bool valid, uint32_t& vm,
                                            uint32_t& ve) {
    vm = ve = 0;
    const uint32_t i0 = uni(A.gvt_off[g]), i1 = uni(A.gvt_off[g + 1]);
    for (uint32_t i = i0; i < i1; i++) {
        const uint32_t ent = uni(A.gvt[i]);
        const uint32_t a = ent >> 24, j = ent & 0xFFFFFFu;
        const uint32_t cap = uni(A.vt_meta[a * 8u + MXP_VTM_CAP]), tb = uni(A.vt_meta[a * 8u + MXP_VTM_TBASE]);
        if (valid) {
            const uint32_t k = A.vt_cls[(uint64_t)a * MXP_VT_PITCH(A.n) + req];
            const uint2 w = *(const uint2*)(A.vt_tm + 2u * ((uint64_t)tb + (uint64_t)j * cap + k));
            vm |= w.x;
            ve |= w.y;
        }
    }
}

// value-class error pairs are not logged per pair (the host expands the class records): count them
// (errcount[1]), c per lane
__device__ __forceinline__ void vt_count_n(const mxp_kargs& A, uint32_t c) {
    if (!A.errlog || !__ballot(c != 0)) return;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off, 64);
    if (__lane_id() == 0) atomicAdd(A.errcount + 1, c);
}
__device__ __forceinline__ void vt_count_errors(const mxp_kargs& A, uint32_t ve) {
    vt_count_n(A, (uint32_t)__builtin_popcount(ve));
}

}  // namespace

// Phase 1 + in-wave phase 2 over 32-rule groups.
//
// Workgroup = 4 wavefronts over one tile of 64 requests (one per lane); wave w takes
// `groups_per_wave` consecutive entries of the group list (kargs.glist).  Per group:
//   phase 1  every rule's leading atom at once: each column segment loads its column value once per
//            lane and compares it with the segment's constants (scalar operands), giving per lane the
//            32-bit words eq / ok; the group's mode masks turn them into match / error / continue
//            words with a handful of bit operations;
//   phase 2  (kVM only) the VM runs, rule by rule, for the continuing lanes -- indexed rules
//            excepted: their continuing pairs are enumerated by mxp_index_kernel.
// The host splits the groups: those that can leave phase 1 with continuing lanes (rules without a
// guard, OR guards, non-indexed AND guards) go to mxp_eval_kernel (kVM), the rest to the lean
// mxp_guard_kernel, which carries no VM and so keeps far fewer registers.  Group descriptors are
// fetched four at a time with one vector load (lane 16 j + f = word f of the j-th group) and read
// back with v_readlane.  Results: one coalesced store per word and plane, out[g * N + request].
// Lean kernel's column cache: a group's segments alternate between columns (C4: the path and five
// header columns), so instead of reloading a column whenever the segment's column changes, each
// thread keeps the (kind, value) of columns < MXP_CC it has loaded in LDS slots of its own.
__shared__ uint64_t g_ccv[MXP_CC][256];
__shared__ uint8_t g_cck[MXP_CC][256];

template <bool kVM, bool kRefs = false, bool kNfa = kRefs>
__device__ __forceinline__ void eval_groups(const mxp_kargs& A, uint64_t (*regs)[256]) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = uni(tid >> 6);
    const uint32_t req = A.q0 + blockIdx.x * 64u + lane;
    const bool valid = req < A.q1;
    const uint64_t N = A.n;
    const uint32_t i0 = (blockIdx.y * 4u + wave) * A.groups_per_wave;
    const uint32_t i1 = min(i0 + A.groups_per_wave, A.n_glist);
    // Eval mode (out_vals) needs every result register: whole programs, no guards, no index
    const bool guards_on = !(A.out_vals || (A.flags & 2u));
    uint32_t cached = MXP_VM_DONE;
    uint32_t ck = MXP_ABSENT;
    uint64_t cv = 0;
    uint32_t have = 0;  // (lean kernel) columns in this thread's LDS slots -- wave-uniform
    for (uint32_t c0 = i0; c0 < i1; c0 += 4) {
        uint32_t D = 0;
        if (c0 + (lane >> 4) < i1) D = ((const uint32_t*)(A.groups + A.glist[c0 + (lane >> 4)]))[lane & 15u];
        const uint32_t cn = min(4u, i1 - c0);
        for (uint32_t j = 0; j < cn; j++) {
#define GF(f) __builtin_amdgcn_readlane(D, j * 16u + (f))
            const uint32_t all = GF(0), guarded = GF(1), only = GF(2), orm = GF(3), neg = GF(4), indexed = GF(5),
                           seg0 = GF(6), nseg = GF(7), g = GF(12);
            const uint32_t r0 = g * 32u;
            uint32_t m = 0, e = 0, cont = 0;
            if (guards_on) {
                // ---- phase 1
                uint32_t eq = 0, ok = 0;
                // segments 1..16 of the group: one vector load (lane 4 k + f = field f of segment k + 1),
                // read back with v_readlane -- instead of a chain of scalar loads, one per segment
                uint32_t SD = 0;
                if (nseg > 1 && lane < 4u * min(nseg - 1u, 16u)) SD = ((const uint32_t*)(A.segs + seg0))[lane];
                for (uint32_t s = 0; s < nseg; s++) {
                    uint32_t col, okset, rules, cmp;
                    if (s == 0) {
                        col = GF(8);
                        okset = GF(9);
                        rules = GF(10);
                        cmp = GF(11);
                    } else if (s <= 16u) {
                        col = __builtin_amdgcn_readlane(SD, 4u * (s - 1u));
                        okset = __builtin_amdgcn_readlane(SD, 4u * (s - 1u) + 1u);
                        rules = __builtin_amdgcn_readlane(SD, 4u * (s - 1u) + 2u);
                        cmp = __builtin_amdgcn_readlane(SD, 4u * (s - 1u) + 3u);
                    } else {
                        const mxp_seg* S = A.segs + seg0 + s - 1;
                        col = uni(S->col);
                        okset = uni(S->okset);
                        rules = uni(S->rules);
                        cmp = uni(S->cmp);
                    }
                    if (col != cached) {
                        cached = col;
                        if (!kVM && col < MXP_CC && ((have >> col) & 1u)) {
                            ck = g_cck[col][tid];
                            cv = g_ccv[col][tid];
                        } else {
                            if (valid) {
                                ck = A.kinds[(uint64_t)col * N + req];
                                cv = A.vals[(uint64_t)col * N + req];
                            }
                            if (!kVM && col < MXP_CC) {
                                have |= 1u << col;
                                g_cck[col][tid] = (uint8_t)ck;
                                g_ccv[col][tid] = cv;
                            }
                        }
                    }
                    ok |= ((okset >> ck) & 1u) ? rules : 0u;
                    if (cmp) eq |= seg_eq((cuint64*)A.gk + r0, cmp, cv);
                }
#undef GF
                const uint32_t atom = eq ^ neg;
                const uint32_t andm = guarded & ~(only | orm);
                // indexed rules: atom unknown here (no compare), match 0, continuing pairs
                // enumerated by mxp_index_kernel
                m = atom & (only | orm) & ok;
                cont = (((atom & andm) | (~atom & orm)) & ok & ~indexed) | (all & ~guarded);
                e = guarded & ~ok;
                if (!valid) m = e = cont = 0;
                if (e && A.errlog) log_guard_errors(A, e, r0, req);
            } else {
                cont = valid ? all : 0u;
            }
            // ---- phase 2 (in-wave)
            if (kVM) {
                for (uint32_t bits = wave_or(cont); bits && !(A.flags & 1u); bits &= bits - 1) {
                    const uint32_t k = __builtin_ctz(bits);
                    const uint32_t bit = 1u << k;
                    const bool need = (cont & bit) != 0;
                    const uint32_t rule = r0 + k;
                    const uint32_t gm = uni(A.guards[rule].mode);
                    const uint32_t pc0 = (!guards_on || (gm & 0xFFu) == GM_NONE) ? 0u : (gm >> 16);
                    const uint32_t base = uni(A.rule_off[rule]);
                    const uint32_t len = uni(A.rule_off[rule + 1]) - base;
                    const uint32_t code = run_rule<kRefs, kNfa>(A, ((cuint32*)A.prog) + (uint64_t)base * 4u, len, pc0, need, rule,
                                                   req, regs, tid);
                    if (need) {
                        m |= code == PC_TRUE ? bit : 0u;
                        e |= code >= PC_ERROR ? bit : 0u;
                    }
                }
            }
            const uint32_t m_own = m;  // (value-class bits are counted per class, mxp_vt_eval_kernel)
            if (kVM && A.gvt_off) {  // value-class rules of the group (after the guard errors were logged)
                uint32_t vm, ve;
                vt_words_of(A, g, req, valid, vm, ve);
                vt_count_errors(A, ve);
                m |= vm;
                e |= ve;
            }
            if (valid) {
                if (A.out_match) A.out_match[(uint64_t)g * N + req] = m;
                if (A.out_err) A.out_err[(uint64_t)g * N + req] = e;
                if (A.req_err && e) A.req_err[req] = 1;
            }
            if (counting(A)) {
                // fused hit counters: per rule of the group, the lanes whose match bit is set
                const uint32_t mc = valid ? m_own : 0u;
                for (uint32_t bits = wave_or(mc); bits; bits &= bits - 1) {
                    const uint32_t k = __builtin_ctz(bits);
                    const uint32_t c = (uint32_t)__builtin_popcountll(__ballot((mc >> k) & 1u));
                    if (lane == 0) atomicAdd(A.hits + r0 + k, (unsigned long long)c);
                }
            }
        }
    }
}

extern "C" __global__ __launch_bounds__(256) void mxp_eval_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    eval_groups<true>(A, regs);
}

// mxp_eval_kernel for rule sets / batches with bit-parallel NFA regexps (kargs.nfa)
extern "C" __global__ __launch_bounds__(256) void mxp_eval_nfa_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    eval_groups<true, false, true>(A, regs);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void mxp_guard_kernel(mxp_kargs A) { eval_groups<false>(A, nullptr); }

// The lean groups with two requests per lane (a wave covers 128 requests): the kernel is bound by
// scalar issue, and the per-group scalar work -- descriptor decode, segment loop, branches -- is now
// spent once per 128 requests instead of once per 64 (C4 5.068 -> 4.850 ms per evaluation,
// profiles/r1_v18_ab_guard2.log).  The columns < MXP_CC the lean groups read are loaded into LDS
// once per workgroup and shared by its four waves (9 KB; 6 waves/SIMD): C4 4.87-4.90 -> 4.64-4.66
// ms, builds alternated (profiles/r1_v19_ab_guard2_shared_cache.log).  MXP_DEBUG_FLAGS 65536 =
// mxp_guard_kernel, one request per lane.
extern "C" __global__ __launch_bounds__(256) void mxp_guard2_kernel(mxp_kargs A) {
    __shared__ uint64_t ccv[MXP_CC][128];
    __shared__ uint8_t cck[MXP_CC][128];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = uni(tid >> 6);
    const uint32_t reqa = A.q0 + blockIdx.x * 128u + lane, reqb = reqa + 64u;
    const bool va = reqa < A.q1, vb = reqb < A.q1;
    const uint64_t N = A.n;
    const uint32_t i0 = (blockIdx.y * 4u + wave) * A.groups_per_wave;
    const uint32_t i1 = min(i0 + A.groups_per_wave, A.n_glist);
    // the workgroup's 128 requests, columns < MXP_CC the lean groups read (kargs.lean_cols):
    // loaded once into LDS, shared by the four waves
    const uint32_t have = uni(A.lean_cols) & ((1u << MXP_CC) - 1u);
    if (tid < 128u) {
        const uint32_t q = A.q0 + blockIdx.x * 128u + tid;
        for (uint32_t c = 0; c < MXP_CC; c++) {
            if (!((have >> c) & 1u)) continue;
            uint8_t k = MXP_ABSENT;
            uint64_t v = 0;
            if (q < A.q1) {
                k = A.kinds[(uint64_t)c * N + q];
                v = A.vals[(uint64_t)c * N + q];
            }
            cck[c][tid] = k;
            ccv[c][tid] = v;
        }
    }
    __syncthreads();
    uint32_t cached = MXP_VM_DONE;
    uint32_t cka = MXP_ABSENT, ckb = MXP_ABSENT;
    uint64_t cva = 0, cvb = 0;
    for (uint32_t c0 = i0; c0 < i1; c0 += 4) {
        uint32_t D = 0;
        if (c0 + (lane >> 4) < i1) D = ((const uint32_t*)(A.groups + A.glist[c0 + (lane >> 4)]))[lane & 15u];
        const uint32_t cn = min(4u, i1 - c0);
        for (uint32_t j = 0; j < cn; j++) {
#define GF(f) __builtin_amdgcn_readlane(D, j * 16u + (f))
            const uint32_t guarded = GF(1), only = GF(2), orm = GF(3), neg = GF(4), seg0 = GF(6), nseg = GF(7),
                           g = GF(12);
            const uint32_t r0 = g * 32u;
            uint32_t eqa = 0, oka = 0, eqb = 0, okb = 0;
            uint32_t SD = 0;
            if (nseg > 1 && lane < 4u * min(nseg - 1u, 16u)) SD = ((const uint32_t*)(A.segs + seg0))[lane];
            for (uint32_t sg = 0; sg < nseg; sg++) {
                uint32_t col, okset, rules, cmp;
                if (sg == 0) {
                    col = GF(8);
                    okset = GF(9);
                    rules = GF(10);
                    cmp = GF(11);
                } else if (sg <= 16u) {
                    col = __builtin_amdgcn_readlane(SD, 4u * (sg - 1u));
                    okset = __builtin_amdgcn_readlane(SD, 4u * (sg - 1u) + 1u);
                    rules = __builtin_amdgcn_readlane(SD, 4u * (sg - 1u) + 2u);
                    cmp = __builtin_amdgcn_readlane(SD, 4u * (sg - 1u) + 3u);
                } else {
                    const mxp_seg* S = A.segs + seg0 + sg - 1;
                    col = uni(S->col);
                    okset = uni(S->okset);
                    rules = uni(S->rules);
                    cmp = uni(S->cmp);
                }
                if (col != cached) {
                    cached = col;
                    if (col < MXP_CC && ((have >> col) & 1u)) {
                        cka = cck[col][lane];
                        cva = ccv[col][lane];
                        ckb = cck[col][64u + lane];
                        cvb = ccv[col][64u + lane];
                    } else {
                        cka = ckb = MXP_ABSENT;
                        cva = cvb = 0;
                        if (va) {
                            cka = A.kinds[(uint64_t)col * N + reqa];
                            cva = A.vals[(uint64_t)col * N + reqa];
                        }
                        if (vb) {
                            ckb = A.kinds[(uint64_t)col * N + reqb];
                            cvb = A.vals[(uint64_t)col * N + reqb];
                        }
                    }
                }
                oka |= ((okset >> cka) & 1u) ? rules : 0u;
                okb |= ((okset >> ckb) & 1u) ? rules : 0u;
                if (cmp) {
                    eqa |= seg_eq((cuint64*)A.gk + r0, cmp, cva);
                    eqb |= seg_eq((cuint64*)A.gk + r0, cmp, cvb);
                }
            }
#undef GF
            uint32_t ma = (eqa ^ neg) & (only | orm) & oka, mb = (eqb ^ neg) & (only | orm) & okb;
            uint32_t ea = guarded & ~oka, eb = guarded & ~okb;
            // (groups with value-class rules never come here: build_plan routes them to the VM kernel)
            if (va && A.errlog && ea) log_guard_errors(A, ea, r0, reqa);
            if (vb && A.errlog && eb) log_guard_errors(A, eb, r0, reqb);
            if (va) {
                if (A.out_match) A.out_match[(uint64_t)g * N + reqa] = ma;
                if (A.out_err) A.out_err[(uint64_t)g * N + reqa] = ea;
                if (A.req_err && ea) A.req_err[reqa] = 1;
            }
            if (vb) {
                if (A.out_match) A.out_match[(uint64_t)g * N + reqb] = mb;
                if (A.out_err) A.out_err[(uint64_t)g * N + reqb] = eb;
                if (A.req_err && eb) A.req_err[reqb] = 1;
            }
            if (counting(A)) {
                const uint32_t m2a = va ? ma : 0u, m2b = vb ? mb : 0u;
                for (uint32_t bits = wave_or(m2a | m2b); bits; bits &= bits - 1) {
                    const uint32_t k = __builtin_ctz(bits);
                    const uint32_t c = (uint32_t)__builtin_popcountll(__ballot((m2a >> k) & 1u)) +
                                       (uint32_t)__builtin_popcountll(__ballot((m2b >> k) & 1u));
                    if (lane == 0) atomicAdd(A.hits + r0 + k, (unsigned long long)c);
                }
            }
        }
    }
}

// mxp_eval_kernel with referenced-attribute records (mxp_eval_refs)
extern "C" __global__ __launch_bounds__(256) void mxp_eval_refs_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    eval_groups<true, true>(A, regs);
}

// Groups holding deep rules (programs with more than MXP_VM_MAXREG values live at once, e.g. nine
// right-nested comparisons; lower.cpp colouring): the same VM over a 64-register file, 128 KB of
// LDS -- one workgroup per CU, launched only for rule sets that have such rules (Plan::d_gdeep)
extern "C" __global__ __launch_bounds__(256) void mxp_eval_deep_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_DEEPREG][256];
    eval_groups<true, false, false>(A, regs);
}
extern "C" __global__ __launch_bounds__(256) void mxp_eval_deep_nfa_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_DEEPREG][256];
    eval_groups<true, false, true>(A, regs);
}
extern "C" __global__ __launch_bounds__(256) void mxp_eval_deep_refs_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_DEEPREG][256];
    eval_groups<true, true>(A, regs);
}

// Chunks of uniform indexed groups (vm.h mxp_fill): every word is a function of the guard column's
// kind alone -- match 0, error = the rules whose type check fails -- so a lane computes it once for
// each of its requests and streams 16-byte stores over the chunk's groups (1 KB per
// wave-instruction).  A wave covers `fill_span` spans of 256 requests (span s of group g lands at
// row g, requests q0 + 256 s ..), so one group row gets 1 KB x span contiguous bytes from the wave
// before the next row.  Workgroup = 4 waves; grid y = chunk.
#define MXP_FILL_SPAN_MAX 8
extern "C" __global__ __launch_bounds__(256) void mxp_fill_kernel(mxp_kargs A) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uni(threadIdx.x >> 6);
    const mxp_fill* F = A.fills + blockIdx.y;
    const uint32_t col = uni(F->col), okset = uni(F->okset), g0 = uni(F->g0), n = uni(F->n), moff = uni(F->moff);
    const uint32_t span = uni(A.fill_span);
    const uint64_t N = A.n;
    const uint32_t Q1 = A.q1;        // chunk end (chunks start at multiples of 1024)
    const uint32_t qw = A.q0 + (blockIdx.x * 4u + wave) * 256u * span;  // the wave's first request
    if (qw >= Q1) return;
    const uint32_t q0 = qw + lane * 4u;
    const bool vec = (N & 3u) == 0 && (Q1 & 3u) == 0;  // rows 16-byte aligned, the lane's 4 requests all present
    uint32_t bad[MXP_FILL_SPAN_MAX][4];  // per request: ~0 when the guard column fails its type check
    uint32_t any = 0;
#pragma unroll
    for (uint32_t sp = 0; sp < MXP_FILL_SPAN_MAX; sp++) {
        const uint32_t q = q0 + sp * 256u;
        if (sp < span && vec && q < Q1) {
            const uint32_t k4 = *(const uint32_t*)(A.kinds + (uint64_t)col * N + q);
#pragma unroll
            for (int r = 0; r < 4; r++) bad[sp][r] = ((okset >> ((k4 >> (8 * r)) & 0xFFu)) & 1u) ? 0u : ~0u;
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool in = sp < span && q + r < Q1;
                const uint32_t k = in ? A.kinds[(uint64_t)col * N + q + r] : 0u;
                bad[sp][r] = (in && !((okset >> k) & 1u)) ? ~0u : 0u;
            }
        }
        any |= bad[sp][0] | bad[sp][1] | bad[sp][2] | bad[sp][3];
    }
    if (A.req_err && any) {  // a failed type check errs every rule of the chunk's groups
        uint32_t masks = 0;
        for (uint32_t g = 0; g < n; g++) masks |= uni(A.fill_masks[moff + g]);
        if (masks)
            for (uint32_t sp = 0; sp < span; sp++)
                for (uint32_t r = 0; r < 4; r++)
                    if (bad[sp][r] && q0 + sp * 256u + r < Q1) A.req_err[q0 + sp * 256u + r] = 1;
    }
    if (A.errlog && any) {
        for (uint32_t g = 0; g < n; g++) {
            const uint32_t mask = uni(A.fill_masks[moff + g]);
            for (uint32_t sp = 0; sp < span; sp++)
                for (uint32_t r = 0; r < 4; r++)
                    if (bad[sp][r] && q0 + sp * 256u + r < Q1) log_guard_errors(A, mask, (g0 + g) * 32u, q0 + sp * 256u + r);
        }
    }
    // non-temporal streaming stores (A/B on C2: 0.828 vs 0.867 ms per evaluation,
    // profiles/r1_v15_ab_nt.log); MXP_DEBUG_FLAGS 128 = plain stores (ablation)
    const bool nt = !(A.flags & 128u);
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    for (uint32_t g = 0; g < n; g++) {
        const uint32_t mask = uni(A.fill_masks[moff + g]);
        const uint64_t row = (uint64_t)(g0 + g) * N;
#pragma unroll
        for (uint32_t sp = 0; sp < MXP_FILL_SPAN_MAX; sp++) {
            const uint32_t q = q0 + sp * 256u;
            if (sp >= span || qw + sp * 256u >= Q1) break;  // wave-uniform
            const uint64_t at = row + q;
            if (vec) {
                const v4u m = v4u{0u, 0u, 0u, 0u};
                const v4u er = v4u{bad[sp][0] & mask, bad[sp][1] & mask, bad[sp][2] & mask, bad[sp][3] & mask};
                if (q < Q1) {
                    if (nt) {
                        if (A.out_match) __builtin_nontemporal_store(m, (v4u*)(A.out_match + at));
                        if (A.out_err) __builtin_nontemporal_store(er, (v4u*)(A.out_err + at));
                    } else {
                        if (A.out_match) *(v4u*)(A.out_match + at) = m;
                        if (A.out_err) *(v4u*)(A.out_err + at) = er;
                    }
                }
            } else {
                for (uint32_t r = 0; r < 4; r++) {
                    if (q + r >= Q1) break;
                    if (A.out_match) A.out_match[at + r] = 0u;
                    if (A.out_err) A.out_err[at + r] = bad[sp][r] & mask;
                }
            }
        }
    }
}


// ---------------------------------------------------------------------------------------------
// Value classes.  A rule whose program reads one column, as a string (or a map[key] virtual
// column), computes a function of that column's (kind, string id) alone.  When a batch's column
// holds few distinct such values (pack time: engine.cpp pack_host), the rules of that column are
// evaluated once per distinct value -- a "class" -- and each request's words are gathered from its
// class: C4's 2000 header rules run on 17 classes per header instead of 1M requests.
//   mxp_vt_classify_kernel  per request and active column: the class (slot of an open-addressing
//                           table of class keys, mxp_vt_key; the first request to claim a slot is
//                           its representative);
//   mxp_vt_eval_kernel      the VM over (class representative, rule) pairs: lane = class, wave =
//                           one bitmap word of the column's rules; class words stored class-minor
//                           (word j of class k at tbase + j * cap + k, so a wave's gathers for one
//                           word hit one or two cache lines);
//   vt_words_of             the writers of the bitmaps (fill, lean, VM kernels) OR the class words
//                           of each request into its group words.
// Requests per workgroup of mxp_vt_classify_kernel and its LDS table (twice as many slots, so
// the workgroup's distinct keys always fit).
#define MXP_VTC_REQ 1024u
#define MXP_VTC_LCAP 2048u
// The batch's value-class dictionary, built once at upload (mxp_engine::pack_dict): per active column
// the class keys, a representative request of each and the class sizes.
extern "C" __global__ __launch_bounds__(256) void mxp_vt_classify_kernel(mxp_kargs A) {
    // The hot keys of a low-cardinality column would serialise on a handful of global addresses if
    // every request probed the global table (and L1 may keep a stale EMPTY line), so a workgroup
    // first dedups its 1024 requests' keys in an LDS table (40 KB: 4 workgroups per CU), resolves each distinct key against the
    // global table once (compare-and-swap, the inserter's request becomes the class
    // representative), then hands every request its class from LDS.
    __shared__ unsigned long long lkey[MXP_VTC_LCAP];
    __shared__ uint32_t lcls[MXP_VTC_LCAP];
    __shared__ uint32_t lrep[MXP_VTC_LCAP];
    __shared__ uint32_t lcnt[MXP_VTC_LCAP];  // requests per local slot (class sizes, with A.hits)
    const bool count = true;  // class sizes (feed mxp_vt_eval_kernel's fused hit counters)
    const uint32_t tid = threadIdx.x;
    const uint64_t N = A.n;
    const uint32_t base = A.q0 + blockIdx.x * MXP_VTC_REQ;
    for (uint32_t a = 0; a < A.n_vt; a++) {
        const uint32_t col = uni(A.vt_meta[a * 8u + MXP_VTM_COL]), cap = uni(A.vt_meta[a * 8u + MXP_VTM_CAP]),
                       kb = uni(A.vt_meta[a * 8u + MXP_VTM_KBASE]);
        for (uint32_t i = tid; i < MXP_VTC_LCAP; i += 256u) {
            lkey[i] = MXP_VT_EMPTY;
            lcnt[i] = 0;
        }
        __syncthreads();
        // 1. local slots of this thread's requests (req = base + tid + 256 r)
        uint32_t loc[MXP_VTC_REQ / 256u];
#pragma unroll
        for (uint32_t r = 0; r < MXP_VTC_REQ / 256u; r++) {
            const uint32_t req = base + tid + 256u * r;
            uint32_t h = 0xFFFFFFFFu;
            if (req < A.q1) {
                const uint64_t key = mxp_vt_key(A.kinds[(uint64_t)col * N + req], A.vals[(uint64_t)col * N + req]);
                h = mxp_hash64(key) & (MXP_VTC_LCAP - 1u);
                for (;;) {
                    const unsigned long long cur = lkey[h];
                    if (cur == key) break;
                    if (cur == MXP_VT_EMPTY) {
                        const unsigned long long old =
                            atomicCAS(&lkey[h], (unsigned long long)MXP_VT_EMPTY, (unsigned long long)key);
                        if (old == MXP_VT_EMPTY) {
                            lrep[h] = req;
                            break;
                        }
                        if (old == key) break;
                    }
                    h = (h + 1u) & (MXP_VTC_LCAP - 1u);
                }
            }
            loc[r] = h;
            if (count) {
                // class sizes: one LDS add per distinct slot of the wave (a low-cardinality column puts
                // most of a wave's lanes on a few slots: per-lane atomics there serialise)
                for (uint64_t pend = __ballot(h != 0xFFFFFFFFu); pend;) {
                    const uint32_t sl = __builtin_amdgcn_readlane(h, (uint32_t)__builtin_ctzll(pend));
                    const uint64_t same = __ballot(h == sl);
                    if ((tid & 63u) == (uint32_t)__builtin_ctzll(same)) atomicAdd(&lcnt[sl], (uint32_t)__builtin_popcountll(same));
                    pend &= ~same;
                }
            }
        }
        __syncthreads();
        // 2. each distinct key of the workgroup against the global table (room for twice the
        // batch's distinct keys, counted at pack time: the probe ends)
        unsigned long long* T = A.vt_keys + kb;
        for (uint32_t i = tid; i < MXP_VTC_LCAP; i += 256u) {
            const unsigned long long key = lkey[i];
            if (key == MXP_VT_EMPTY) continue;
            uint32_t h = mxp_hash64(key) & (cap - 1u);
            for (;;) {
                // (read first: every workgroup meets the column's few hot keys, and a CAS on a slot
                // another workgroup already holds would serialise at L2 for nothing)
                unsigned long long old = __hip_atomic_load(T + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old == MXP_VT_EMPTY) {
                    old = atomicCAS(T + h, (unsigned long long)MXP_VT_EMPTY, key);
                    if (old == MXP_VT_EMPTY) {
                        A.vt_rep[kb + h] = lrep[i];
                        break;
                    }
                }
                if (old == key) break;
                h = (h + 1u) & (cap - 1u);
            }
            lcls[i] = h;
            if (count) atomicAdd(A.vt_cnt + kb + h, lcnt[i]);
        }
        __syncthreads();
        (void)loc;  // (the classes of the requests are the evaluation's: mxp_vt_lookup_kernel)
        __syncthreads();
    }
}

// The batch's final class tables from the packer's provisional ones (pack.hip mxp_pack_vtd_*): every
// key of active slot a (candidate column F.cand[a]) into its table of the capacity the host sized
// (the keys are distinct: a compare-and-swap on an empty slot, probing on), with its class size
// and representative request.  grid (MXP_VTD_CAP / 256, active slots).
extern "C" __global__ __launch_bounds__(256) void mxp_vtd_final_kernel(mxp_kargs A, mxp_vtd_final_args F) {
    const uint32_t a = blockIdx.y, i = blockIdx.x * 256u + threadIdx.x;
    if (i >= MXP_VTD_CAP) return;
    const uint64_t at = (uint64_t)F.cand[a] * MXP_VTD_CAP + i;
    const unsigned long long key = F.tkey[at];
    if (key == MXP_VT_EMPTY) return;
    const uint32_t cap = A.vt_meta[a * 8u + MXP_VTM_CAP], kb = A.vt_meta[a * 8u + MXP_VTM_KBASE];
    unsigned long long* T = A.vt_keys + kb;
    uint32_t h = mxp_hash64(key) & (cap - 1u);
    while (atomicCAS(T + h, (unsigned long long)MXP_VT_EMPTY, key) != MXP_VT_EMPTY) h = (h + 1u) & (cap - 1u);
    const uint2 cr = F.tcr[at];
    A.vt_rep[kb + h] = cr.y;
    A.vt_cnt[kb + h] = cr.x;
}

extern "C" hipError_t mxp_launch_vtd_final(const mxp_kargs* args, const mxp_vtd_final_args* f, hipStream_t s) {
    hipLaunchKernelGGL(mxp_vtd_final_kernel, dim3(MXP_VTD_CAP / 256u, args->n_vt), dim3(256), 0, s, *args, *f);
    return hipGetLastError();
}

// The evaluation's class of every request [q0, q1) per active column: a read-only probe of the
// batch's dictionary (built at upload by mxp_vt_classify_kernel, so it holds every key of the
// batch), whose few hot lines stay in L1.  A thread takes 4 consecutive requests: one 4-byte kinds
// load, two 16-byte value loads and one 8-byte class store, and four independent probes in flight
// (one request per thread measured 30 us on C4).  grid (request blocks of 1024, active columns).
__device__ __forceinline__ uint32_t vt_probe(const unsigned long long* __restrict__ T, uint32_t cap,
                                             unsigned long long key) {
    uint32_t h = mxp_hash64(key) & (cap - 1u);
    // (every batch key is in the table, which is at most half full: the probe ends at the key; an
    // empty slot -- a batch changed after upload -- ends it too, on a slot vt_eval leaves at 0)
    for (uint32_t i = 0; i < cap; i++, h = (h + 1u) & (cap - 1u)) {
        const unsigned long long k = T[h];
        if (k == key || k == MXP_VT_EMPTY) break;
    }
    return h;
}
extern "C" __global__ __launch_bounds__(256) void mxp_vt_lookup_kernel(mxp_kargs A) {
    const uint32_t a = blockIdx.y, q = A.q0 + (blockIdx.x * 256u + threadIdx.x) * 4u, Q1 = A.q1;
    if (q >= Q1) return;
    const uint64_t N = A.n;
    const uint32_t col = uni(A.vt_meta[a * 8u + MXP_VTM_COL]), cap = uni(A.vt_meta[a * 8u + MXP_VTM_CAP]),
                   kb = uni(A.vt_meta[a * 8u + MXP_VTM_KBASE]);
    const unsigned long long* __restrict__ T = A.vt_keys + kb;
    const uint64_t at = (uint64_t)col * N + q;
    uint16_t* const C = A.vt_cls + (uint64_t)a * MXP_VT_PITCH(N) + q;
    if ((N & 3u) == 0 && (q & 3u) == 0 && q + 4u <= Q1) {
        const uint32_t k4 = *(const uint32_t*)(A.kinds + at);
        const ulonglong2 v01 = *(const ulonglong2*)(A.vals + at), v23 = *(const ulonglong2*)(A.vals + at + 2u);
        const uint32_t h0 = vt_probe(T, cap, mxp_vt_key(k4 & 0xFFu, v01.x));
        const uint32_t h1 = vt_probe(T, cap, mxp_vt_key((k4 >> 8) & 0xFFu, v01.y));
        const uint32_t h2 = vt_probe(T, cap, mxp_vt_key((k4 >> 16) & 0xFFu, v23.x));
        const uint32_t h3 = vt_probe(T, cap, mxp_vt_key(k4 >> 24, v23.y));
        *(uint64_t*)C = (uint64_t)h0 | (uint64_t)h1 << 16 | (uint64_t)h2 << 32 | (uint64_t)h3 << 48;
        return;
    }
    for (uint32_t r = 0; r < 4u && q + r < Q1; r++)
        C[r] = (uint16_t)vt_probe(T, cap, mxp_vt_key(A.kinds[at + r], A.vals[at + r]));
}

// grid x: class tiles of 64 (slot by slot), y: groups of 4 words (one per wave)
template <bool kNfa>
__device__ __forceinline__ void vt_eval_body(const mxp_kargs& A, uint64_t (*regs)[256]) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = uni(tid >> 6);
    uint32_t t = blockIdx.x, a = 0;
    for (; a + 1 < A.n_vt; a++) {
        const uint32_t nt = uni(A.vt_meta[a * 8u + MXP_VTM_CAP]) / 64u;
        if (t < nt) break;
        t -= nt;
    }
    const uint32_t* M = A.vt_meta + a * 8u;
    const uint32_t cap = uni(M[MXP_VTM_CAP]), kb = uni(M[MXP_VTM_KBASE]), tb = uni(M[MXP_VTM_TBASE]),
                   nw = uni(M[MXP_VTM_NW]), woff = uni(M[MXP_VTM_WOFF]);
    const uint32_t j = blockIdx.y * 4u + wave;
    if (j >= nw || t * 64u >= cap) return;  // wave-uniform; the VM needs no block barrier
    const uint32_t k = t * 64u + lane;
    const bool live = __hip_atomic_load(A.vt_keys + kb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != MXP_VT_EMPTY;
    const uint32_t rep = live ? A.vt_rep[kb + k] : 0u;
    const uint32_t g = uni(A.vt_words[2u * (woff + j)]), mask = uni(A.vt_words[2u * (woff + j) + 1u]);
    uint32_t m = 0, e = 0;
    for (uint32_t bits = mask; bits; bits &= bits - 1u) {
        const uint32_t b = __builtin_ctz(bits);
        const uint32_t rule = g * 32u + b;
        const uint32_t base = uni(A.rule_off[rule]);
        const uint32_t len = uni(A.rule_off[rule + 1]) - base;
        const uint32_t code = run_rule<false, kNfa>(A, ((cuint32*)A.prog) + (uint64_t)base * 4u, len, 0u, live, rule, rep, regs, tid);
        if (live) {
            m |= code == PC_TRUE ? 1u << b : 0u;
            e |= code >= PC_ERROR ? 1u << b : 0u;
        }
    }
    *(uint2*)(A.vt_tm + 2u * ((uint64_t)tb + (uint64_t)j * cap + k)) = make_uint2(m, e);
    if (counting(A)) {
        // fused hit counters of the value-class rules: per rule, the sizes of the classes whose
        // word holds its match bit (the merge kernels count none of these bits)
        const uint32_t c = live ? A.vt_cnt[kb + k] : 0u;
        for (uint32_t bits = wave_or(live ? m : 0u); bits; bits &= bits - 1u) {
            const uint32_t bb = __builtin_ctz(bits);
            uint32_t sum = (m >> bb) & 1u ? c : 0u;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) sum += (uint32_t)__shfl_xor((int)sum, off, 64);
            if (lane == 0 && sum) atomicAdd(A.hits + g * 32u + bb, (unsigned long long)sum);
        }
    }
}

extern "C" __global__ __launch_bounds__(256) void mxp_vt_eval_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    vt_eval_body<false>(A, regs);
}

extern "C" __global__ __launch_bounds__(256) void mxp_vt_eval_nfa_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    vt_eval_body<true>(A, regs);
}

// Fill chunks with value-class merge entries: as mxp_fill_kernel (words of uniform indexed groups
// depend on their guard column's kind), plus the class words of each request.  A lane owns 4
// consecutive requests (one 16-byte store per plane and group), a wave 256; the requests' classes
// are loaded once (4 x u16 per active column) and kept in registers.  kLds: the class words of the
// chunk's merge entries come from the workgroup's LDS copy (S; lane a of PB / PJ = LDS base and
// first staged word position of active slot a), else from global memory (vt_tm).
// ascending sort of 8 values (Batcher's odd-even merge network, 19 compare-exchanges)
__device__ __forceinline__ void sort8(uint32_t (&x)[8]) {
#define MXP_CX(a, b)                          \
    {                                         \
        const uint32_t lo = min(x[a], x[b]);  \
        x[b] = max(x[a], x[b]);               \
        x[a] = lo;                            \
    }
    MXP_CX(0, 1) MXP_CX(2, 3) MXP_CX(4, 5) MXP_CX(6, 7) MXP_CX(0, 2) MXP_CX(1, 3) MXP_CX(4, 6) MXP_CX(5, 7)
    MXP_CX(1, 2) MXP_CX(5, 6) MXP_CX(0, 4) MXP_CX(1, 5) MXP_CX(2, 6) MXP_CX(3, 7) MXP_CX(2, 4) MXP_CX(3, 5)
    MXP_CX(1, 2) MXP_CX(3, 4) MXP_CX(5, 6)
#undef MXP_CX
}

// one sorted deferred pair x (g << 8 | plane << 7 | request % 4 << 5 | bit) into the lane's words
__device__ __forceinline__ void dtp_merge(uint32_t x, bool on, uint32_t (&m)[4], uint32_t (&e)[4]) {
    const uint32_t b = on ? 1u << (x & 31u) : 0u, r = (x >> 5) & 3u;
    const uint32_t bm = (x & 128u) ? 0u : b, be = (x & 128u) ? b : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        m[k] |= r == k ? bm : 0u;
        e[k] |= r == k ? be : 0u;
    }
}

// The deferred index pairs of a lane's quad of requests in one fill chunk (mxp_dtp_sort_kernel):
// up to 8 u16 entries, sorted here (group first) into a queue in four registers whose head the
// group loop consumes while it names the current group.
struct DtpQueue {
    uint32_t q0 = ~0u, q1 = ~0u, q2 = ~0u, q3 = ~0u;
    __device__ __forceinline__ void load(const mxp_kargs& A, uint32_t chunk, uint32_t req0, bool in) {
        if (!A.dtp_slots || !in) return;
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const uint64_t qi = (uint64_t)chunk * MXP_DTP_ROW(A.dtp_tiles) + (req0 >> 2);
        const uint32_t dk = A.dtp_qn[qi];
        const v4u sl = *(const v4u*)(A.dtp_slots + qi * 8u);
        decode(dk, sl);
    }
    // the sorted queue from a quad's raw count and slot row (load, or a prefetch of them)
    template <typename V4>
    __device__ __forceinline__ void decode(uint32_t dk, const V4& sl) {
        if (!dk) return;
        const uint32_t h[4] = {sl.x, sl.y, sl.z, sl.w};
        uint32_t x[8];
#pragma unroll
        for (uint32_t i = 0; i < 8; i++) x[i] = i < dk ? (h[i >> 1] >> (16u * (i & 1u))) & 0xFFFFu : 0xFFFFu;
        sort8(x);
        q0 = x[0] | x[1] << 16;
        q1 = x[2] | x[3] << 16;
        q2 = x[4] | x[5] << 16;
        q3 = x[6] | x[7] << 16;
    }
    // whether some lane's queue holds an error-plane entry (wave-uniform)
    __device__ __forceinline__ bool any_err() const { return __ballot(has_err()) != 0; }
    // (pads, 0xFFFF, carry the plane bit too: only real entries count)
    __device__ __forceinline__ bool has_err() const {
        bool h = false;
        const uint32_t w[4] = {q0, q1, q2, q3};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t x = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
            h |= x != 0xFFFFu && (x & 128u);
        }
        return h;
    }
    // merge() for a group known at compile time (the unrolled fills): the hit test is one compare
    // with an inline constant, and the error plane is touched only when some lane queued an entry
    // for it (kErr)
    template <uint32_t G, bool kErr>
    __device__ __forceinline__ void merge_c(uint32_t (&m)[4], uint32_t (&e)[4]) {
        for (;;) {
            const uint32_t x = q0;
            const bool hit = ((x >> 8) & 0xFFu) == G;
            if (!__ballot(hit)) break;
            const uint32_t b = hit ? 1u << (x & 31u) : 0u, r = (x >> 5) & 3u;
            const uint32_t bm = (kErr && (x & 128u)) ? 0u : b;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) m[k] |= r == k ? bm : 0u;
            if (kErr) {
                const uint32_t be = (x & 128u) ? b : 0u;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) e[k] |= r == k ? be : 0u;
            }
            if (hit) {
                q0 = __builtin_amdgcn_alignbit(q1, q0, 16);
                q1 = __builtin_amdgcn_alignbit(q2, q1, 16);
                q2 = __builtin_amdgcn_alignbit(q3, q2, 16);
                q3 = q3 >> 16 | 0xFFFF0000u;
            }
        }
    }
    // OR the head entries naming group g into the words (pads, 0xFFFF, name no group)
    __device__ __forceinline__ void merge(uint32_t g, uint32_t (&m)[4], uint32_t (&e)[4]) {
        for (;;) {
            const uint32_t x = q0 & 0xFFFFu;
            const bool hit = (x >> 8) == g;
            if (!__ballot(hit)) break;
            dtp_merge(x, hit, m, e);
            if (hit) {
                q0 = __builtin_amdgcn_alignbit(q1, q0, 16);
                q1 = __builtin_amdgcn_alignbit(q2, q1, 16);
                q2 = __builtin_amdgcn_alignbit(q3, q2, 16);
                q3 = q3 >> 16 | 0xFFFF0000u;
            }
        }
    }
};

template <bool kLds>
__device__ __forceinline__ void vtfill_wave(const mxp_kargs& A, const mxp_fill* F, uint32_t chunk, uint32_t qw,
                                            const uint2* S, const uint32_t* RW) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t col = uni(F->col), okset = uni(F->okset), g0 = uni(F->g0), n = uni(F->n), moff = uni(F->moff);
    const uint64_t N = A.n;
    const uint32_t Q1 = A.q1;
    if (qw >= Q1) return;
    const uint32_t q0 = qw + lane * 4u;
    const bool vec = (N & 3u) == 0 && (Q1 & 3u) == 0 && (q0 & 3u) == 0;
    const uint32_t nvt = uni(A.n_vt);
    uint32_t bad[4];
    // 4 x u16 classes per active column, as (lo, hi) u32 pairs of one register vector: a merge
    // entry's slot a is wave-uniform, so clv[2a] compiles to an indexed register move
    // (s_set_gpr_idx_on) instead of a select over every slot
    typedef uint32_t vcls __attribute__((ext_vector_type(2 * MXP_VT_MAX)));
    vcls clv;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool in = q0 + r < Q1;
        const uint32_t k = in ? A.kinds[(uint64_t)col * N + q0 + r] : 0u;
        bad[r] = (in && !((okset >> k) & 1u)) ? ~0u : 0u;
    }
#pragma unroll
    for (uint32_t a = 0; a < MXP_VT_MAX; a++) {
        uint64_t c = 0;
        if (a < nvt) {
            const uint16_t* C = A.vt_cls + (uint64_t)a * MXP_VT_PITCH(N);
            if (vec && q0 < Q1) {
                c = *(const uint64_t*)(C + q0);
            } else {
                for (uint32_t r = 0; r < 4; r++)
                    if (q0 + r < Q1) c |= (uint64_t)C[q0 + r] << (16u * r);
            }
        }
        clv[2 * a] = (uint32_t)c;
        clv[2 * a + 1] = (uint32_t)(c >> 32);
    }
    const bool any = (bad[0] | bad[1] | bad[2] | bad[3]) != 0;
    DtpQueue dq;
    dq.load(A, chunk, q0, q0 < Q1);
    const bool dany = __ballot(dq.q0 != ~0u) != 0;
    const bool nt = !(A.flags & 128u);
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    // the active slots' (cap, tbase), the chunk's group masks and merge entries: one vector load
    // each, read back with v_readlane -- no chain of dependent scalar loads per group
    const uint32_t MV = lane < 2u * MXP_VT_MAX && (lane >> 1) < nvt ? A.vt_meta[(lane >> 1) * 8u + MXP_VTM_CAP + (lane & 1u)] : 0u;
    const uint32_t FM = lane < n ? A.fill_masks[moff + lane] : 0u;
    const uint32_t GM = kLds && lane < n ? A.gvt_mask[g0 + lane] : 0u;  // slots each group names
    const uint32_t GO = lane <= n ? A.gvt_off[g0 + lane] : 0u;
    const uint32_t e0 = __builtin_amdgcn_readlane(GO, 0), ecount = __builtin_amdgcn_readlane(GO, n) - e0;
    uint32_t GE0 = lane < ecount ? A.gvt[e0 + lane] : 0u, GE1 = lane + 64u < ecount ? A.gvt[e0 + 64u + lane] : 0u;
    uint32_t anyerr[4] = {0u, 0u, 0u, 0u};
    for (uint32_t g = 0; g < n; g++) {
        const uint32_t G = g0 + g;
        const uint32_t mask = __builtin_amdgcn_readlane(FM, g);
        uint32_t m[4] = {0u, 0u, 0u, 0u}, e[4], ve[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int r = 0; r < 4; r++) e[r] = bad[r] & mask;
        if (A.errlog && any && mask)
            for (uint32_t r = 0; r < 4; r++)
                if (e[r] && q0 + r < Q1) log_guard_errors(A, e[r], G * 32u, q0 + r);
        const uint32_t i0 = __builtin_amdgcn_readlane(GO, g) - e0, i1 = __builtin_amdgcn_readlane(GO, g + 1) - e0;
        if constexpr (kLds) {
            // staged (<= 128 entries): the group's entries in slot order, one per slot it names --
            // unrolled over the slots so each one's classes come from fixed registers (no indexed
            // register move) and its row from one readlane
            const uint32_t gm = __builtin_amdgcn_readlane(GM, g);
            const uint4 ra = *(const uint4*)(RW + g * MXP_VT_MAX), rb = *(const uint4*)(RW + g * MXP_VT_MAX + 4u);
            const uint32_t rows[MXP_VT_MAX] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
#pragma unroll
            for (uint32_t a = 0; a < MXP_VT_MAX; a++) {
                if (!(gm & (1u << a))) continue;
                const uint32_t row = rows[a];
                const uint64_t c = (uint64_t)clv[2u * a] | (uint64_t)clv[2u * a + 1u] << 32;
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) {
                    const uint2 w = S[row + ((uint32_t)(c >> (16u * r)) & 0xFFFFu)];
                    m[r] |= w.x;
                    ve[r] |= w.y;
                }
            }
        } else
        for (uint32_t i = i0; i < i1; i++) {
            const uint32_t ent = i < 64u ? __builtin_amdgcn_readlane(GE0, i)
                                 : i < 128u ? __builtin_amdgcn_readlane(GE1, i - 64u) : uni(A.gvt[e0 + i]);
            const uint32_t a = ent >> 24, j = ent & 0xFFFFFFu;
            const uint32_t au = __builtin_amdgcn_readfirstlane(a);
            const uint64_t c = (uint64_t)clv[2u * au] | (uint64_t)clv[2u * au + 1u] << 32;
            if constexpr (kLds) {
                const uint32_t row = j;  // (the entry's LDS row, computed above; staged chunks have <= 128 entries)
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) {
                    const uint2 w = S[row + ((uint32_t)(c >> (16u * r)) & 0xFFFFu)];
                    m[r] |= w.x;
                    ve[r] |= w.y;
                }
            } else {
                const uint32_t cap = __builtin_amdgcn_readlane(MV, 2u * a);
                const uint32_t tb = __builtin_amdgcn_readlane(MV, 2u * a + 1u);
                const uint64_t row = (uint64_t)tb + (uint64_t)j * cap;
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) {
                    const uint2 w = *(const uint2*)(A.vt_tm + 2u * (row + ((c >> (16u * r)) & 0xFFFFu)));
                    m[r] |= w.x;
                    ve[r] |= w.y;
                }
            }
        }
        uint32_t vmask[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            vmask[r] = q0 + r < Q1 ? ~0u : 0u;
            e[r] |= ve[r];
        }
        if (A.errlog) {
            uint32_t c = 0;
#pragma unroll
            for (int r = 0; r < 4; r++) c += (uint32_t)__builtin_popcount(ve[r] & vmask[r]);
            vt_count_n(A, c);
        }
        if (dany) dq.merge(g, m, e);  // the index kernel's true / error pairs in this group's words
        // (no hit counting: a uniform group's words hold no true bit but the value classes', which
        // mxp_vt_eval_kernel counts per class)
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) anyerr[r] |= e[r];  // (request error flags: once, after the loop)
        const uint64_t at = (uint64_t)G * N + q0;
        if (vec && q0 < Q1) {
            const v4u mv = v4u{m[0], m[1], m[2], m[3]};
            const v4u ev = v4u{e[0], e[1], e[2], e[3]};
            if (nt) {
                if (A.out_match) __builtin_nontemporal_store(mv, (v4u*)(A.out_match + at));
                if (A.out_err) __builtin_nontemporal_store(ev, (v4u*)(A.out_err + at));
            } else {
                if (A.out_match) *(v4u*)(A.out_match + at) = mv;
                if (A.out_err) *(v4u*)(A.out_err + at) = ev;
            }
        } else {
            for (uint32_t r = 0; r < 4; r++) {
                if (q0 + r >= Q1) break;
                if (A.out_match) A.out_match[at + r] = m[r];
                if (A.out_err) A.out_err[at + r] = e[r];
            }
        }
    }
    if (A.req_err)
        for (uint32_t r = 0; r < 4; r++)
            if (anyerr[r] && q0 + r < Q1) A.req_err[q0 + r] = 1;
}

// mxp_fill_kernel for deferred index pairs (kargs.dtp_slots): one span of 256 requests per wave (a
// lane owns one quad, whose sorted pairs it merges into each group's words before storing them)
extern "C" __global__ __launch_bounds__(256) void mxp_fill_dtp_kernel(mxp_kargs A) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = uni(threadIdx.x >> 6);
    const mxp_fill* F = A.fills + blockIdx.y;
    const uint32_t col = uni(F->col), okset = uni(F->okset), g0 = uni(F->g0), n = uni(F->n), moff = uni(F->moff);
    const uint64_t N = A.n;
    const uint32_t Q1 = A.q1;
    const uint32_t qw = A.q0 + (blockIdx.x * 4u + wave) * 256u;
    if (qw >= Q1) return;
    const uint32_t q0 = qw + lane * 4u;
    const bool vec = (N & 3u) == 0 && (Q1 & 3u) == 0;
    uint32_t bad[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool in = q0 + r < Q1;
        const uint32_t k = in ? A.kinds[(uint64_t)col * N + q0 + r] : 0u;
        bad[r] = (in && !((okset >> k) & 1u)) ? ~0u : 0u;
    }
    const bool any = (bad[0] | bad[1] | bad[2] | bad[3]) != 0;
    // (a pair Resolve's evaluation: only the request error flags and records unless pairs overflowed)
    const bool store = !A.dtp_lazy || uni(*A.dtp_lazy) != 0u;
    DtpQueue dq;
    if (store) dq.load(A, A.dtp_cbase + blockIdx.y, q0, q0 < Q1);
    const bool dany = __ballot(dq.q0 != ~0u) != 0;
    if (A.req_err && any) {
        uint32_t masks = 0;
        for (uint32_t g = 0; g < n; g++) masks |= uni(A.fill_masks[moff + g]);
        if (masks)
            for (uint32_t r = 0; r < 4; r++)
                if (bad[r] && q0 + r < Q1) A.req_err[q0 + r] = 1;
    }
    if (A.errlog && any)
        for (uint32_t g = 0; g < n; g++) {
            const uint32_t mask = uni(A.fill_masks[moff + g]);
            for (uint32_t r = 0; r < 4; r++)
                if (bad[r] && q0 + r < Q1) log_guard_errors(A, mask, (g0 + g) * 32u, q0 + r);
        }
    if (!store) return;
    const bool nt = !(A.flags & 128u);
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    for (uint32_t g = 0; g < n; g++) {
        const uint32_t mask = uni(A.fill_masks[moff + g]);
        uint32_t m[4] = {0u, 0u, 0u, 0u}, e[4];
#pragma unroll
        for (int r = 0; r < 4; r++) e[r] = bad[r] & mask;
        if (dany) dq.merge(g, m, e);
        const uint64_t at = (uint64_t)(g0 + g) * N + q0;
        if (vec && q0 < Q1) {
            const v4u mv = v4u{m[0], m[1], m[2], m[3]}, ev = v4u{e[0], e[1], e[2], e[3]};
            if (nt) {
                if (A.out_match) __builtin_nontemporal_store(mv, (v4u*)(A.out_match + at));
                if (A.out_err) __builtin_nontemporal_store(ev, (v4u*)(A.out_err + at));
            } else {
                if (A.out_match) *(v4u*)(A.out_match + at) = mv;
                if (A.out_err) *(v4u*)(A.out_err + at) = ev;
            }
        } else {
            for (uint32_t r = 0; r < 4; r++) {
                if (q0 + r >= Q1) break;
                if (A.out_match) A.out_match[at + r] = m[r];
                if (A.out_err) A.out_err[at + r] = e[r];
            }
        }
    }
}

// MXP_DEBUG_FLAGS 2097152: every chunk gathers class words from global memory (A/B)
extern "C" __global__ __launch_bounds__(256) void mxp_vtfill_kernel(mxp_kargs A) {
    const uint32_t wave = uni(threadIdx.x >> 6);
    vtfill_wave<false>(A, A.fills + blockIdx.y, A.dtp_cbase + blockIdx.y, A.q0 + (blockIdx.x * 4u + wave) * 256u, nullptr,
                       nullptr);
}

// The default: a workgroup stages its chunk's class-word rows in LDS once -- per active slot a, the
// contiguous rows of the word positions the chunk's merge entries name (slot a's positions grow
// with the group) -- then covers MXP_VTF_TILES tiles of 1024 requests (4 waves x 256) gathering
// from LDS instead of L1/L2 (C4: ~60 entries x 4 gathers per request and chunk).  A chunk whose
// rows exceed the 32 KB budget gathers from global memory.  100 VGPRs with the deferred-pair queue, 32 KB: 4 workgroups per CU (measured
// faster than 96 VGPRs forced to 5: C4 1.715 vs 1.78 ms, profiles/r2_v14_ablibs_vtfill_occ_c4.log).
#define MXP_VTF_STAGE 4096u
extern "C" __global__ __launch_bounds__(256) void mxp_vtfill_lds_kernel(mxp_kargs A) {
    __shared__ uint2 S[MXP_VTF_STAGE];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uni(tid >> 6);
    const mxp_fill* F = A.fills + blockIdx.y;
    const uint32_t g0 = uni(F->g0), n = uni(F->n), nvt = uni(A.n_vt);
    // staging plan, computed alike by every wave: per slot a its [jlo, jhi] over the chunk's entries
    const uint32_t e0 = uni(A.gvt_off[g0]), ecount = uni(A.gvt_off[g0 + n]) - e0;
    const uint32_t E0 = lane < ecount ? A.gvt[e0 + lane] : 0xFFFFFFFFu;
    const uint32_t E1 = lane + 64u < ecount ? A.gvt[e0 + 64u + lane] : 0xFFFFFFFFu;
    const uint32_t capl = lane < nvt ? A.vt_meta[lane * 8u + MXP_VTM_CAP] : 0u;
    const uint32_t tbl = lane < nvt ? A.vt_meta[lane * 8u + MXP_VTM_TBASE] : 0u;
    uint32_t PB = 0, PJ = 0, total = 0;
    for (uint32_t a = 0; a < nvt; a++) {
        const uint32_t lo = wave_min(min((E0 >> 24) == a ? (E0 & 0xFFFFFFu) : 0xFFFFFFFFu,
                                         (E1 >> 24) == a ? (E1 & 0xFFFFFFu) : 0xFFFFFFFFu));
        const uint32_t hi = wave_max(max((E0 >> 24) == a && E0 != 0xFFFFFFFFu ? (E0 & 0xFFFFFFu) + 1u : 0u,
                                         (E1 >> 24) == a && E1 != 0xFFFFFFFFu ? (E1 & 0xFFFFFFu) + 1u : 0u));
        const uint32_t rows = hi > lo ? hi - lo : 0u;
        if (lane == a) {
            PB = total;
            PJ = rows ? lo : 0u;
        }
        total += rows * __builtin_amdgcn_readlane(capl, a);
    }
    const bool staged = ecount <= 128u && n <= MXP_FILL_CHUNK && total <= MXP_VTF_STAGE && !(A.flags & 2097152u);
    // the LDS row of every (group, slot) merge entry of the chunk, so the group loop reads them with
    // two broadcast LDS loads per group and no scalar arithmetic (the scalar unit, one per CU,
    // bounded this kernel)
    __shared__ uint32_t RW[MXP_FILL_CHUNK * MXP_VT_MAX];
    __shared__ uint32_t PL[3 * MXP_VT_MAX];  // per slot: LDS base, first staged position, capacity
    if (staged) {
        for (uint32_t a = 0; a < nvt; a++) {
            const uint32_t base = __builtin_amdgcn_readlane(PB, a);
            const uint32_t next = a + 1u < nvt ? __builtin_amdgcn_readlane(PB, a + 1u) : total;
            const uint64_t src = (uint64_t)__builtin_amdgcn_readlane(tbl, a) +
                                 (uint64_t)__builtin_amdgcn_readlane(PJ, a) * __builtin_amdgcn_readlane(capl, a);
            for (uint32_t i = tid; i < next - base; i += 256u) S[base + i] = *(const uint2*)(A.vt_tm + 2u * (src + i));
        }
        if (tid < nvt) {
            PL[3u * tid] = PB;
            PL[3u * tid + 1u] = PJ;
            PL[3u * tid + 2u] = capl;
        }
        __syncthreads();
        if (tid < n) {  // thread t: group t's entries
            const uint32_t i1 = A.gvt_off[g0 + tid + 1u];
            for (uint32_t i = A.gvt_off[g0 + tid]; i < i1; i++) {
                const uint32_t ent = A.gvt[i], a = ent >> 24, j = ent & 0xFFFFFFu;
                RW[tid * MXP_VT_MAX + a] = PL[3u * a] + (j - PL[3u * a + 1u]) * PL[3u * a + 2u];
            }
        }
        __syncthreads();
    }
    for (uint32_t t = 0; t < MXP_VTF_TILES; t++) {
        const uint32_t qw = A.q0 + ((blockIdx.x * MXP_VTF_TILES + t) * 4u + wave) * 256u;
        if (staged)
            vtfill_wave<true>(A, F, A.dtp_cbase + blockIdx.y, qw, S, RW);
        else
            vtfill_wave<false>(A, F, A.dtp_cbase + blockIdx.y, qw, nullptr, nullptr);
    }
}

// Value-class fill for batches whose active class tables all have the minimum capacity (64 slots:
// at most 32 distinct values per column -- C4's header columns).  The workgroup stages, per active
// slot a and group g of the chunk, the 64 class words of the bitmap word g's rules of slot a take
// (zero where g names no rule of slot a) at a FIXED place, [a][g][class]: a request's address for
// slot a is computed once per tile, and group g's word is then a ds_read_b32 with the immediate
// offset g * 256 -- the group loop is unrolled, so a gather costs one LDS instruction and one OR,
// against an address add, a 64-bit gather and two ORs in mxp_vtfill_lds_kernel, whose issue rate
// bounded it (SQ r3: 2.2e8 VALU instructions per C4 evaluation).  Error words stay in global memory:
// they are gathered (through the staged word positions) only when some class word of the chunk
// holds an error bit (none in C4), so LDS holds the match words alone.
#define MXP_VTI_CAP 64u
template <uint32_t V>
struct GroupC {
    static constexpr uint32_t value = V;
    static constexpr bool ct = true;
};
struct GroupR {
    uint32_t value;
    static constexpr bool ct = false;
};
template <uint32_t G, uint32_t NG, typename F>
__device__ __forceinline__ void for_groups(F& f) {
    if constexpr (G < NG) {
        f(GroupC<G>{});
        for_groups<G + 1, NG>(f);
    }
}
// Two kernels per column count share this body.  The fast one (kSlow false) takes the wave-tiles
// of the common case -- no guard-kind errors among the wave's requests, no class error words in the
// chunk, no error-plane pairs in the wave's queues -- with the group loop unrolled at compile time,
// and marks every other wave-tile in kargs.vtf_slow; the slow one, launched right after on the same
// grid, runs the general loop on the marked wave-tiles only (a workgroup with none returns before
// staging).  Keeping the general loop out of the fast kernel keeps its registers at ~50 VGPRs:
// in one kernel the error paths set the count (147) and with it the occupancy.
template <uint32_t NVT, bool kSlow>
__device__ __forceinline__ void vtfill_imm_body(const mxp_kargs& A, uint32_t bx, uint32_t by, uint32_t gx) {
    __shared__ uint32_t SM[NVT * MXP_FILL_CHUNK * MXP_VTI_CAP];
    __shared__ uint32_t SJ[NVT * MXP_FILL_CHUNK];  // word position of (slot, group), ~0: none
    __shared__ uint32_t eflag;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = uni(tid >> 6);
    // (the wave-tile marks of this workgroup: [MXP_VTF_TILES][4 waves])
    uint8_t* const slow = A.vtf_slow + ((uint64_t)by * gx + bx) * (MXP_VTF_TILES * 4u);
    if constexpr (kSlow) {
        if (!__syncthreads_or(tid < MXP_VTF_TILES * 4u ? slow[tid] : 0)) return;
    }
    const mxp_fill* F = A.fills + by;
    const uint32_t col = uni(F->col), okset = uni(F->okset), g0 = uni(F->g0), n = uni(F->n), moff = uni(F->moff);
    const uint32_t chunk = A.dtp_cbase + by;
    // 1. staging: zero, then each (group, slot) merge entry's 64 class words into its fixed row
    for (uint32_t i = tid; i < NVT * MXP_FILL_CHUNK * MXP_VTI_CAP; i += 256u) SM[i] = 0u;
    if (tid < NVT * MXP_FILL_CHUNK) SJ[tid] = ~0u;
    if (tid == 0) eflag = 0u;
    __syncthreads();
    const uint32_t TB = lane < NVT ? A.vt_meta[lane * 8u + MXP_VTM_TBASE] : 0u;
    uint32_t eor = 0u;
    for (uint32_t g = 0; g < n; g++) {
        const uint32_t i0 = uni(A.gvt_off[g0 + g]), i1 = uni(A.gvt_off[g0 + g + 1u]);
        for (uint32_t x = tid; x < (i1 - i0) * MXP_VTI_CAP; x += 256u) {
            const uint32_t ent = A.gvt[i0 + x / MXP_VTI_CAP], a = ent >> 24, j = ent & 0xFFFFFFu, k = x % MXP_VTI_CAP;
            const uint32_t tb = __builtin_amdgcn_ds_bpermute((int)(a << 2), (int)TB);
            const uint2 w = *(const uint2*)(A.vt_tm + 2u * ((uint64_t)tb + (uint64_t)j * MXP_VTI_CAP + k));
            SM[(a * MXP_FILL_CHUNK + g) * MXP_VTI_CAP + k] = w.x;
            if (k == 0) SJ[a * MXP_FILL_CHUNK + g] = j;
            eor |= w.y;
        }
    }
    if (__ballot(eor != 0u)) {
        if (lane == 0) atomicOr(&eflag, 1u);
    }
    __syncthreads();
    const bool errs = eflag != 0u;
    const uint64_t N = A.n;
    const uint32_t Q1 = A.q1;
    const bool nt = !(A.flags & 128u);
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t FM = lane < n ? A.fill_masks[moff + lane] : 0u;
    // A wave-tile's inputs: the guard column's kinds, the classes per slot, the deferred-pair queue's
    // count and slot row.  The fast kernel loads tile t + 1's while tile t's words are stored: its
    // loads then wait only for themselves, not for the tile's 16 stores ahead of them in the
    // memory counter.
    struct TileIn {
        uint32_t k4, dk;
        uint64_t c[NVT];
        v4u sl;
    };
    auto fetch = [&](uint32_t t, TileIn& T) __attribute__((always_inline)) {
        const uint32_t q0 = A.q0 + ((bx * MXP_VTF_TILES + t) * 4u + wave) * 256u + lane * 4u;
        const bool vec = (N & 3u) == 0 && (Q1 & 3u) == 0 && (q0 & 3u) == 0;
        T.k4 = 0u;
        if (vec && q0 < Q1) {
            T.k4 = *(const uint32_t*)(A.kinds + (uint64_t)col * N + q0);
        } else {
            for (uint32_t r = 0; r < 4; r++)
                if (q0 + r < Q1) T.k4 |= (uint32_t)A.kinds[(uint64_t)col * N + q0 + r] << (8u * r);
        }
#pragma unroll
        for (uint32_t a = 0; a < NVT; a++) {
            const uint16_t* C = A.vt_cls + (uint64_t)a * MXP_VT_PITCH(N);
            uint64_t c = 0;
            if (vec && q0 < Q1) {
                c = *(const uint64_t*)(C + q0);
            } else {
                for (uint32_t r = 0; r < 4; r++)
                    if (q0 + r < Q1) c |= (uint64_t)C[q0 + r] << (16u * r);
            }
            T.c[a] = c;
        }
        T.dk = 0u;
        T.sl = v4u{0u, 0u, 0u, 0u};
        if (A.dtp_slots && q0 < Q1) {
            const uint64_t qi = (uint64_t)chunk * MXP_DTP_ROW(A.dtp_tiles) + (q0 >> 2);
            T.dk = A.dtp_qn[qi];
            T.sl = *(const v4u*)(A.dtp_slots + qi * 8u);
        }
    };
    TileIn nx;
    if constexpr (!kSlow) fetch(0u, nx);
    for (uint32_t t = 0; t < MXP_VTF_TILES; t++) {
        const uint32_t qw = A.q0 + ((bx * MXP_VTF_TILES + t) * 4u + wave) * 256u;
        if (qw >= Q1) break;
        if constexpr (kSlow) {
            if (!slow[t * 4u + wave]) continue;
        }
        TileIn cur;
        if constexpr (kSlow)
            fetch(t, cur);
        else
            cur = nx;
        const uint32_t q0 = qw + lane * 4u;
        // (the request count passes through an empty asm per tile, so the compiler derives each
        // unrolled group's row base here instead of hoisting 16 of them out of the tile loop into
        // spilled scalar registers)
        uint64_t Nt = N;
        asm volatile("" : "+s"(Nt));
        const bool vec = (N & 3u) == 0 && (Q1 & 3u) == 0 && (q0 & 3u) == 0;
        uint32_t bad[4];
#pragma unroll
        for (uint32_t r = 0; r < 4; r++) {
            const bool in = q0 + r < Q1;
            const uint32_t k = (cur.k4 >> (8u * r)) & 0xFFu;
            bad[r] = (in && !((okset >> k) & 1u)) ? ~0u : 0u;
        }
        // each request's byte address per slot: [a][g = 0][its class] (kept in registers: the
        // unrolled groups add only an immediate offset)
        uint32_t adb[NVT][4];
#pragma unroll
        for (uint32_t a = 0; a < NVT; a++)
#pragma unroll
            for (uint32_t r = 0; r < 4; r++)
                adb[a][r] = 4u * (a * MXP_FILL_CHUNK * MXP_VTI_CAP + ((uint32_t)(cur.c[a] >> (16u * r)) & (MXP_VTI_CAP - 1u)));
        const bool any = (bad[0] | bad[1] | bad[2] | bad[3]) != 0;
        const bool wbad = __ballot(any) != 0;
        DtpQueue dq;
        dq.decode(cur.dk, cur.sl);
        if constexpr (!kSlow) {
            if (t + 1u < MXP_VTF_TILES) fetch(t + 1u, nx);
        }
        const bool dany = __ballot(dq.q0 != ~0u) != 0;
        const bool derr = dany && dq.any_err();
        uint32_t anyerr[4] = {0u, 0u, 0u, 0u};
        // One group's words.  GroupC<g> (the fast path: a full chunk, no guard-kind errors in the
        // wave, no class error words in the chunk, no error-plane pairs in the wave) is unrolled at compile time -- the class words are ds_read_b32 at
        // the immediate offset g * 256, the pair test compares with an inline constant, the store is
        // the row's scalar base plus the lane's byte offset; GroupR (runtime g) is the general loop.
        auto group = [&](auto gc) __attribute__((always_inline)) {
            constexpr bool ct = decltype(gc)::ct;
            const uint32_t g = gc.value;
            if (ct && g >= n) return;  // (a rule set's last chunk: fewer groups)
            const uint32_t G = g0 + g;
            uint32_t m[4] = {0u, 0u, 0u, 0u}, e[4] = {0u, 0u, 0u, 0u};
            if constexpr (!ct) {
                const uint32_t mask = __builtin_amdgcn_readlane(FM, g);
#pragma unroll
                for (int r = 0; r < 4; r++) e[r] = bad[r] & mask;
                if (A.errlog && any && mask)
                    for (uint32_t r = 0; r < 4; r++)
                        if (e[r] && q0 + r < Q1) log_guard_errors(A, e[r], G * 32u, q0 + r);
            }
#pragma unroll
            for (uint32_t a = 0; a < NVT; a++)
#pragma unroll
                for (uint32_t r = 0; r < 4; r++)
                    m[r] |= *(const uint32_t*)((const char*)SM + adb[a][r] + g * (MXP_VTI_CAP * 4u));
            if constexpr (!ct) {
                if (errs) {
                    uint32_t ve[4] = {0u, 0u, 0u, 0u};
                    for (uint32_t a = 0; a < NVT; a++) {
                        const uint32_t j = SJ[a * MXP_FILL_CHUNK + g];
                        if (j == ~0u) continue;
                        const uint64_t row = (uint64_t)__builtin_amdgcn_readlane(TB, a) + (uint64_t)j * MXP_VTI_CAP;
#pragma unroll
                        for (uint32_t r = 0; r < 4; r++)
                            ve[r] |= A.vt_tm[2u * (row + ((adb[a][r] >> 2) & (MXP_VTI_CAP - 1u))) + 1u];
                    }
                    if (A.errlog) {
                        uint32_t c = 0;
#pragma unroll
                        for (int r = 0; r < 4; r++) c += q0 + r < Q1 ? (uint32_t)__builtin_popcount(ve[r]) : 0u;
                        vt_count_n(A, c);
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) e[r] |= ve[r];
                }
                if (dany) dq.merge(g, m, e);
#pragma unroll
                for (uint32_t r = 0; r < 4; r++) anyerr[r] |= e[r];
            } else {
                if (dany) dq.template merge_c<decltype(gc)::value, false>(m, e);
            }
            // (row bases wave-uniform: scalar arithmetic, one address add per store)
            uint32_t* const om = A.out_match ? A.out_match + (uint64_t)G * Nt : nullptr;
            uint32_t* const oe = A.out_err ? A.out_err + (uint64_t)G * Nt : nullptr;
            if (vec && q0 < Q1) {
                const v4u mv = v4u{m[0], m[1], m[2], m[3]};
                const v4u ev = v4u{e[0], e[1], e[2], e[3]};
                if (nt) {
                    if (om) __builtin_nontemporal_store(mv, (v4u*)(om + q0));
                    if (oe) __builtin_nontemporal_store(ev, (v4u*)(oe + q0));
                } else {
                    if (om) *(v4u*)(om + q0) = mv;
                    if (oe) *(v4u*)(oe + q0) = ev;
                }
            } else {
                for (uint32_t r = 0; r < 4; r++) {
                    if (q0 + r >= Q1) break;
                    if (om) om[q0 + r] = m[r];
                    if (oe) oe[q0 + r] = e[r];
                }
            }
        };
        if constexpr (kSlow) {
#pragma nounroll
            for (uint32_t g = 0; g < n; g++) group(GroupR{g});
        } else {
            const bool to_slow = wbad || errs || derr;
            if (lane == 0) slow[t * 4u + wave] = to_slow ? 1u : 0u;
            if (to_slow) continue;
            for_groups<0, MXP_FILL_CHUNK>(group);
        }
        if (A.req_err)
            for (uint32_t r = 0; r < 4; r++)
                if (anyerr[r] && q0 + r < Q1) A.req_err[q0 + r] = 1;
    }
}
static_assert(MXP_VTF_TILES * 4u == 16u, "mxp_vtfill_imm_slow: a thread per mark of 16 blocks");
#define MXP_VTFILL_IMM(K)                                                                                      \
    extern "C" __global__ __launch_bounds__(256) void mxp_vtfill_imm##K##_kernel(mxp_kargs A) {                \
        vtfill_imm_body<K, false>(A, blockIdx.x, blockIdx.y, gridDim.x);                                       \
    }                                                                                                          \
    extern "C" __global__ __launch_bounds__(256) void mxp_vtfill_imm_slow##K##_kernel(mxp_kargs A, uint32_t gx, \
                                                                                     uint32_t gy) {            \
        __shared__ uint32_t bm;                                                                                \
        const uint32_t vb0 = blockIdx.x * 16u, vb = vb0 + threadIdx.x / 16u;                                   \
        if (threadIdx.x == 0) bm = 0u;                                                                         \
        __syncthreads();                                                                                       \
        if (vb < gx * gy && A.vtf_slow[(uint64_t)vb * (MXP_VTF_TILES * 4u) + threadIdx.x % 16u])               \
            atomicOr(&bm, 1u << (threadIdx.x / 16u));                                                          \
        __syncthreads();                                                                                       \
        for (uint32_t m = bm; m; m &= m - 1u) {                                                                \
            const uint32_t b = vb0 + (uint32_t)__builtin_ctz(m);                                               \
            vtfill_imm_body<K, true>(A, b % gx, b / gx, gx);                                                   \
        }                                                                                                      \
    }
MXP_VTFILL_IMM(1)
MXP_VTFILL_IMM(2)
MXP_VTFILL_IMM(3)
MXP_VTFILL_IMM(4)
MXP_VTFILL_IMM(5)
MXP_VTFILL_IMM(6)
MXP_VTFILL_IMM(7)
MXP_VTFILL_IMM(8)
#undef MXP_VTFILL_IMM

// Deferred pairs, filed for the fill (kargs.dtp_*).  One workgroup per tile of 1024 requests (16
// index waves) files the tile's recorded pairs by (value-class fill chunk, lane quad = request / 4)
// into 8 u16 slots per quad (counts in LDS, MXP_DTP_WIN chunks at a time); a quad's pairs past 8
// are staged in LDS and appended to the overflow list with one global atomic per workgroup.
#define MXP_DTP_WIN 32u
#define MXP_DTP_OVQ 512u
#define MXP_DTP_HIST 16384u  // rule sets up to this size count deferred pairs in the sort kernel
extern "C" __global__ __launch_bounds__(256) void mxp_dtp_sort_kernel(mxp_kargs A) {
    // the next evaluation's overflow counters (kargs.dtp_ovf_next): reset here, no memset launch
    if (blockIdx.x == 0 && threadIdx.x < 2u && A.dtp_ovf_next) A.dtp_ovf_next[threadIdx.x] = 0u;
    // entries per (chunk of the window, quad): two u16 counters per word (a quad gets at most 4 x 512
    // pairs of one chunk)
    __shared__ uint32_t cnt[MXP_DTP_WIN * 128u];
    __shared__ uint32_t ovq[MXP_DTP_OVQ][2];
    __shared__ uint32_t ovn, ovbase;
    // fused hit counters (kargs.dtp_part): per rule the tile's true pairs, two u16 per word (a rule
    // has at most 1024 pairs in a tile of 1024 requests)
    extern __shared__ uint32_t hc[];  // (dynamic: (n_rules + 1) / 2 words when counting)
    const uint32_t tid = threadIdx.x, t = A.dtp_t0 + blockIdx.x;
    const bool hist = A.dtp_part != nullptr;
    const uint32_t R2 = (A.n_rules + 1u) / 2u;
    if (hist)
        for (uint32_t i = tid; i < R2; i += 256u) hc[i] = 0u;
    const uint32_t nwaves = (A.n + 63u) / 64u, w0 = t * 16u;
    const uint32_t nw = min(16u, nwaves - w0);
    const uint64_t nq = MXP_DTP_ROW(A.dtp_tiles);  // quads per chunk row
    for (uint32_t cw0 = 0; cw0 < A.dtp_nchunks; cw0 += MXP_DTP_WIN) {
        const uint32_t cwn = min(MXP_DTP_WIN, A.dtp_nchunks - cw0);
        for (uint32_t i = tid; i < cwn * 128u; i += 256u) cnt[i] = 0u;
        if (tid == 0) ovn = 0u;
        __syncthreads();
        // four index waves' lists at a time, four entries of each per thread: 16 entries' loads (entry,
        // then its chunk) in flight together (a list holds ~1k entries, so one step covers it)
        for (uint32_t wb = 0; wb < nw; wb += 4u) {
            uint32_t nl[4];
#pragma unroll
            for (uint32_t g = 0; g < 4u; g++) nl[g] = wb + g < nw ? min(uni(A.dtp_n[w0 + wb + g]), A.dtp_cap) : 0u;
            const uint32_t nmax = max(max(nl[0], nl[1]), max(nl[2], nl[3]));
            for (uint32_t i0 = tid; i0 < nmax; i0 += 1024u) {
            uint32_t ev[16], cv[16];
#pragma unroll
            for (uint32_t u = 0; u < 16u; u++) {
                const uint32_t g = u >> 2, i = i0 + 256u * (u & 3u);
                ev[u] = i < nl[g] ? A.dtp_ent[(uint64_t)(w0 + wb + g) * A.dtp_cap + i] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (uint32_t u = 0; u < 16u; u++) cv[u] = ev[u] != 0xFFFFFFFFu ? A.dtp_chunk[(ev[u] & 0x7FFFFFu) >> 5] : 0u;
#pragma unroll
            for (uint32_t u = 0; u < 16u; u++) {
                const uint32_t e = ev[u], w = wb + (u >> 2);
                if (e == 0xFFFFFFFFu) continue;
                const uint32_t rule = e & 0x7FFFFFu, ch = cv[u];
                // fused hit counters (first window pass): a true pair into the workgroup's histogram
                if (hist && cw0 == 0 && !((e >> 23) & 1u)) atomicAdd(&hc[rule >> 1], 1u << ((rule & 1u) << 4));
                const uint32_t c = (ch >> 8) - cw0, ql = w * 64u + (e >> 24);
                if (c >= cwn) continue;
                const uint32_t qi = c * 256u + (ql >> 2), sh = (qi & 1u) << 4;
                const uint32_t at = (atomicAdd(&cnt[qi >> 1], 1u << sh) >> sh) & 0xFFFFu;
                if (at < 8u) {
                    A.dtp_slots[((uint64_t)(cw0 + c) * nq + t * 256u + (ql >> 2)) * 8u + at] =
                        (uint16_t)(((ch & 0xFFu) << 8) | (((e >> 23) & 1u) << 7) | ((ql & 3u) << 5) | (e & 31u));
                    continue;
                }
                const uint32_t o = atomicAdd(&ovn, 1u);
                const uint32_t rr = rule | (((e >> 23) & 1u) << 31);
                if (o < MXP_DTP_OVQ) {
                    ovq[o][0] = t * 1024u + ql;
                    ovq[o][1] = rr;
                } else {  // (the LDS stage is full: straight to the list)
                    const uint32_t gi = atomicAdd(&A.dtp_ovf_n[0], 1u);
                    if (gi < A.dtp_ovf_cap) {
                        A.dtp_ovf[2ull * gi] = t * 1024u + ql;
                        A.dtp_ovf[2ull * gi + 1] = rr;
                    } else {
                        __hip_atomic_store(&A.dtp_ovf_n[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            }
        }
        __syncthreads();
        if (hist && cw0 == 0)  // the tile's counts, summed over the tiles by mxp_dtp_hits_kernel
            for (uint32_t i = tid; i < R2; i += 256u) A.dtp_part[(uint64_t)t * R2 + i] = hc[i];
        for (uint32_t i = tid; i < cwn * 256u; i += 256u)
            A.dtp_qn[(uint64_t)(cw0 + (i >> 8)) * nq + t * 256u + (i & 255u)] = (uint8_t)min((cnt[i >> 1] >> ((i & 1u) << 4)) & 0xFFFFu, 8u);
        const uint32_t no = min(ovn, MXP_DTP_OVQ);
        if (tid == 0 && no) ovbase = atomicAdd(&A.dtp_ovf_n[0], no);
        __syncthreads();
        for (uint32_t i = tid; i < no; i += 256u) {
            const uint32_t g = ovbase + i;
            if (g < A.dtp_ovf_cap) {
                A.dtp_ovf[2ull * g] = ovq[i][0];
                A.dtp_ovf[2ull * g + 1] = ovq[i][1];
            } else {
                __hip_atomic_store(&A.dtp_ovf_n[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
}


// The sort workgroups' per-tile histograms summed into the hit counters: a thread sums one u16
// pair column over 64 tiles (grid y = tile blocks) and adds the two rules' counts.
extern "C" __global__ __launch_bounds__(256) void mxp_dtp_hits_kernel(const uint32_t* __restrict__ part, uint32_t tiles,
                                                                      uint32_t n_rules, unsigned long long* hits) {
    const uint32_t R2 = (n_rules + 1u) / 2u;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= R2) return;
    const uint32_t t0 = blockIdx.y * 64u, t1 = min(t0 + 64u, tiles);
    uint32_t lo = 0, hi = 0;
#pragma unroll 8
    for (uint32_t t = t0; t < t1; t++) {
        const uint32_t v = part[(uint64_t)t * R2 + i];
        lo += v & 0xFFFFu;
        hi += v >> 16;
    }
    if (lo) atomicAdd(hits + 2u * i, (unsigned long long)lo);
    if (hi && 2u * i + 1u < n_rules) atomicAdd(hits + 2u * i + 1u, (unsigned long long)hi);
}

// Guard-index phase: the continuing pairs of indexed rules (`attr == K && <continuation>`), found
// per request by a hash lookup of its column value instead of by comparing against every rule.
// Workgroup = 4 wavefronts, one tile of 64 requests each (one request per lane).  Lanes walk their
// own posting lists in lockstep; at every step the lanes whose rules share a continuation template
// run it together (each lane's rule constants preloaded into its registers).  mxp_eval_kernel has
// already written both bitmaps for these rules (match 0, error on a failed guard type check); true
// and error results are OR-ed in.
namespace {

// In-wave pair queue (LDS): the postings the probes find are appended as (rule, request) pairs and
// run 64 at a time -- one pair per lane, lanes sharing a template together -- so the VM runs on
// dense wavefronts however sparse the hits are per request.  Entry: rule | table << 31 (table 1:
// kargs.rule_tmpl2, the composite resume point), request.
#define MXP_IXQ 256u
#ifndef MXP_LITE_WAVES
#define MXP_LITE_WAVES 5
#endif
__shared__ uint32_t g_ixq[4][MXP_IXQ][2];  // per wave of the index kernel's workgroup
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// no '\n' in bytes [L, n) of a string at an 8-aligned address (its words are read whole: the string
// pool is padded)
__device__ __forceinline__ bool tail_clear(StrRef s, uint32_t L) {
    for (uint32_t w = L / 8u; w * 8u < s.n; w++) {
        uint64_t x = ld8a(s.p + w * 8u) ^ 0x0A0A0A0A0A0A0A0Aull;  // (zero bytes: newlines)
        if (w * 8u < L) x |= (1ull << ((L - w * 8u) * 8u)) - 1ull;  // bytes before L
        if (s.n - w * 8u < 8u) x |= ~0ull << ((s.n - w * 8u) * 8u);  // bytes past the end
        // 0x80 where a byte of x is zero (exact per byte: no borrow between bytes)
        if (~(((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x | 0x7F7F7F7F7F7F7F7Full)) return false;
    }
    return true;
}

__shared__ uint64_t g_cm[4][64];  // dense-alias masks of the wave's 64 requests (kargs.dense_of)
struct PairQueue {
    uint32_t wave;
    uint32_t n;        // pending entries (wave-uniform)
    uint32_t ntrue;    // true pairs this lane has set (kargs.stats)
    uint32_t base;     // first request of the wave's tile
    // profiling instantiations only (kProf): time in run_pairs, its calls, VM passes, pairs
    uint64_t p_vm;
    uint32_t p_runs, p_passes, p_pairs;
};

// A true pair of an indexed rule: rules with many duplicates ("dense" canonical rules, kargs.dense_of)
// only set their bit in the request's mask (LDS) -- the wave writes the bits of the rule and all its
// aliases once per bitmap word at the end (inject_dense); the rest OR their bits in at once.
template <bool kDtp>
__device__ __forceinline__ uint32_t pair_true(const mxp_kargs& A, PairQueue& Q, uint32_t rule, uint32_t req) {
    if (A.dense_of) {
        const uint32_t d = A.dense_of[rule];
        if (d != 0xFFu) {
            atomicOr((unsigned long long*)&g_cm[Q.wave][req - Q.base], 1ull << d);
            return 0u;  // counted by mxp_inject_kernel
        }
    }
    return set_true<kDtp>(A, rule, req);
}

// run entries [off, off + cnt) of the queue, cnt <= 64
template <bool kRefs, bool kNfa, bool kDtp, bool kProf = false, bool kLite = false>
__device__ void run_pairs(const mxp_kargs& A, PairQueue& Q, uint32_t off, uint32_t cnt, uint64_t (*regs)[256],
                          uint32_t tid) {
    const uint64_t t0 = kProf ? (uint64_t)wall_clock64() : 0ull;
    const uint32_t lane = tid & 63u;
    wave_sync_lds();
    bool pending = lane < cnt;
    uint32_t rule = 0, req = 0, t = MXP_VM_DONE, res = MXP_VM_DONE;
    if (pending) {
        const uint32_t e = g_ixq[Q.wave][off + lane][0], w1 = g_ixq[Q.wave][off + lane][1];
        req = Q.base + (w1 & 63u);
        pending = e != 0xFFFFFFFFu;  // a direct posting, already OR-ed
        rule = e & 0x7FFFFFFFu;
        if (pending) t = w1 >> 8;
    }
    wave_sync_lds();
    for (uint64_t bal = __ballot(pending); bal; bal = __ballot(pending)) {
        const uint32_t tt = __builtin_amdgcn_readlane(t, (uint32_t)__builtin_ctzll(bal));
        const bool mine = pending && t == tt;
        const mxp_tmpl* T = A.tmpls + tt;
        const uint32_t toff = uni(T->off), pc0 = uni(T->pc0), len_t = uni(T->len), nconst = uni(T->nconst),
                       creg0 = uni(T->creg0);
        if (mine)
            for (uint32_t c = 0; c < nconst; c++) regs[creg0 + c][tid] = A.rconst[(uint64_t)rule * MXP_VM_MAXREG + c];
        cuint32* P = ((cuint32*)A.prog) + ((uint64_t)toff - pc0) * 4u;
        const uint32_t code = run_rule<kRefs, kNfa, kLite>(A, P, len_t, pc0, mine, rule, req, regs, tid, true);
        if (mine) res = code;
        pending = pending && !mine;
        if (kProf) Q.p_passes++;
    }
    // results out after the VM loop (its registers are dead here)
    if (res == PC_TRUE) Q.ntrue += pair_true<kDtp>(A, Q, rule, req);
    if (res >= PC_ERROR && res != MXP_VM_DONE) set_error<kDtp>(A, rule, req);
    if (kProf) {
        Q.p_vm += (uint64_t)wall_clock64() - t0;
        Q.p_runs++;
        Q.p_pairs += cnt;
    }
}

// Appends every lane's postings [start, start + len) to the queue (direct postings are true pairs:
// OR-ed at once) and runs full 64-pair batches; `final` drains the queue.  The free entries are
// shared out by a prefix sum over the lanes' remaining postings (lower lanes first), so the queue
// never overflows, one lane's long list fills whole batches (C2: a request without a path takes its
// service's ~39 equality postings in one round, not ten rounds of four), and the VM has one call
// site (one inlined copy).
// Literal-key regexp postings of a prefix slot (subject `s`, key length L; L = 0 elsewhere): code
// 509, an exact key, is a true pair when the subject ends at the key; code 508, a `.*$` tail key,
// when no '\n' follows it.  Direct postings and the dead literal-key ones take no queue entry.
template <bool kRefs, bool kNfa, bool kDtp, bool kProf = false, bool kLite = false>
__device__ __forceinline__ void process_slot(const mxp_kargs& A, PairQueue& Q, uint32_t tbl, uint32_t start,
                                             uint32_t len, uint32_t req, bool final, uint64_t (*regs)[256],
                                             uint32_t tid, StrRef s = StrRef{nullptr, 0}, uint32_t L = 0) {
    const uint32_t lane = tid & 63u;
    const uint32_t* __restrict__ tmpl_of = tbl ? A.rule_tmpl2 : A.rule_tmpl;
    uint32_t j0 = 0;
    for (;;) {
        if (Q.n < 64u && __ballot(j0 < len)) {
            const uint32_t want = j0 < len ? len - j0 : 0u, freeq = MXP_IXQ - Q.n;  // freeq > 192
            const uint32_t before = wave_incl_sum(want, lane) - want;
            const uint32_t take = before >= freeq ? 0u : min(want, freeq - before);
            // posting-major order: entry j of every lane, then entry j + 1, ...  Lanes whose requests
            // share a posting list (a common key) put the SAME rule side by side, so a 64-pair batch
            // runs one rule's constants and its true bits -- and its aliases' -- land in one bitmap
            // row: coalesced atomics instead of one row per lane
            const uint32_t tmax = wave_max(take);
            const uint64_t below = (1ull << lane) - 1ull;
            uint32_t pos = Q.n;
            for (uint32_t j = 0; j < tmax; j++) {
                uint32_t rule = 0, t = MXP_TMPL_SKIP;
                if (j < take) {
                    const uint32_t pe = A.postings[start + j0 + j];
                    rule = pe;
                    if (A.post_tmpl) {  // the template rides in the posting (kargs.postings)
                        rule = pe & 0x7FFFFFu;
                        const uint32_t code = pe >> 23;
                        t = code == 511u ? MXP_TMPL_DIRECT : code == 510u ? tmpl_of[rule]
                          : (code | 1u) == 509u  // (one test for both literal-key codes: no spills)
                              ? ((code == 509u ? s.n == L : tail_clear(s, L)) && L ? MXP_TMPL_DIRECT : MXP_TMPL_SKIP)
                              : code;
                    } else {
                        t = tmpl_of[rule];
                    }
                    if (t == MXP_TMPL_DIRECT) {
                        Q.ntrue += pair_true<kDtp>(A, Q, rule, req);
                        t = MXP_TMPL_SKIP;
                    }
                }
                const bool queued = t != MXP_TMPL_SKIP;
                const uint64_t act = __ballot(queued);
                if (queued) {
                    // (entry: rule | table, then the request's lane in the wave | template << 8)
                    const uint32_t at = pos + (uint32_t)__builtin_popcountll(act & below);
                    g_ixq[Q.wave][at][0] = rule | (tbl << 31);
                    g_ixq[Q.wave][at][1] = (req - Q.base) | (t << 8);
                }
                pos += (uint32_t)__builtin_popcountll(act);
            }
            j0 += take;
            Q.n = pos;
        }
        const bool more = __ballot(j0 < len) != 0;
        if (Q.n >= 64u || (Q.n > 0u && (final || more))) {
            const uint32_t k = min(Q.n, 64u);
            run_pairs<kRefs, kNfa, kDtp, kProf, kLite>(A, Q, Q.n - k, k, regs, tid);
            Q.n -= k;
            continue;
        }
        if (!more) break;
    }
}

// equality probe: postings of the entry whose key is v (len 0: none)
__device__ __forceinline__ void eq_probe(const mxp_kargs& A, uint32_t hoff, uint32_t hmask, uint64_t v, uint32_t& start,
                                         uint32_t& len) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    uint32_t fi = 0xFFFFFFFFu;
    for (uint32_t slot = mxp_hash64(v) & hmask;; slot = (slot + 1) & hmask) {
        const mxp_hent E = A.hents[hoff + slot];
        if (E.len == 0) break;
        if (E.klo == lo && E.khi == hi) {
            fi = hoff + slot;
            break;
        }
    }
    if (fi != 0xFFFFFFFFu) {
        start = A.hents[fi].start;
        len = A.hents[fi].len;
    }
}

// Incremental hash of a string's leading bytes (vm.h mxp_str_step / mxp_str_final): key lengths are
// probed in ascending order, so whole 8-byte words are folded in once.
struct PrefixHash {
    uint64_t h;
    uint32_t words;
    __device__ __forceinline__ uint64_t at(const uint8_t* p, uint32_t L) {
        for (; (words + 1) * 8u <= L; words++) h = mxp_str_step(h, ld8a(p + words * 8u));
        uint64_t hl = h;
        const uint32_t rem = L - words * 8u;
        if (rem) hl = mxp_str_step(hl, ld8a(p + words * 8u) & ((1ull << (rem * 8u)) - 1ull));
        return mxp_str_final(hl, L);
    }
    // the same hash from a string head (kargs.heads): L <= 12, words w0 (bytes 0..7), w1 (8..11)
    __device__ __forceinline__ uint64_t at_head(uint64_t w0, uint64_t w1, uint32_t L) {
        if (words == 0u && L >= 8u) {
            h = mxp_str_step(h, w0);
            words = 1u;
        }
        uint64_t hl = h;
        const uint32_t rem = L - words * 8u;
        if (rem) hl = mxp_str_step(hl, (words ? w1 : w0) & ((1ull << (rem * 8u)) - 1ull));
        return mxp_str_final(hl, L);
    }
};

// L leading bytes of a head (words w0, w1; L <= 12) against a key string at an 8-aligned address
__device__ __forceinline__ bool head_eq(uint64_t w0, uint64_t w1, const uint8_t* k, uint32_t L) {
    const uint64_t m0 = L >= 8u ? ~0ull : (1ull << (L * 8u)) - 1ull;
    if ((w0 ^ ld8a(k)) & m0) return false;
    if (L <= 8u) return true;
    return ((w1 ^ ld8a(k + 8)) & ((1ull << ((L - 8u) * 8u)) - 1ull)) == 0ull;
}

// Prefix (or composite K2) keys of KC consecutive key lengths probed together: the KC hashes, then
// the KC occupancy words, then the KC first entry pairs, then the KC postings ranges -- each round
// of loads independent across the lengths, so a wave waits ~3 round trips per KC lengths instead
// of ~2-3 per length (the waves of C4's lite index kernel were chains of such loads).  A slot
// whose entry belongs to another key continues its linear probe alone (load factor <= 1/8).
// Lengths past kc, past the string, or of lanes without a string (sok false) find nothing.  (The
// lite kernel's; MXP_LITE_WAVES 5 keeps its registers spill-free.)
#ifndef MXP_PROBE_KC
#define MXP_PROBE_KC 2
#endif
constexpr uint32_t KC = MXP_PROBE_KC;

// entry pair (E, K) at `at` against the key of length L: 1 match, 0 another key, -1 empty slot
__device__ __forceinline__ int entry_check(const mxp_kargs& A, const mxp_hent& E, const mxp_hent& K, uint32_t tag,
                                           bool comp, uint32_t vlo, uint32_t vhi, uint32_t L, StrRef s, uint32_t hw1,
                                           bool by_head) {
    if (E.len == 0) return -1;
    if (E.khi != tag) return 0;
    if (comp && (K.klo != vlo || K.khi != vhi)) return 0;
    if ((E.len >> 24) != min(L, 255u)) return 0;
    if (L <= (comp ? 12u : 20u)) {  // the key inline (see index_body)
        const uint64_t k0 = (uint64_t)E.klo | ((uint64_t)(comp ? K.start : K.klo) << 32);
        const uint64_t k1 = comp ? (uint64_t)K.len : ((uint64_t)K.khi | ((uint64_t)K.start << 32));
        const uint64_t w0 = by_head ? (uint64_t)s.p : ld8a(s.p);
        const uint64_t w1 = by_head ? (uint64_t)hw1 : (L > 8u ? ld8a(s.p + 8) : 0ull);
        const uint64_t w2 = L > 16u ? ld8a(s.p + 16) : 0ull;
        const uint64_t m0 = L >= 8u ? ~0ull : (1ull << (L * 8u)) - 1ull;
        const uint64_t m1 = L >= 16u ? ~0ull : L > 8u ? (1ull << ((L - 8u) * 8u)) - 1ull : 0ull;
        const uint64_t m2 = L > 16u ? (1ull << ((L - 16u) * 8u)) - 1ull : 0ull;
        return (((w0 ^ k0) & m0) == 0 && ((w1 ^ k1) & m1) == 0 && ((w2 ^ (uint64_t)K.len) & m2) == 0) ? 1 : 0;
    }
    const StrRef k = str_of(A, E.klo);
    return (k.n == L && (by_head ? head_eq((uint64_t)s.p, hw1, k.p, L) : bytes_eq_a(s.p, k.p, L))) ? 1 : 0;
}

__device__ __forceinline__ void probe_chunk(const mxp_kargs& A, PrefixHash& ph, StrRef s, uint32_t hw1, bool by_head,
                                            bool sok, bool comp, uint32_t vlo, uint32_t vhi, uint32_t pmask,
                                            uint32_t poff, uint32_t boff, const uint32_t* Ls, uint32_t kc,
                                            uint32_t (&st)[KC], uint32_t (&ln)[KC]) {
    uint32_t slot[KC], tag[KC], L[KC], bw[KC];
    bool act[KC];
#pragma unroll
    for (uint32_t j = 0; j < KC; j++) {
        L[j] = j < kc ? uni(Ls[j]) : 0u;
        act[j] = j < kc && sok && L[j] <= s.n;
        slot[j] = 0u;
        tag[j] = 0u;
        if (act[j]) {
            const uint64_t hf = by_head ? ph.at_head((uint64_t)s.p, hw1, L[j]) : ph.at(s.p, L[j]);
            slot[j] = (uint32_t)hf & pmask;
            tag[j] = (uint32_t)(hf >> 32);
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < KC; j++) bw[j] = act[j] && A.hbits ? A.hbits[boff + (slot[j] >> 5)] : ~0u;
    mxp_hent E[KC], K[KC];
#pragma unroll
    for (uint32_t j = 0; j < KC; j++) {
        act[j] = act[j] && ((bw[j] >> (slot[j] & 31u)) & 1u);
        if (act[j]) {
            E[j] = A.hents[poff + 2u * slot[j]];
            K[j] = A.hents[poff + 2u * slot[j] + 1u];
        }
    }
    uint32_t fi[KC];
#pragma unroll
    for (uint32_t j = 0; j < KC; j++) {
        fi[j] = 0xFFFFFFFFu;
        if (!act[j]) continue;
        int r = entry_check(A, E[j], K[j], tag[j], comp, vlo, vhi, L[j], s, hw1, by_head);
        // (another key in the slot: the rest of the linear probe, this length alone)
        for (uint32_t sl = (slot[j] + 1u) & pmask; r == 0; sl = (sl + 1u) & pmask) {
            if (A.hbits && !((A.hbits[boff + (sl >> 5)] >> (sl & 31u)) & 1u)) {
                r = -1;
                break;
            }
            slot[j] = sl;
            r = entry_check(A, A.hents[poff + 2u * sl], A.hents[poff + 2u * sl + 1u], tag[j], comp, vlo, vhi, L[j], s,
                            hw1, by_head);
        }
        if (r == 1) fi[j] = poff + 2u * slot[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < KC; j++) {
        st[j] = 0u;
        ln[j] = 0u;
        if (fi[j] != 0xFFFFFFFFu) {
            st[j] = A.hents[fi[j]].start;
            ln[j] = A.hents[fi[j]].len & 0xFFFFFFu;
        }
    }
}

}  // namespace

// Guard-index phase: the pairs of indexed rules, found per request by hash lookups of its column
// value (equality indexes), of its leading bytes at every key length the index holds (prefix
// indexes: `startsWith` atoms and anchored regexp literals), or of both (composite indexes:
// `A == K1 && B.startsWith(K2) && ...`) instead of by testing every rule.
// Workgroup = 4 wavefronts, one tile of 64 requests each (one request per lane).  mxp_eval_kernel
// has already written both bitmaps for these rules (match 0, error on a failed type check of the
// guard column); true and error results are OR-ed in.
namespace {

// kProf: the profiling instantiations (kargs.wave_t, MXP_WAVE_TIMES) -- the hot kernels carry no
// timing code
template <bool kRefs, bool kNfa = kRefs, bool kDtp = false, bool kProf = false, bool kLite = false>
__device__ __forceinline__ void index_body(const mxp_kargs& A, uint64_t (*regs)[256]) {
    // chunked prefix probes in the lite kernel only (same-box A/B, profiles/r5_s8_ab_probe_c{2,4}.log:
    // KC 2 at 5 waves/SIMD C4 0.697 -> 0.691 ms, C2 0.4005 -> 0.3983 ms; KC 4 slower)
    constexpr bool kChunk = kLite && KC > 1;
    // after the fill (kargs.dtp_gate): the deferred pairs' overflow list OR-ed in, then -- only when
    // that list filled -- every pair again
    if (A.dtp_gate) {
        const uint32_t no = min(uni(A.dtp_ovf_n[0]), A.dtp_ovf_cap);
        for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < no; i += gridDim.x * 256u) {
            const uint32_t q = A.dtp_ovf[2ull * i], e = A.dtp_ovf[2ull * i + 1];
            const uint32_t rule = e & 0x7FFFFFFFu;
            atomicOr(((e >> 31) ? A.out_err : A.out_match) + (uint64_t)(rule >> 5) * A.n + q, 1u << (rule & 31u));
        }
        // a counted evaluation's gate for the next one: stream (no true-pair count was kept)
        if (A.gate_out && blockIdx.x == 0 && threadIdx.x == 0) *A.gate_out = 0u;
        if (uni(*A.dtp_gate) == 0u) return;
    }
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = uni(tid >> 6);
    const uint64_t N = A.n;
    const uint32_t tile = blockIdx.x * 4u + wave;  // 64 requests per wave
    const uint64_t t_start = kProf ? (uint64_t)wall_clock64() : 0ull;
    PairQueue Q{wave, 0u, 0u, A.q0 + tile * 64u, 0ull, 0u, 0u, 0u};
    const uint32_t req = Q.base + (tid & 63u);
    const bool valid = req < A.q1;
    if (A.dense_of) g_cm[wave][tid & 63u] = 0ull;
    if (kDtp && (tid & 63u) == 0) g_dtpn[wave] = 0u;
    if constexpr (kDtp)
        if (A.req_err_init) g_rerr[wave][tid & 63u] = 0;
    if (A.dense_of || kDtp) wave_sync_lds();
    uint32_t nmark = 0;  // profiling (kargs.wave_t): slots done
    if (kProf && (tid & 63u) == 0)
        for (uint32_t i = 3; i < 8; i++) A.wave_t[8ull * tile + i] = 0ull;
    // x == n_idx: a last pass with no probes that drains the pair queue
    for (uint32_t x = 0; x <= A.n_idx; x++) {
        const bool final = x == A.n_idx;
        const mxp_index* X = A.idx + (final ? 0u : x);
        const uint32_t col = uni(X->col), okset = uni(X->okset), hmask = uni(X->hmask), hoff = uni(X->hoff),
                       kind = uni(X->prefix), plen0 = uni(X->plen0), nplen = uni(X->nplen);
        const bool comp = kind == MXP_IX_COMPOSITE;
        // kinds and values of both columns are loaded together (independent loads, one round trip)
        bool ok = false;
        uint64_t v = 0;
        if (valid && !final) {  // (the last pass only drains the queue)
            const uint32_t k = A.kinds[(uint64_t)col * N + req];
            const uint64_t vv = A.vals[(uint64_t)col * N + req];
            ok = ((okset >> k) & 1u) != 0;
            v = ok ? vv : 0ull;
        }
        // the string whose leading bytes are probed: the column itself (prefix index) or, for a
        // composite (A == K1 && B.startsWith(K2) && ...), B -- when B is not a string the lane takes
        // the composite's equality table over K1 instead (continuation after A: it raises B's error)
        bool sok = ok && kind == MXP_IX_PREFIX;
        uint64_t sv = v;
        uint32_t pmask = hmask, poff = hoff;
        if (comp) {
            const uint32_t col2 = uni(X->col2), okset2 = uni(X->okset2);
            pmask = uni(X->hmask2);
            poff = uni(X->hoff2);
            if (valid && !final) {
                const uint32_t k = A.kinds[(uint64_t)col2 * N + req];
                const uint64_t vv = A.vals[(uint64_t)col2 * N + req];
                sok = ok && ((okset2 >> k) & 1u) != 0;
                if (sok) sv = vv;
            }
        }
        // short keys (every key length <= 12) hash and verify from the string's head (kargs.heads):
        // one coalesced 16-byte load instead of the descriptor and the bytes (scattered, dependent)
        const uint32_t lmax = (!final && kind != MXP_IX_EQ && nplen) ? uni(A.plens[plen0 + nplen - 1u]) : 0u;
        const uint32_t hslot = uni(X->hslot), boff = uni(X->boff);
        const bool by_head = A.heads && hslot != MXP_VM_DONE && lmax <= 12u;
        // (the head's first word rides in the string pointer's registers: one of the two is live)
        StrRef s{nullptr, 0};
        uint32_t hw1 = 0;
        if (sok) {
            if (by_head) {
                const uint4 hd = A.heads[(uint64_t)hslot * N + req];
                s.p = (const uint8_t*)((uint64_t)hd.x | ((uint64_t)hd.y << 32));
                hw1 = hd.z;
                s.n = hd.w;
            } else {
                s = str_of(A, sv);
            }
        }
        PrefixHash ph{comp ? mxp_composite_seed(v) : 0ull, 0};
        const uint32_t vlo = (uint32_t)v, vhi = (uint32_t)(v >> 32);
        // probe slots: equality 1; prefix one per key length (shortest first); composite the
        // equality fallback, then one per K2 length
        const uint32_t nslot = final ? 1u : kind == MXP_IX_EQ ? 1u : nplen + (comp ? 1u : 0u);
        uint32_t cst[KC], cln[KC];  // the current chunk's postings ranges (probe_chunk; kChunk only)
        for (uint32_t p = 0; p < nslot; p++) {
            uint32_t start = 0, len = 0;
            const bool eq_slot = kind == MXP_IX_EQ || (comp && p == 0);
            if (final) {
            } else if (eq_slot) {
                if (ok && (!comp || !sok)) eq_probe(A, hoff, hmask, v, start, len);
            } else {
                const uint32_t pp = p - (comp ? 1u : 0u);  // (the prefix length's index)
                if constexpr (kChunk) {
                // KC lengths at a time (probe_chunk); this length's range from the chunk's registers
                const uint32_t j = pp % KC;
                if (j == 0u) probe_chunk(A, ph, s, hw1, by_head, sok, comp, vlo, vhi, pmask, poff, boff,
                                         A.plens + plen0 + pp, min(KC, nplen - pp), cst, cln);
#pragma unroll
                for (uint32_t i = 0; i < KC; i++)
                    if (i == j) {  // (selects: no dynamically indexed registers)
                        start = cst[i];
                        len = cln[i];
                    }
                } else {
                const uint32_t L = uni(A.plens[plen0 + pp]);
                // the probe yields the entry's index; its postings range is read after the loop (reading
                // start / len from the loop's 16-byte entry value was miscompiled at -O3 by this
                // ROCm 7.2 hipcc: lanes resumed with another entry's range)
                uint32_t fi = 0xFFFFFFFFu;
                if (sok && L <= s.n) {
                    const uint64_t hf = by_head ? ph.at_head((uint64_t)s.p, hw1, L) : ph.at(s.p, L);
                    const uint32_t tag = (uint32_t)(hf >> 32);
                    for (uint32_t slot = (uint32_t)hf & pmask;; slot = (slot + 1) & pmask) {
                        // an empty slot, told by the occupancy bitmap (no entry-pair request)
                        if (A.hbits && !((A.hbits[boff + (slot >> 5)] >> (slot & 31u)) & 1u)) break;
                        // entry pairs (vm.h mxp_index): both halves in one 32-byte load pair
                        const uint32_t at = poff + 2u * slot;
                        const mxp_hent E = A.hents[at];
                        const mxp_hent K = A.hents[at + 1u];
                        if (E.len == 0) break;
                        if (E.khi != tag) continue;
                        if (comp && (K.klo != vlo || K.khi != vhi)) continue;
                        if ((E.len >> 24) != min(L, 255u)) continue;  // (this order: no spills in the lite kernel)
                        if (L <= (comp ? 12u : 20u)) {  // the key inline: no key-string loads
                            // key words: composite {bytes 0..3 | 4..7, 8..11}, prefix {0..3 | 4..7, 8..15, 16..19}
                            const uint64_t k0 = (uint64_t)E.klo | ((uint64_t)(comp ? K.start : K.klo) << 32);
                            const uint64_t k1 = comp ? (uint64_t)K.len : ((uint64_t)K.khi | ((uint64_t)K.start << 32));
                            const uint64_t w0 = by_head ? (uint64_t)s.p : ld8a(s.p);
                            const uint64_t w1 = by_head ? (uint64_t)hw1 : (L > 8u ? ld8a(s.p + 8) : 0ull);
                            const uint64_t w2 = L > 16u ? ld8a(s.p + 16) : 0ull;  // (prefix keys only; L <= 12 by head)
                            const uint64_t m0 = L >= 8u ? ~0ull : (1ull << (L * 8u)) - 1ull;
                            const uint64_t m1 = L >= 16u ? ~0ull : L > 8u ? (1ull << ((L - 8u) * 8u)) - 1ull : 0ull;
                            const uint64_t m2 = L > 16u ? (1ull << ((L - 16u) * 8u)) - 1ull : 0ull;
                            if (((w0 ^ k0) & m0) == 0 && ((w1 ^ k1) & m1) == 0 && ((w2 ^ (uint64_t)K.len) & m2) == 0) {
                                fi = at;
                                break;
                            }
                            continue;
                        }
                        const StrRef k = str_of(A, E.klo);
                        if (k.n == L && (by_head ? head_eq((uint64_t)s.p, hw1, k.p, L) : bytes_eq_a(s.p, k.p, L))) {
                            fi = at;
                            break;
                        }
                    }
                }
                if (fi != 0xFFFFFFFFu) {
                    start = A.hents[fi].start;
                    len = A.hents[fi].len & 0xFFFFFFu;
                }
                }
            }
            if (A.flags & 1024u) {  // ablation: probes only (results invalid)
                if (len) Q.ntrue += start & 1u;
                continue;
            }
            if (final || __ballot(len != 0))
                process_slot<kRefs, kNfa, kDtp, kProf, kLite>(A, Q, comp && p > 0 ? 1u : 0u, start, len, req, final, regs, tid,
                                                              s, kind == MXP_IX_PREFIX && !eq_slot && !final
                                                                     ? uni(A.plens[plen0 + p]) : 0u);
            if (kProf && (tid & 63u) == 0 && (final || nmark < 4u)) {  // profiling: phase marks
                A.wave_t[8ull * tile + 3u + (final ? 4u : nmark)] = (uint64_t)wall_clock64();
                nmark++;
            }
        }
    }
    if (A.dense_of) {  // masks for mxp_inject_kernel
        wave_sync_lds();
        if (valid) A.dense_cm[req] = g_cm[wave][tid & 63u];
    }
    if (kDtp) {  // the tile's deferred-pair count for mxp_dtp_sort_kernel
        wave_sync_lds();
        if ((tid & 63u) == 0) A.dtp_n[Q.base >> 6] = min(g_dtpn[wave], A.dtp_cap);
        // the evaluation's first writer of the request error flags: all of the tile's, one
        // coalesced store (the later kernels only set flags; no memset)
        if (A.req_err && A.req_err_init && valid) A.req_err[req] = g_rerr[wave][tid & 63u];
    }
    if (kProf && (tid & 63u) == 0) {  // profiling: this tile's start / end (100 MHz clock), XCC
        A.wave_t[8ull * tile] = t_start;
        A.wave_t[8ull * tile + 1] = (uint64_t)wall_clock64();
        A.wave_t[8ull * tile + 2] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) |  // hwreg(XCC_ID, 0, 4)
                                    ((uint64_t)Q.p_passes << 8) | ((uint64_t)Q.p_runs << 24) | ((uint64_t)Q.p_pairs << 40);
        A.wave_t[8ull * tile + 6] = Q.p_vm;  // (mark 3 of 0..3 is unused by these workloads: time in run_pairs)
    }
    if (A.stats) {
        uint32_t t = Q.ntrue;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += (uint32_t)__shfl_xor((int)t, off, 64);
        if ((tid & 63u) == 0 && t) atomicAdd((unsigned long long*)A.stats, (unsigned long long)t);
    }
}

}  // namespace

// 6 waves/SIMD (80 VGPRs, two of them spilled: 12 bytes of scratch per lane).  Same-box A/B against
// the 5-wave build without spills (MXP_DEBUG_FLAGS 8192): C4 5.31 -> 5.10 ms, C2 0.720 vs 0.718 ms
// (profiles/r1_v17_ab_ix6_*.log)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void mxp_index_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false>(A, regs);
}
// deferred index pairs (kargs.dtp_ent): true / error pairs recorded for the value-class fill.  5
// waves/SIMD (96 VGPRs, 20 bytes of scratch) against 6 (80 VGPRs, 56 bytes of spills, which the PMC
// counters see as ~80 MB of scratch writes per C2 evaluation): same-box C2 0.531 / 0.532 -> 0.524 /
// 0.522 ms, C4 1.512 / 1.536 -> 1.491 / 1.519 ms (4 waves: 0.522, 1.514; profiles/r3_v3_ab_ix_occupancy_*.log)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void mxp_index_dtp_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false, false, true>(A, regs);
}
// ... for lite continuation templates (kargs.tmpl_lite: no lookups, virtual columns or regexps)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MXP_LITE_WAVES))) void mxp_index_dtp_lite_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false, false, true, false, true>(A, regs);
}
// profiling (MXP_WAVE_TIMES): the two hot instantiations with wave start / end / phase marks
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void mxp_index_prof_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false, false, false, true>(A, regs);
}
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void mxp_index_dtp_prof_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false, false, true, true>(A, regs);
}
// MXP_DEBUG_FLAGS 8192: the same body at 5 waves/SIMD (no scratch) -- A/B ablation
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void mxp_index5_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false>(A, regs);
}

// mxp_index_kernel for rule sets / batches with bit-parallel NFA regexps (kargs.nfa)
extern "C" __global__ __launch_bounds__(256) void mxp_index_nfa_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<false, true>(A, regs);
}

// mxp_index_kernel with referenced-attribute records (mxp_eval_refs)
extern "C" __global__ __launch_bounds__(256) void mxp_index_refs_kernel(mxp_kargs A) {
    __shared__ uint64_t regs[MXP_VM_MAXREG][256];
    index_body<true>(A, regs);
}

// After mxp_index_kernel, when the rule set has dense canonical rules (kargs.dense_of): every bitmap
// word holding a dense rule or alias gets the bits of its requests' masks with one coalesced atomic
// per word and wavefront (lane = request), plus the fused hit counters of those rules.  Words whose
// dense rules are false for the whole wave are skipped.  Workgroup = 4 waves x 64 requests.
extern "C" __global__ __launch_bounds__(256) void mxp_inject_kernel(mxp_kargs A) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t req = A.q0 + (blockIdx.x * 4u + uni(threadIdx.x >> 6)) * 64u + lane;
    const bool valid = req < A.q1;
    const uint64_t cm = valid ? A.dense_cm[req] : 0ull;
    uint32_t mlo = (uint32_t)cm, mhi = (uint32_t)(cm >> 32);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mlo |= (uint32_t)__shfl_xor((int)mlo, off, 64);
        mhi |= (uint32_t)__shfl_xor((int)mhi, off, 64);
    }
    const uint64_t M = ((uint64_t)uni(mhi) << 32) | uni(mlo);
    if (M == 0) return;
    uint32_t t = 0;  // pairs set (kargs.stats)
    // slots of 16 dwords (vm.h MXP_INJ_*): dense-id mask, word, count, up to 12 entries -- one
    // scalar s_load_dwordx16 each
    for (uint32_t k = 0; k < A.n_inj; k++) {
        const cuint32* S = (const cuint32*)A.inj + (uint64_t)k * MXP_INJ_SLOT;
        const uint64_t dm = (uint64_t)S[0] | ((uint64_t)S[1] << 32);
        if (!(dm & M)) continue;
        const uint32_t w = S[2], n = S[3];
        uint32_t bits = 0;
#pragma unroll
        for (uint32_t j = 0; j < MXP_INJ_SLOT - 4; j++) {
            if (j >= n) break;
            const uint32_t ent = S[4 + j];  // bit | dense id << 5
            const uint32_t on = (uint32_t)(cm >> (ent >> 5)) & 1u;
            bits |= on << (ent & 31u);
            if (counting(A)) {
                const uint32_t c = (uint32_t)__builtin_popcountll(__ballot(on != 0));
                if (lane == 0 && c) atomicAdd(A.hits + w * 32u + (ent & 31u), (unsigned long long)c);
            }
        }
        if (bits && A.out_match) atomicOr(A.out_match + (uint64_t)w * A.n + req, bits);
        t += (uint32_t)__builtin_popcount(bits);
    }
    if (A.stats) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += (uint32_t)__shfl_xor((int)t, off, 64);
        if (lane == 0 && t) atomicAdd((unsigned long long*)A.stats, (unsigned long long)t);
    }
}

// Per-rule hit counters: hits[rule] += number of requests whose match bit for the rule is set.
// The bitmap is streamed once (1.3 GB at R = 10k, N = 1M), so the counting must cost well under one
// VALU op per word and lane: each lane folds its words into bit-sliced counters with a Harley-Seal
// carry-save adder tree (ones / twos / fours / eights / sixteens planes, then one byte-packed
// "thirty-twos" counter per bit: P[j] byte f counts bit 8 f + j), about 3.3 VALU ops per word.
// The per-bit counts are unpacked once at the end, reduced over the block and added with one
// atomic per rule.  Grid: x = 32-rule word, y = request slices (sized so that no byte counter
// exceeds 255 steps).  Loads: 8 x 16 B per lane per step, each a contiguous 1 KB per wavefront.
namespace {

__device__ __forceinline__ void csa(uint32_t& h, uint32_t& l, uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t u = a ^ b;
    h = (a & b) | (u & c);
    l = u ^ c;
}

// 16 words into the running planes; returns the sixteens carry-out
__device__ __forceinline__ uint32_t hs16(const uint32_t* d, uint32_t& ones, uint32_t& twos, uint32_t& fours,
                                         uint32_t& eights) {
    uint32_t twosA, twosB, foursA, foursB, eightsA, eightsB, sixteens;
    csa(twosA, ones, ones, d[0], d[1]);
    csa(twosB, ones, ones, d[2], d[3]);
    csa(foursA, twos, twos, twosA, twosB);
    csa(twosA, ones, ones, d[4], d[5]);
    csa(twosB, ones, ones, d[6], d[7]);
    csa(foursB, twos, twos, twosA, twosB);
    csa(eightsA, fours, fours, foursA, foursB);
    csa(twosA, ones, ones, d[8], d[9]);
    csa(twosB, ones, ones, d[10], d[11]);
    csa(foursA, twos, twos, twosA, twosB);
    csa(twosA, ones, ones, d[12], d[13]);
    csa(twosB, ones, ones, d[14], d[15]);
    csa(foursB, twos, twos, twosA, twosB);
    csa(eightsB, fours, fours, foursA, foursB);
    csa(sixteens, eights, eights, eightsA, eightsB);
    return sixteens;
}

template <bool kVec>
__device__ __forceinline__ void hits_body(const uint32_t* __restrict__ row, uint32_t n, uint32_t n_rules,
                                          unsigned long long* __restrict__ hits) {
    const uint32_t w = blockIdx.x;
    const uint32_t nthreads = gridDim.y * blockDim.x;
    const uint32_t t = blockIdx.y * blockDim.x + threadIdx.x;
    uint32_t ones = 0, twos = 0, fours = 0, eights = 0, sixteens = 0;
    uint32_t P[8];
#pragma unroll
    for (int j = 0; j < 8; j++) P[j] = 0;
    for (uint64_t base = 0; base < n; base += nthreads * 32u) {
        uint32_t d[32];
        if (kVec) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint64_t i = base + ((uint64_t)j * nthreads + t) * 4u;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (i < n) v = *(const uint4*)(row + i);
                d[4 * j] = v.x;
                d[4 * j + 1] = v.y;
                d[4 * j + 2] = v.z;
                d[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const uint64_t i = base + (uint64_t)j * nthreads + t;
                d[j] = i < n ? row[i] : 0u;
            }
        }
        const uint32_t sA = hs16(d, ones, twos, fours, eights);
        const uint32_t sB = hs16(d + 16, ones, twos, fours, eights);
        uint32_t thirtytwos;
        csa(thirtytwos, sixteens, sixteens, sA, sB);
#pragma unroll
        for (int j = 0; j < 8; j++) P[j] += (thirtytwos >> j) & 0x01010101u;
    }
    __shared__ uint32_t red[32][8];
#pragma unroll
    for (int k = 0; k < 32; k++) {
        uint32_t c = 32u * ((P[k & 7] >> (8 * (k >> 3))) & 0xFFu) + 16u * ((sixteens >> k) & 1u) +
                     8u * ((eights >> k) & 1u) + 4u * ((fours >> k) & 1u) + 2u * ((twos >> k) & 1u) + ((ones >> k) & 1u);
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor((int)c, off, 64);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        uint32_t c = 0;
        for (uint32_t i = 0; i < blockDim.x / 64; i++) c += red[threadIdx.x][i];
        const uint32_t rule = w * 32 + threadIdx.x;
        if (rule < n_rules && c) atomicAdd(&hits[rule], (unsigned long long)c);
    }
}

}  // namespace

// The next evaluation's fused / streamed choice (block (0, 0), before anything else reads it): gate
// = 1 when this evaluation's guard-index true pairs were few enough (stats x 125 <= words x
// requests: one atomic per true pair costs less than re-reading the match bitmap), and the pair
// count reset for that evaluation.  force: 1 always fused, 2 never.
__device__ __forceinline__ void next_gate(unsigned long long* stats, uint32_t* gate_next, uint32_t n, uint32_t force) {
    if (!gate_next || blockIdx.x || blockIdx.y || threadIdx.x) return;
    const unsigned long long v = *stats;
    *gate_next = force == 1u ? 1u : force == 2u ? 0u : (v * 125ull <= (unsigned long long)gridDim.x * n ? 1u : 0u);
    *stats = 0ull;
}

extern "C" __global__ __launch_bounds__(256) void mxp_hits_kernel(const uint32_t* __restrict__ match, uint32_t n,
                                                                  uint32_t n_rules,
                                                                  unsigned long long* __restrict__ hits,
                                                                  const uint32_t* __restrict__ gate,
                                                                  unsigned long long* stats, uint32_t* gate_next,
                                                                  uint32_t force) {
    next_gate(stats, gate_next, n, force);
    if (gate && *gate) return;  // the evaluation kernels counted (fused)
    hits_body<true>(match + (uint64_t)blockIdx.x * n, n, n_rules, hits);
}

// ragged n (rows not 16-byte aligned): one word per load
extern "C" __global__ __launch_bounds__(256) void mxp_hits_ragged_kernel(const uint32_t* __restrict__ match, uint32_t n,
                                                                         uint32_t n_rules,
                                                                         unsigned long long* __restrict__ hits,
                                                                         const uint32_t* __restrict__ gate,
                                                                         unsigned long long* stats, uint32_t* gate_next,
                                                                         uint32_t force) {
    next_gate(stats, gate_next, n, force);
    if (gate && *gate) return;
    hits_body<false>(match + (uint64_t)blockIdx.x * n, n, n_rules, hits);
}

extern "C" hipError_t mxp_launch_eval(const mxp_kargs* args, uint32_t grid_x, uint32_t grid_y, int vm, hipStream_t s) {
    if (vm == 2 && args->refs)
        hipLaunchKernelGGL(mxp_eval_deep_refs_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (vm == 2 && args->nfa)
        hipLaunchKernelGGL(mxp_eval_deep_nfa_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (vm == 2)
        hipLaunchKernelGGL(mxp_eval_deep_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (vm && args->refs)
        hipLaunchKernelGGL(mxp_eval_refs_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (vm && args->nfa)
        hipLaunchKernelGGL(mxp_eval_nfa_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (vm)
        hipLaunchKernelGGL(mxp_eval_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else if (args->flags & 65536u)
        hipLaunchKernelGGL(mxp_guard_kernel, dim3(grid_x, grid_y), dim3(256), 0, s, *args);
    else
        hipLaunchKernelGGL(mxp_guard2_kernel, dim3((grid_x + 1) / 2, grid_y), dim3(256), 0, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_dtp_hits(const uint32_t* part, uint32_t tiles, uint32_t n_rules,
                                          unsigned long long* hits, hipStream_t s) {
    const uint32_t R2 = (n_rules + 1u) / 2u;
    hipLaunchKernelGGL(mxp_dtp_hits_kernel, dim3((R2 + 255u) / 256u, (tiles + 63u) / 64u), dim3(256), 0, s, part, tiles,
                       n_rules, hits);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_fill(const mxp_kargs* args, uint32_t n_fills, hipStream_t s) {
    if (args->dtp_slots) {
        hipLaunchKernelGGL(mxp_fill_dtp_kernel, dim3((args->q1 - args->q0 + 1023u) / 1024u, n_fills), dim3(256), 0, s, *args);
        return hipGetLastError();
    }
    const uint32_t per_block = 1024u * (args->fill_span ? args->fill_span : 1u);
    hipLaunchKernelGGL(mxp_fill_kernel, dim3((args->q1 - args->q0 + per_block - 1) / per_block, n_fills), dim3(256), 0, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_vtfill(const mxp_kargs* args, uint32_t n_fills, hipStream_t s) {
    if (args->flags & 2097152u) {
        hipLaunchKernelGGL(mxp_vtfill_kernel, dim3((args->q1 - args->q0 + 1023u) / 1024u, n_fills), dim3(256), 0, s, *args);
    } else {
        const uint32_t per = 1024u * MXP_VTF_TILES;
        const dim3 grid((args->q1 - args->q0 + per - 1u) / per, n_fills);
        // every active class table at 64 slots: the immediate-offset kernel for this many columns
        // (flag 33554432: mxp_vtfill_lds_kernel -- A/B)
        // (and its general loop for the wave-tiles it leaves, kargs.vtf_slow)
        void (*k)(mxp_kargs) = mxp_vtfill_lds_kernel;
        void (*ks)(mxp_kargs, uint32_t, uint32_t) = nullptr;
        if (args->vt_imm && args->vtf_slow && !(args->flags & 33554432u)) {
            switch (args->n_vt) {
#define MXP_VTFILL_CASE(K)                  \
    case K:                                 \
        k = mxp_vtfill_imm##K##_kernel;      \
        ks = mxp_vtfill_imm_slow##K##_kernel; \
        break;
                MXP_VTFILL_CASE(1)
                MXP_VTFILL_CASE(2)
                MXP_VTFILL_CASE(3)
                MXP_VTFILL_CASE(4)
                MXP_VTFILL_CASE(5)
                MXP_VTFILL_CASE(6)
                MXP_VTFILL_CASE(7)
                MXP_VTFILL_CASE(8)
#undef MXP_VTFILL_CASE
            default: break;
            }
        }
        hipLaunchKernelGGL(k, grid, dim3(256), 0, s, *args);
        // (the slow kernel's workgroups take 16 of the fast grid's blocks each: one flag byte per
        // thread, then the marked blocks in turn -- a launch of the fast grid's 5,120 blocks, each
        // reading its marks, took 7 us on C4)
        if (ks) hipLaunchKernelGGL(ks, dim3((grid.x * grid.y + 15u) / 16u), dim3(256), 0, s, *args, grid.x, grid.y);
    }
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_dtp_sort(const mxp_kargs* args, hipStream_t s) {
    const size_t lds = args->dtp_part ? (size_t)((args->n_rules + 1u) / 2u) * 4u : 0u;
    hipLaunchKernelGGL(mxp_dtp_sort_kernel, dim3(args->dtp_tn ? args->dtp_tn : args->dtp_tiles), dim3(256), lds, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_vt_classify(const mxp_kargs* args, hipStream_t s) {
    hipLaunchKernelGGL(mxp_vt_classify_kernel, dim3((args->q1 - args->q0 + MXP_VTC_REQ - 1u) / MXP_VTC_REQ), dim3(256), 0, s,
                       *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_vt_lookup(const mxp_kargs* args, hipStream_t s) {
    hipLaunchKernelGGL(mxp_vt_lookup_kernel, dim3((args->q1 - args->q0 + 1023u) / 1024u, args->n_vt), dim3(256), 0, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_vt_eval(const mxp_kargs* args, uint32_t tiles, uint32_t wchunks, hipStream_t s) {
    if (!tiles || !wchunks) return hipSuccess;
    if (args->nfa)
        hipLaunchKernelGGL(mxp_vt_eval_nfa_kernel, dim3(tiles, wchunks), dim3(256), 0, s, *args);
    else
        hipLaunchKernelGGL(mxp_vt_eval_kernel, dim3(tiles, wchunks), dim3(256), 0, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_inject(const mxp_kargs* args, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(mxp_inject_kernel, dim3(grid), dim3(256), 0, s, *args);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_index(const mxp_kargs* args, uint32_t grid, hipStream_t s) {
    if (args->refs)
        hipLaunchKernelGGL(mxp_index_refs_kernel, dim3(grid), dim3(256), 0, s, *args);
    else if (args->nfa)
        hipLaunchKernelGGL(mxp_index_nfa_kernel, dim3(grid), dim3(256), 0, s, *args);
    else if (args->dtp_ent && args->wave_t)
        hipLaunchKernelGGL(mxp_index_dtp_prof_kernel, dim3(grid), dim3(256), 0, s, *args);
    else if (args->dtp_ent && args->tmpl_lite)
        hipLaunchKernelGGL(mxp_index_dtp_lite_kernel, dim3(grid), dim3(256), 0, s, *args);
    else if (args->dtp_ent)
        hipLaunchKernelGGL(mxp_index_dtp_kernel, dim3(grid), dim3(256), 0, s, *args);
    else if (args->wave_t)
        hipLaunchKernelGGL(mxp_index_prof_kernel, dim3(grid), dim3(256), 0, s, *args);
    else
        if (args->flags & 8192u)
            hipLaunchKernelGGL(mxp_index5_kernel, dim3(grid), dim3(256), 0, s, *args);
        else
            hipLaunchKernelGGL(mxp_index_kernel, dim3(grid), dim3(256), 0, s, *args);
    return hipGetLastError();
}

// String heads (kargs.heads): per column and request, a string value's first 12 bytes (zero past
// its length; pools are 8-aligned with 16 bytes of tail slack) and its length; zero for other kinds.
// Only the columns a prefix or composite index probes have heads: row k of `heads` is column cols[k].
extern "C" __global__ __launch_bounds__(256) void mxp_heads_kernel(mxp_kargs A, const uint32_t* __restrict__ cols,
                                                                   uint4* __restrict__ heads) {
    const uint32_t req = blockIdx.x * 256u + threadIdx.x, row = blockIdx.y;
    if (req >= A.n) return;
    const uint64_t at = (uint64_t)cols[row] * A.n + req;
    uint4 h = make_uint4(0u, 0u, 0u, 0u);
    if (A.kinds[at] == MXP_STRING) {
        const StrRef r = str_of(A, A.vals[at]);
        const uint64_t w0 = r.n ? ld8a(r.p) : 0ull, w1 = r.n > 8u ? ld8a(r.p + 8) : 0ull;
        const uint64_t m0 = r.n >= 8u ? ~0ull : (1ull << (r.n * 8u)) - 1ull;
        const uint64_t m1 = r.n >= 12u ? 0xFFFFFFFFull : r.n > 8u ? (1ull << ((r.n - 8u) * 8u)) - 1ull : 0ull;
        h = make_uint4((uint32_t)(w0 & m0), (uint32_t)((w0 & m0) >> 32), (uint32_t)(w1 & m1), r.n);
    }
    heads[(uint64_t)row * A.n + req] = h;
}

extern "C" hipError_t mxp_launch_heads(const mxp_kargs* args, const uint32_t* cols, uint32_t nrow, uint4* heads, hipStream_t s) {
    hipLaunchKernelGGL(mxp_heads_kernel, dim3((args->n + 255u) / 256u, nrow), dim3(256), 0, s, *args, cols, heads);
    return hipGetLastError();
}

// Fused or streamed hit counters, decided on the device without a host round trip: after an
// evaluation, gate = 1 when its guard-index true pairs were few enough (stats x 125 <= words x
// requests: one atomic per true pair costs less than re-reading the match bitmap) -- the NEXT
// evaluation's kernels then count in place and its mxp_hits_kernel returns at once; else the kernels
// skip counting and mxp_hits_kernel streams the bitmap.  force: 1 always fused, 2 never.
extern "C" __global__ void mxp_hits_gate_kernel(const unsigned long long* stats, uint32_t n, uint32_t n_words,
                                                uint32_t* gate, uint32_t force) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *gate = force == 1u ? 1u : force == 2u ? 0u : (*stats * 125ull <= (unsigned long long)n_words * n ? 1u : 0u);
}

extern "C" hipError_t mxp_launch_hits_gate(const unsigned long long* stats, uint32_t n, uint32_t n_words,
                                           uint32_t* gate, uint32_t force, hipStream_t s) {
    hipLaunchKernelGGL(mxp_hits_gate_kernel, dim3(1), dim3(64), 0, s, stats, n, n_words, gate, force);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_hits(const uint32_t* match, uint32_t n, uint32_t n_rules, uint32_t n_words,
                                      unsigned long long* hits, hipStream_t s, const uint32_t* gate,
                                      unsigned long long* stats, uint32_t* gate_next, uint32_t force) {
    // slices: enough blocks to fill the chip (~16 per CU), at least 32 words per thread, and at most
    // 255 32-word steps per thread (the byte-packed counters)
    const uint64_t per_block = 256ull * 32u;
    uint64_t gy = (4096u + n_words - 1) / (n_words ? n_words : 1);
    const uint64_t most = (n + per_block - 1) / per_block, least = (n + per_block * 255u - 1) / (per_block * 255u);
    if (gy > most) gy = most;
    if (gy < least) gy = least;
    if (gy < 1) gy = 1;
    if (gy > 65535) return hipErrorInvalidValue;
    if ((n & 3u) == 0 && (((uintptr_t)match) & 15u) == 0)
        hipLaunchKernelGGL(mxp_hits_kernel, dim3(n_words, (uint32_t)gy), dim3(256), 0, s, match, n, n_rules, hits, gate,
                           stats, gate_next, force);
    else
        hipLaunchKernelGGL(mxp_hits_ragged_kernel, dim3(n_words, (uint32_t)gy), dim3(256), 0, s, match, n, n_rules, hits,
                           gate, stats, gate_next, force);
    return hipGetLastError();
}
