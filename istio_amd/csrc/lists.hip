// lists.hip -- gfx950 list-adapter check kernel (lists.cpp builds the tables).
//
// One symbol per lane.  HandleListEntry (mixer/adapter/list/list.go:68-101) on each:
//   string lists   hash the symbol 8 bytes at a time (ASCII upper-cased on the fly for the
//                  case-insensitive kind; a symbol with bytes >= 0x80 takes Go's strings.ToUpper
//                  per rune, goupper.h), probe the open-addressing table, compare bytes on a hash
//                  hit (stringList.go:73-80);
//   regex lists    one DFA for the union of the patterns (regexList.go:26-33: first match wins,
//                  and only "found" is reported), stepped rune by rune (dfa_dev.h);
//   IP lists       net.ParseIP on the symbol (netparse.h, the same code the host uses), then a
//                  binary search of the disjoint interval set of the address family
//                  (ipList.go:77-92; "is not a valid IP address" -> INVALID_ARGUMENT);
// then the whitelist / blacklist decision.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mxp.h"
#include "goupper.h"
#include "lists.h"
#include "vm.h"
#include "dfa_dev.h"

namespace {

__device__ __forceinline__ uint64_t ld8u(const uint8_t* p) { return mxp_ld8(p); }

__device__ __forceinline__ uint64_t tail_mask(uint32_t rem) {
    return rem >= 8 ? ~0ull : ((1ull << (rem * 8u)) - 1ull);
}

__constant__ uint32_t kUpperRows[MXP_UPPER_N][3] = {MXP_UPPER_ROWS};

// probe the entry table for a key given by its hash and length; `same(e)` compares the entry bytes
// (slots: lists.h MXP_LIST_SLOT -- tag, length and pool offset in one word)
template <class Same>
__device__ __forceinline__ bool string_probe(const mxp_list_args& A, uint64_t h, uint32_t n, Same same) {
    const uint32_t tag = (uint32_t)(h >> 44);
    const uint32_t want = n < MXP_LIST_LONG ? n : MXP_LIST_LONG;
    for (uint32_t slot = (uint32_t)h & A.hmask;; slot = (slot + 1) & A.hmask) {
        const uint64_t t = A.htab[slot];
        if (t == MXP_LIST_EMPTY) return false;
        if ((uint32_t)(t >> 44) != tag || ((uint32_t)(t >> 32) & 0xFFFu) != want) continue;
        uint64_t off = (uint64_t)(uint32_t)t * 8u;
        if (want == MXP_LIST_LONG) {  // a long entry: its descriptor
            const uint64_t d = A.ent_desc[(uint32_t)t];
            if ((uint32_t)(d & 0xFFFFFFu) != n) continue;
            off = d >> 24;
        }
        if (same(A.ent_pool + off)) return true;
    }
}

// a case-insensitive symbol with bytes >= 0x80: the key is Go's strings.ToUpper of it (goupper.h),
// streamed twice -- once into the hash, once against a candidate entry's bytes
__device__ __forceinline__ bool string_member_go(const mxp_list_args& A, const uint8_t* s, uint32_t n) {
    MxpUpperStream st(s, n, kUpperRows);
    uint64_t h = 0, w;
    uint32_t len = 0, k;
    while ((k = st.next8(&w)) != 0) {
        h = mxp_hash_step(h, w);
        len += k;
    }
    h = mxp_hash_final(h, len);
    return string_probe(A, h, len, [&](const uint8_t* e) {
        MxpUpperStream again(s, n, kUpperRows);
        uint64_t x;
        uint32_t m;
        for (uint32_t i = 0; (m = again.next8(&x)) != 0; i += 8)
            if (x != (ld8u(e + i) & tail_mask(m))) return false;
        return true;
    });
}

__device__ bool string_member(const mxp_list_args& A, const uint8_t* s, uint32_t n, bool upper) {
    uint64_t h = 0, hi = 0;
    for (uint32_t i = 0; i < n; i += 8) {
        uint64_t w = ld8u(s + i) & tail_mask(n - i);
        hi |= w;
        h = mxp_hash_step(h, upper ? mxp_upper8(w) : w);
    }
    // strings.ToUpper's per-rune path (non-ASCII runes, invalid bytes)
    if (upper && (hi & 0x8080808080808080ull)) return string_member_go(A, s, n);
    h = mxp_hash_final(h, n);
    return string_probe(A, h, n, [&](const uint8_t* e) {
        bool eq = true;
        for (uint32_t i = 0; i < n && eq; i += 8) {
            const uint64_t m = tail_mask(n - i);
            uint64_t w = ld8u(s + i) & m;
            if (upper) w = mxp_upper8(w);
            eq = w == (ld8u(e + i) & m);
        }
        return eq;
    });
}

// index of the last interval starting at or below x (or -1)
__device__ __forceinline__ int find4(const uint32_t* lo, uint32_t n, uint32_t x) {
    int a = 0, b = (int)n - 1, r = -1;
    while (a <= b) {
        const int m = (a + b) >> 1;
        if (lo[m] <= x) {
            r = m;
            a = m + 1;
        } else {
            b = m - 1;
        }
    }
    return r;
}

__device__ __forceinline__ bool le128(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah < bh || (ah == bh && al <= bl);
}

__device__ bool ip_member(const mxp_list_args& A, const uint8_t ip[16]) {
    if (mxpnet::is_v4(ip)) {
        const uint32_t x = (uint32_t)ip[12] << 24 | (uint32_t)ip[13] << 16 | (uint32_t)ip[14] << 8 | ip[15];
        const int k = find4(A.v4lo, A.n4, x);
        return k >= 0 && x <= A.v4hi[k];
    }
    uint64_t xh = 0, xl = 0;
    for (int i = 0; i < 8; i++) xh = xh << 8 | ip[i];
    for (int i = 8; i < 16; i++) xl = xl << 8 | ip[i];
    int a = 0, b = (int)A.n6 - 1, r = -1;
    while (a <= b) {
        const int m = (a + b) >> 1;
        if (le128(A.v6lo[2 * m], A.v6lo[2 * m + 1], xh, xl)) {
            r = m;
            a = m + 1;
        } else {
            b = m - 1;
        }
    }
    return r >= 0 && le128(xh, xl, A.v6hi[2 * r], A.v6hi[2 * r + 1]);
}

// the last IPv4 interval starting at or below x, from the /16 directory: the intervals starting in
// x's /16 block, else the one before them (kargs.v4dir; one load, then a search of the block's few)
__device__ __forceinline__ int find4_dir(const mxp_list_args& A, uint32_t x) {
    const uint32_t k = x >> 16;
    const int a0 = (int)A.v4dir[k], a1 = (int)A.v4dir[k + 1u];
    int a = a0, b = a1 - 1, r = a0 - 1;
    while (a <= b) {
        const int m = (a + b) >> 1;
        if (A.v4lo[m] <= x) {
            r = m;
            a = m + 1;
        } else {
            b = m - 1;
        }
    }
    return r;
}

// bytes [8i, 8i + 8) of a symbol at any address, from aligned words q[] of its window
__device__ __forceinline__ uint64_t funnel8(uint64_t lo, uint64_t hi, uint32_t sh) {
    return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
}

// parseIPv4 (ip.go; leading zeros allowed in Go 1.9) of a dotted quad of at most 15 bytes held in
// registers: two 8-byte words from one three-load window, every byte position unrolled (no
// dependent byte loads).  *x = the address; false when it is no IPv4 literal.
__device__ __forceinline__ bool parse_v4_reg(const uint8_t* s, uint32_t n, uint32_t* x) {
    const uintptr_t a = (uintptr_t)s;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint32_t span = sh / 8u + n;  // bytes of the window the symbol reaches into
    const uint64_t q0 = q[0], q1 = span > 8u ? q[1] : 0ull, q2 = span > 16u ? q[2] : 0ull;
    const uint64_t w0 = funnel8(q0, q1, sh), w1 = funnel8(q1, q2, sh);
    uint32_t acc = 0, ip = 0, ndig = 0, ngrp = 0;
    bool ok = true;
#pragma unroll
    for (uint32_t i = 0; i < 15u; i++) {
        if (i < n) {
            const uint32_t c = (uint32_t)((i < 8u ? w0 >> (8u * i) : w1 >> (8u * (i - 8u))) & 0xFFu);
            if (c == '.') {
                ok = ok && ndig > 0u && ngrp < 3u;
                ip = ip << 8 | acc;
                acc = 0;
                ndig = 0;
                ngrp++;
            } else {
                const uint32_t d = c - '0';
                acc = acc * 10u + d;
                ok = ok && d < 10u && acc <= 255u;
                ndig++;
            }
        }
    }
    *x = ip << 8 | acc;
    return ok && ngrp == 3u && ndig > 0u;
}

// string / case-insensitive membership of a symbol of at most 64 bytes: its words loaded once (one
// window of independent loads), hashed and compared from registers; the candidate entry's words
// loaded together.  false in *done when the symbol needs the general path (longer, or bytes >= 0x80
// in a case-insensitive list).
__device__ __forceinline__ bool string_member_reg(const mxp_list_args& A, const uint8_t* s, uint32_t n, bool upper,
                                                  bool* done) {
    *done = false;
    if (n > 64u) return false;
    const uintptr_t a = (uintptr_t)s;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint32_t nw = (n + 7u) / 8u;
    uint64_t raw[9];
#pragma unroll
    for (uint32_t i = 0; i < 9u; i++) raw[i] = i <= nw ? q[i] : 0ull;
    uint64_t w[8];
    uint64_t h = 0, hi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8u; i++) {
        uint64_t x = funnel8(raw[i], raw[i + 1], sh) & tail_mask(i * 8u < n ? n - i * 8u : 0u);
        hi |= x;
        if (upper) x = mxp_upper8(x);
        w[i] = x;
        if (i < nw) h = mxp_hash_step(h, x);
    }
    if (upper && (hi & 0x8080808080808080ull)) return false;  // strings.ToUpper's per-rune path
    *done = true;
    h = mxp_hash_final(h, n);
    return string_probe(A, h, n, [&](const uint8_t* e) {
        uint64_t diff = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8u; i++)
            if (i < nw) diff |= (ld8u(e + 8u * i) & tail_mask(n - i * 8u)) ^ w[i];
        return diff == 0ull;
    });
}

// The symbol of lookup q: a blob entry, or (fused listentry) the Eval result of one rule.  Returns
// false with codes[q] written when the lookup is settled before the membership test.
__device__ __forceinline__ bool list_symbol(const mxp_list_args& A, uint32_t q, const uint8_t** sp, uint32_t* np) {
    if (A.vals) {
        // listentry ProcessCheck (template.gen.go:2170-2183): Value = mapper.Eval(param.Value).(string)
        if (A.err_word[q] & A.err_bit) {
            A.codes[q] = MXP_LISTENTRY_EVAL_ERROR;
            return false;
        }
        uint64_t id = A.vals[(uint64_t)q * A.vstride];
        if (A.viface) {
            if (MXP_FH_KIND(id) != MXP_STRING) {
                A.codes[q] = MXP_LISTENTRY_NOT_STRING;
                return false;
            }
            id = MXP_FH_ID(id);
        }
        const bool g = id < A.n_gstr;
        const uint64_t d = g ? A.gstr_off[id] : A.bstr_off[id - A.n_gstr];
        *sp = (g ? A.gstr : A.bstr) + (d >> 24);
        *np = (uint32_t)(d & 0xFFFFFFu);
    } else {
        const uint64_t o0 = A.sym_off[q], o1 = A.sym_off[q + 1];
        *sp = A.sym + o0;
        *np = (uint32_t)(o1 - o0);
    }
    return true;
}

__device__ __forceinline__ void list_decide(const mxp_list_args& A, uint32_t q, bool found) {
    A.codes[q] = A.blacklist ? (found ? MXP_RPC_PERMISSION_DENIED : MXP_RPC_OK)
                             : (found ? MXP_RPC_OK : MXP_RPC_NOT_FOUND);
}

}  // namespace

// kNfa: the list holds NFA parts (patterns whose own DFA is over budget): only the *_nfa
// instantiations carry the NFA walk (and the wide walk's private memory)
template <bool kNfa>
__device__ __forceinline__ bool rx_part(const mxp_list_args& A, uint32_t k, const uint8_t* s, uint32_t n) {
    if constexpr (kNfa)
        return mxp_rx_run(A.rx, k, s, n);
    else
        return mxp_dfa_run(A.rx, k, s, n);
}

template <bool kNfa>
__device__ __forceinline__ void list_body(const mxp_list_args& A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= A.n) return;
    const uint8_t* s;
    uint32_t n;
    if (!list_symbol(A, q, &s, &n)) return;
    bool found;
    if (A.type == MXP_LIST_IP_ADDRESSES) {
        uint8_t ip[16];
        if (!mxpnet::parse_ip(s, n, ip)) {
            A.codes[q] = MXP_RPC_INVALID_ARGUMENT;
            return;
        }
        found = ip_member(A, ip);
    } else if (A.type == MXP_LIST_REGEX) {
        found = false;  // regexList.checkList: any pattern matches (any part's automaton)
        for (uint32_t k = 0; k < A.rx_n && !found; k++) found = rx_part<kNfa>(A, k, s, n);
    } else {
        found = string_member(A, s, n, A.type == MXP_LIST_CASE_INSENSITIVE_STRINGS);
    }
    list_decide(A, q, found);
}
// IP lists with the address families in waves of their own.  net.ParseIP decides the family by the
// symbol's first '.' or ':' (ip.go ParseIP); with one lookup per lane, a wave holding both families
// ran the IPv4 parse and the IPv6 parse plus its 128-bit search one after the other, and with a
// tenth of the lookups IPv6 nearly every wave held both.  Here each lane finds its symbol's family
// in its first 8 bytes, the workgroup's lanes are regrouped in LDS (IPv4 from the front, the rest
// from the back, one LDS atomic per wave), and each lane then checks the symbol its new slot names:
// all but at most one wave of a workgroup run one family's path.
__device__ __forceinline__ uint64_t byte_eq_mask(uint64_t w, uint32_t c) {
    const uint64_t x = w ^ (0x0101010101010101ull * c);
    return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;  // high bit of each byte == c (first one exact)
}

extern "C" __global__ __launch_bounds__(256) void mxp_list_ip_kernel(mxp_list_args A) {
    __shared__ uint32_t order[256];
    __shared__ uint32_t cnt[2];  // IPv4 lanes taken from the front, the others from the back
    const uint32_t t = threadIdx.x, lane = t & 63u;
    const uint32_t q = blockIdx.x * 256u + t;
    if (t < 2) cnt[t] = 0;
    const uint8_t* s = nullptr;
    uint32_t n = 0;
    int fam = 2;  // 0 IPv4, 1 IPv6 or other, 2 settled (no lookup)
    if (q < A.n && list_symbol(A, q, &s, &n)) {
        const uint64_t w = n ? mxp_ld8(s) & tail_mask(n) : 0ull;
        const uint64_t dot = byte_eq_mask(w, '.'), col = byte_eq_mask(w, ':');
        fam = (dot && (!col || __builtin_ctzll(dot) < __builtin_ctzll(col))) ? 0 : 1;
    }
    __syncthreads();
    const uint64_t b4 = __ballot(fam == 0), b6 = __ballot(fam == 1);
    const uint32_t below = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)((fam == 0 ? b4 : b6) >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)(fam == 0 ? b4 : b6), 0u));
    uint32_t base4 = 0, base6 = 0;
    if (lane == 0) {
        base4 = b4 ? atomicAdd(&cnt[0], (uint32_t)__popcll(b4)) : 0u;
        base6 = b6 ? atomicAdd(&cnt[1], (uint32_t)__popcll(b6)) : 0u;
    }
    base4 = __shfl(base4, 0, 64);
    base6 = __shfl(base6, 0, 64);
    if (fam == 0) order[base4 + below] = t;
    if (fam == 1) order[255u - (base6 + below)] = t;
    __syncthreads();
    const uint32_t c4 = cnt[0], c6 = cnt[1];
    if (t >= c4 && t < 256u - c6) return;  // (settled lanes' slots)
    const uint32_t src = order[t];
    const uint32_t qq = blockIdx.x * 256u + src;
    if (!list_symbol(A, qq, &s, &n)) return;
    uint8_t ip[16];
    bool found;
    if (t < c4) {  // the first separator is '.': parseIPv4
        uint32_t x;
        bool ok;
        if (n <= 15u && (A.opt & MXP_LIST_OPT_V4REG)) {
            ok = parse_v4_reg(s, n, &x);
        } else {
            ok = mxpnet::parse_v4(s, n, ip);
            x = (uint32_t)ip[12] << 24 | (uint32_t)ip[13] << 16 | (uint32_t)ip[14] << 8 | ip[15];
        }
        if (!ok) {
            A.codes[qq] = MXP_RPC_INVALID_ARGUMENT;
            return;
        }
        const int k = (A.opt & MXP_LIST_OPT_V4DIR) ? find4_dir(A, x) : find4(A.v4lo, A.n4, x);
        found = k >= 0 && x <= A.v4hi[k];
    } else {
        if (!mxpnet::parse_ip(s, n, ip)) {
            A.codes[qq] = MXP_RPC_INVALID_ARGUMENT;
            return;
        }
        found = ip_member(A, ip);
    }
    list_decide(A, qq, found);
}

// string and case-insensitive lists alone (the register fast path; no IP or automaton code, so the
// kernel's register budget is the string path's)
extern "C" __global__ __launch_bounds__(256) void mxp_list_str_kernel(mxp_list_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= A.n) return;
    const uint8_t* s;
    uint32_t n;
    if (!list_symbol(A, q, &s, &n)) return;
    const bool upper = A.type == MXP_LIST_CASE_INSENSITIVE_STRINGS;
    bool done = false, found = false;
    if (A.opt & MXP_LIST_OPT_STRREG) found = string_member_reg(A, s, n, upper, &done);
    if (!done) found = string_member(A, s, n, upper);
    list_decide(A, q, found);
}

extern "C" __global__ __launch_bounds__(256) void mxp_list_kernel(mxp_list_args A) { list_body<false>(A); }
extern "C" __global__ __launch_bounds__(256) void mxp_list_nfa_kernel(mxp_list_args A) { list_body<true>(A); }

// REGEX lists with LDS-staged automata: each 1024-thread workgroup copies the hot rows of the parts'
// DFAs (the first lds_states[k] states in BFS order from the start: the shallow levels every lookup
// steps through) and their ASCII class maps into LDS once, then strides over the lookups; a lane
// steps from LDS while its state is staged and from global memory below that.  Two workgroups fill
// a CU's 32 wave slots while sharing one staged copy per 16 waves.
template <bool kNfa>
__device__ __forceinline__ void list_rx_body(const mxp_list_args& A) {
    __shared__ uint32_t TL[MXP_LDS_DFA_WORDS];
    __shared__ uint16_t AL[MXP_LDS_DFA_PARTS * 128u];
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = 0; k < A.lds_nparts; k++) {
        const mxp_dfa_hdr H = A.rx.hdr[k];
        const uint32_t ent = A.lds_plan[k] * H.ncls, base = A.lds_plan[MXP_LDS_DFA_PARTS + k];
        const uint32_t words = H.kind == MXP_RX_DFA16 ? (ent + 1u) / 2u : ent;  // (u16 rows: two a word)
        const uint32_t* src = A.rx.trans + H.trans;
        for (uint32_t i = tid; i < words; i += MXP_LIST_RX_THREADS) TL[base + i] = src[i];
        if (tid < 128u) AL[k * 128u + tid] = A.rx.ascii[H.ascii + tid];
    }
    __syncthreads();
    for (uint32_t q = blockIdx.x * MXP_LIST_RX_THREADS + tid; q < A.n; q += gridDim.x * MXP_LIST_RX_THREADS) {
        const uint8_t* s;
        uint32_t n;
        if (!list_symbol(A, q, &s, &n)) continue;
        bool found = false;  // regexList.checkList: any pattern matches (any part's automaton)
        for (uint32_t k = 0; k < A.rx_n && !found; k++) {
            const uint32_t K = k < A.lds_nparts ? A.lds_plan[k] : 0u;
            if (K) {
                const mxp_dfa_hdr H = A.rx.hdr[k];
                found = mxp_dfa_walk<true>(A.rx, H, TL + A.lds_plan[MXP_LDS_DFA_PARTS + k], AL + k * 128u, K, s, n);
            } else {
                found = rx_part<kNfa>(A, k, s, n);
            }
        }
        list_decide(A, q, found);
    }
}
extern "C" __global__ __launch_bounds__(1024) void mxp_list_rx_kernel(mxp_list_args A) { list_rx_body<false>(A); }
extern "C" __global__ __launch_bounds__(1024) void mxp_list_rx_nfa_kernel(mxp_list_args A) { list_rx_body<true>(A); }

// REGEX lists with literal-prefix dispatch (lists.cpp rxp_build).  Per lookup: the prefix lengths
// worth probing come from the LDS mask of its first three bytes (rxp_lead, staged per workgroup) and
// the short-prefix mask; each is one probe of the prefix table (hash of the symbol's first L bytes,
// kept in registers); a slot names the tail blocks of the patterns with that prefix; a block's header
// and prefix are compared from registers, then the block is copied to the lane's LDS slot and its
// tail automaton stepped from there over the rest of the symbol (one LDS byte per class, one per
// transition).  So a lookup pays ~3 dependent global loads (symbol, slot, block) where the union DFA
// paid one per byte.  Patterns not dispatched stay in the union parts, walked after (from global).
// One lookup through the dispatch: every prefix length its leading bytes allow, every tail with that
// prefix, until one accepts (kLds: each tail stepped from the lane's LDS row).
template <bool kLds>
__device__ __forceinline__ bool rxp_one(const mxp_list_args& A, const uint8_t* s, uint32_t n, uint32_t* row) {
    // the symbol's first 32 bytes (zero past its end): prefix hashes and compares, the walk's bytes
    uint64_t w[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) w[k] = 8u * k < n ? mxp_ld8(s + 8u * k) & tail_mask(n - 8u * k) : 0ull;
    uint32_t lens = A.rxp_short;
    if (n >= 3u) {
        const uint32_t b = (uint32_t)w[0];
        lens |= A.rxp_lead[mxp_rxp_lead(b & 0xFFu, (b >> 8) & 0xFFu, (b >> 16) & 0xFFu)];
    }
    if (n < 32u) lens &= (1u << n) - 1u;  // (prefixes no longer than the symbol)
    bool found = false;
    for (; lens && !found; lens &= lens - 1u) {
        const uint32_t L = (uint32_t)__ffs(lens);  // (bit L - 1: prefix length L)
        uint64_t pre[4], h = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            pre[k] = 8u * k < L ? w[k] & tail_mask(L - 8u * k) : 0ull;
            if (8u * k < L) h = mxp_hash_step(h, pre[k]);
        }
        h = mxp_hash_final(h, L);
        const uint64_t want = (h >> 44) << 44 | (uint64_t)L << 38;
        uint64_t t = 0;
        for (uint32_t slot = (uint32_t)h & A.rxp_mask;; slot = (slot + 1u) & A.rxp_mask) {
            t = A.rxp_tab[slot];
            if (!t || (t & ~0x3FFFFFFFFFull) == want) break;
        }
        if (!t) continue;
        if (A.opt & MXP_LIST_OPT_ABL_PROBE) {  // (ablation: stop at the probe -- results invalid)
            found = true;
            break;
        }
        const uint32_t count = (uint32_t)(t >> 32) & 0x3Fu;
        uint32_t unit = (uint32_t)t;
        for (uint32_t c = 0; c < count && !found; c++) {
            const uint4* blk = (const uint4*)A.rxp_blk + unit;
            const uint4 h0 = blk[0], h1 = blk[1];

            const uint32_t S = h0.x & 0xFFu, C = (h0.x >> 8) & 0xFFu, nq = h0.x >> 24;
            unit += nq;
            // the block's prefix (bytes 4 .. 32, zero padded) against the symbol's first L bytes
            const bool same = pre[0] == ((uint64_t)h0.y | (uint64_t)h0.z << 32) &&
                              pre[1] == ((uint64_t)h0.w | (uint64_t)h1.x << 32) &&
                              pre[2] == ((uint64_t)h1.y | (uint64_t)h1.z << 32) && pre[3] == (uint64_t)h1.w;
            if (!same) continue;
            if (S == 0u || (A.opt & MXP_LIST_OPT_ABL_HDR)) {  // the prefix alone decides (or the ablation stops here)
                found = true;
                break;
            }
            const uint8_t* B = (const uint8_t*)blk;
            if (kLds && nq <= MXP_RXP_BLOCK / 16u) {
                // class nibbles and transitions into the lane's row: every load issued before the
                // first store (one round trip, not one per 16 bytes)
                uint4 v[MXP_RXP_BLOCK / 16u - 2u];
#pragma unroll
                for (uint32_t k = 2; k < MXP_RXP_BLOCK / 16u; k++)
                    if (k < nq) v[k - 2u] = blk[k];
#pragma unroll
                for (uint32_t k = 2; k < MXP_RXP_BLOCK / 16u; k++)
                    if (k < nq) {
                        row[4u * k] = v[k - 2u].x;
                        row[4u * k + 1u] = v[k - 2u].y;
                        row[4u * k + 2u] = v[k - 2u].z;
                        row[4u * k + 3u] = v[k - 2u].w;
                    }
                B = (const uint8_t*)row;
            }
            // the classes of the tail's first 16 bytes first, as nibbles: their loads do not depend
            // on the state, so they are all in flight together and the walk below pays one
            // dependent load (the transition) per byte
            const uint32_t wi = L >> 3, sh = (L & 7u) * 8u;
            auto wsel = [&](uint32_t k) { return k == 0u ? w[0] : k == 1u ? w[1] : k == 2u ? w[2] : k == 3u ? w[3] : 0ull; };
            const uint64_t a0 = wsel(wi), a1 = wsel(wi + 1u), a2 = wsel(wi + 2u);
            const uint64_t t0 = sh ? (a0 >> sh) | (a1 << (64u - sh)) : a0;
            const uint64_t t1 = sh ? (a1 >> sh) | (a2 << (64u - sh)) : a1;
            uint64_t cl = 0;
#pragma unroll
            for (uint32_t j = 0; j < 16u; j++) {
                if (L + j >= n || L + j >= 32u) break;
                const uint32_t b = (uint32_t)((j < 8u ? t0 : t1) >> ((j & 7u) * 8u)) & 0xFFu;
                const uint64_t c = b >= 0x80u ? C - 2u : (B[32u + (b >> 1)] >> ((b & 1u) * 4u)) & 0xFu;
                cl |= c << (4u * j);
            }
            const uint8_t* T = B + MXP_RXP_TRANS;
            uint32_t st = 0;
            for (uint32_t i = L; i < n && st < S; i++) {
                uint32_t cls;
                if (i < L + 16u && i < 32u) {
                    cls = (uint32_t)(cl >> (4u * (i - L))) & 0xFu;
                } else {
                    const uint32_t b = s[i];
                    cls = b >= 0x80u ? C - 2u : (B[32u + (b >> 1)] >> ((b & 1u) * 4u)) & 0xFu;
                }
                st = T[st * C + cls];
            }
            if (st < S) st = T[st * C + C - 1u];  // END of text
            found = st == MXP_RXP_ACC;
        }
    }
    return found;
}

template <bool kNfa, bool kLds>
__device__ __forceinline__ void list_rxp_body(const mxp_list_args& A) {
    // kLds: the candidate's block copied into the lane's LDS row (MXP_RXP_ROW words; odd: the lanes'
    // words fall in different banks) and stepped there; else stepped from global memory, where the
    // tail blocks (a few MB) stay L2-resident and the kernel keeps its waves (no LDS)
    __shared__ uint32_t SLOT[kLds ? MXP_RXP_THREADS * MXP_RXP_ROW : 1];
    const uint32_t nthr = kLds ? MXP_RXP_THREADS : 256u;
    const uint32_t tid = threadIdx.x;
    uint32_t* const row = SLOT + (kLds ? tid * MXP_RXP_ROW : 0u);
    for (uint32_t q = blockIdx.x * nthr + tid; q < A.n; q += gridDim.x * nthr) {
        const uint8_t* s;
        uint32_t n;
        if (!list_symbol(A, q, &s, &n)) continue;
        bool found = rxp_one<kLds>(A, s, n, row);
        for (uint32_t k = 0; k < A.rx_n && !found; k++) found = rx_part<kNfa>(A, k, s, n);
        list_decide(A, q, found);
    }
}
extern "C" __global__ __launch_bounds__(MXP_RXP_THREADS) void mxp_list_rxp_lds_kernel(mxp_list_args A) {
    list_rxp_body<false, true>(A);
}
extern "C" __global__ __launch_bounds__(256) void mxp_list_rxp_kernel(mxp_list_args A) {
    list_rxp_body<false, false>(A);
}
extern "C" __global__ __launch_bounds__(256) void mxp_list_rxp_nfa_kernel(mxp_list_args A) {
    list_rxp_body<true, false>(A);
}

extern "C" hipError_t mxp_launch_list(const mxp_list_args* a, hipStream_t s) {
    if (a->type == MXP_LIST_REGEX && a->rxp_mask) {
        if ((a->opt & MXP_LIST_OPT_RXP_LDS) && !a->rx_nfa) {
            // persistent: five 128-thread workgroups per CU (their LDS: 5 x 31 KB of the 160 KB)
            const uint32_t need = (a->n + MXP_RXP_THREADS - 1u) / MXP_RXP_THREADS;
            const uint32_t grid = need < 1280u ? need : 1280u;
            hipLaunchKernelGGL(mxp_list_rxp_lds_kernel, dim3(grid), dim3(MXP_RXP_THREADS), 0, s, *a);
            return hipGetLastError();
        }
        const uint32_t need = (a->n + 255u) / 256u;
        const uint32_t grid = need < 2048u ? need : 2048u;
        hipLaunchKernelGGL(a->rx_nfa ? mxp_list_rxp_nfa_kernel : mxp_list_rxp_kernel, dim3(grid), dim3(256), 0, s, *a);
        return hipGetLastError();
    }
    if (a->type == MXP_LIST_REGEX && a->lds_nparts) {
        // enough workgroups for 2 per CU (256 CUs), fewer for small batches
        const uint32_t need = (a->n + MXP_LIST_RX_THREADS - 1u) / MXP_LIST_RX_THREADS;
        const uint32_t grid = need < 512u ? need : 512u;
        hipLaunchKernelGGL(a->rx_nfa ? mxp_list_rx_nfa_kernel : mxp_list_rx_kernel, dim3(grid), dim3(MXP_LIST_RX_THREADS),
                           0, s, *a);
        return hipGetLastError();
    }
    if (a->type == MXP_LIST_STRINGS || a->type == MXP_LIST_CASE_INSENSITIVE_STRINGS) {
        hipLaunchKernelGGL(mxp_list_str_kernel, dim3((a->n + 255u) / 256u), dim3(256), 0, s, *a);
        return hipGetLastError();
    }
    if (a->type == MXP_LIST_IP_ADDRESSES && a->ip_split) {
        hipLaunchKernelGGL(mxp_list_ip_kernel, dim3((a->n + 255u) / 256u), dim3(256), 0, s, *a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(a->rx_nfa ? mxp_list_nfa_kernel : mxp_list_kernel, dim3((a->n + 255u) / 256u), dim3(256), 0, s, *a);
    return hipGetLastError();
}
