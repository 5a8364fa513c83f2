// dfa_dev.h -- device layout of compiled regex DFAs (regex.h) and the gfx950 stepping loop, shared
// by the predicate VM (kernels.hip: `matches`) and the list kernel (lists.hip: REGEX lists).
#pragma once

#include <stdint.h>

typedef struct mxp_dfa_hdr {
    uint32_t ncls;      // rune classes + 1 (last column = END of text)
    uint32_t start;
    uint32_t trans;     // first transition (index into mxp_dfa_set.trans)
    uint32_t ascii;     // first ASCII class entry (128 per DFA, index into mxp_dfa_set.ascii)
    uint32_t hi;        // first non-ASCII range (index into hilo / hicls)
    uint32_t hi_n;
    uint32_t skip;      // subject bytes already consumed into `start` (a rule's literal prefix, verified
                        // by the prefix index); MXP_DFA_DECIDED: the prefix alone decides a match
    uint32_t kind;      // MXP_RX_DFA, or MXP_RX_NFA: `trans` is the (8-byte aligned) NFA image
} mxp_dfa_hdr;
#define MXP_DFA_DECIDED 0xFFFFFFFFu
#define MXP_RX_DFA 0u
#define MXP_RX_NFA 1u
// a DFA of at most 65533 states with u16 transitions (regex-list parts, lists.cpp): `trans` indexes the
// u32 array where its u16 rows start; 0xFFFF accept, 0xFFFE reject
#define MXP_RX_DFA16 2u

// Bit-parallel NFA image (u64 words from S.trans + H.trans), for patterns whose DFA is over budget:
//   [0]            m | W << 16 | nvar << 24   (m rune instructions; bit m of a set = MATCH; W words)
//   [1 .. 8]       var_of[64]: assertion-flag value -> closure variant (only flags the program tests)
//   ACC            [ncls - 1][W]   rune instructions that accept each rune class
//   CL             [m + 1][nvar][W] epsilon closure (under the variant's flags) of each rune
//                  instruction's successor; row m = the start threads (re-injected every step)
#define MXP_NFA_HDR_WORDS 9u
#define MXP_NFA_MAX_WORDS 4u    // thread sets of up to 255 rune instructions: registers
#define MXP_NFA_WIDE_WORDS 16u  // up to 1023 (regex.h kNfaMaxPos): private memory, see mxp_nfa_run_wide

typedef struct mxp_dfa_set {
    const mxp_dfa_hdr* hdr;
    const uint32_t* trans;   // next state | 0xFFFFFFFF accept | 0xFFFFFFFE reject
    const uint16_t* ascii;
    const uint32_t* hilo;    // ascending non-ASCII range starts
    const uint16_t* hicls;
    // NFAs wider than MXP_NFA_WIDE_WORDS (mxp_nfa_run_global): thread sets in global memory, one slot
    // of 2 * nfa_wmax * 64 words per wavefront walking one, claimed in nfa_busy[nfa_nslots]
    uint64_t* nfa_scratch;
    uint32_t* nfa_busy;
    uint32_t nfa_nslots;
    uint32_t nfa_wmax;
} mxp_dfa_set;
// bytes of the global thread-set scratch for NFAs of up to wmax words (0: none needed)
#define MXP_NFA_SLOT_WORDS(wmax) (2ull * (wmax) * 64ull)

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>

// 8 bytes at any address of a blob with >= 16 bytes of slack (two aligned loads + funnel shift)
__device__ __forceinline__ uint64_t mxp_ld8(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7) * 8u;
    const uint64_t lo = q[0];
    return sh == 0 ? lo : (lo >> sh) | (q[1] << (64u - sh));
}

// one rune at s[i] (lead byte c0 >= 0x80) as Go's inputString decodes it: invalid -> U+FFFD, width 1
__device__ __forceinline__ uint32_t mxp_decode_hi(const uint8_t* s, uint32_t i, uint32_t n, uint32_t c0,
                                                  uint32_t* width) {
    const uint64_t w = mxp_ld8(s + i);  // bytes i .. i+7 (only those < n are used)
    const uint32_t left = n - i;
    const uint32_t b1 = (uint32_t)(w >> 8) & 0xFF, b2 = (uint32_t)(w >> 16) & 0xFF, b3 = (uint32_t)(w >> 24) & 0xFF;
    uint32_t r = 0xFFFD;
    *width = 1;
    if (c0 >= 0xC2 && c0 <= 0xDF) {
        if (left >= 2 && b1 >= 0x80 && b1 <= 0xBF) {
            r = ((c0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
            *width = 2;
        }
    } else if (c0 >= 0xE0 && c0 <= 0xEF) {
        const uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
        if (left >= 3 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF) {
            r = ((c0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
            *width = 3;
        }
    } else if (c0 >= 0xF0 && c0 <= 0xF4) {
        const uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
        if (left >= 4 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF && b3 >= 0x80 && b3 <= 0xBF) {
            r = ((c0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
            *width = 4;
        }
    }
    return r;
}

// class of a non-ASCII rune: the last range whose start <= r
__device__ __forceinline__ uint32_t mxp_hi_class(const mxp_dfa_set& S, const mxp_dfa_hdr& H, uint32_t r) {
    const uint32_t* lo = S.hilo + H.hi;
    int a = 0, b = (int)H.hi_n - 1, k = 0;
    while (a <= b) {
        const int m = (a + b) >> 1;
        if (lo[m] <= r) {
            k = m;
            a = m + 1;
        } else {
            b = m - 1;
        }
    }
    return S.hicls[H.hi + k];
}

__device__ __forceinline__ bool mxp_rx_word(uint32_t r) {
    return (r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_';
}

// The bit-parallel NFA walk (only over-budget patterns take it; the VM kernels that can meet one are
// separate instantiations, so the DFA-only kernels keep their register budgets).  Per position: the closure of the pending threads
// plus a fresh start thread under the position's assertion flags (what the DFA folds into its
// states); MATCH in the closure -> true; else the threads whose rune instruction accepts the class.
// Programs with more than 255 rune instructions (W > 4): the same walk with the thread sets in
// per-lane arrays indexed at run time -- private (scratch) memory, 256 bytes a lane, which only the
// NFA kernel instantiations carry.  Only patterns whose DFA is over budget AND whose program is that
// wide take it.
__device__ __forceinline__ bool mxp_nfa_run_wide(const mxp_dfa_set& S, const mxp_dfa_hdr& H, const uint8_t* s,
                                                 uint32_t n) {
    const uint64_t* N = (const uint64_t*)(S.trans + H.trans);
    const uint64_t h0 = N[0];
    const uint32_t m = (uint32_t)(h0 & 0xFFFF), W = (uint32_t)(h0 >> 16) & 0xFF, nvar = (uint32_t)(h0 >> 24) & 0xFFFF;
    const uint8_t* var_of = (const uint8_t*)(N + 1);
    const uint64_t* ACC = N + MXP_NFA_HDR_WORDS;
    const uint64_t* CL = ACC + (uint64_t)(H.ncls - 1) * W;
    const uint64_t* CLS = CL + (uint64_t)m * nvar * W;
    const uint16_t* asc = S.ascii + H.ascii;
    // (volatile: kept in private memory -- promoted to registers they would cost every NFA kernel
    // instantiation 64 VGPRs for a path almost no rule set takes)
    volatile uint64_t U[MXP_NFA_WIDE_WORDS], C[MXP_NFA_WIDE_WORDS];
    for (uint32_t w = 0; w < W; w++) U[w] = 0;
    bool begin = true, prev_nl = false, prev_word = false;
    uint32_t i = 0;
    for (;;) {
        const bool end = i >= n;
        uint32_t r = 0, width = 1, cls = 0;
        if (!end) {
            const uint32_t c0 = s[i];
            if (c0 < 0x80) {
                r = c0;
                cls = asc[c0];
            } else {
                r = mxp_decode_hi(s, i, n, c0, &width);
                cls = mxp_hi_class(S, H, r);
            }
        }
        uint32_t f = 0;
        if (begin) f |= 4u | 1u;
        if (prev_nl) f |= 1u;
        if (end) f |= 8u | 2u;
        if (!end && r == '\n') f |= 2u;
        f |= (prev_word != (!end && mxp_rx_word(r))) ? 16u : 32u;
        const uint32_t v = var_of[f];
        for (uint32_t w = 0; w < W; w++) C[w] = CLS[(uint64_t)v * W + w];
        for (uint32_t w = 0; w < W; w++) {
            uint64_t bits = U[w];
            while (bits) {
                const uint32_t j = w * 64u + (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                const uint64_t* q = CL + ((uint64_t)j * nvar + v) * W;
                for (uint32_t x = 0; x < W; x++) C[x] |= q[x];
            }
        }
        if ((C[m >> 6] >> (m & 63)) & 1u) return true;
        if (end) return false;
        const uint64_t* a = ACC + (uint64_t)cls * W;
        for (uint32_t w = 0; w < W; w++) U[w] = C[w] & a[w];
        begin = false;
        prev_nl = r == '\n';
        prev_word = mxp_rx_word(r);
        i += width;
    }
}

// Programs wider than 1023 rune instructions (W > MXP_NFA_WIDE_WORDS): the same walk with the thread
// sets in global memory.  The lanes here claim one slot of the engine's (or list's) scratch for their
// wavefront -- the first active lane takes a free slot by compare-and-swap and hands it to the
// others -- lay U and C out word-major with the lane minor (coalesced), and free the slot when all of
// them are done.  Holders never wait on anything, so a wave that finds every slot taken only spins
// until one is freed.
__device__ __noinline__ bool mxp_nfa_run_global(const mxp_dfa_set& S, const mxp_dfa_hdr& H, const uint8_t* s,
                                                uint32_t n) {
    const uint64_t* N = (const uint64_t*)(S.trans + H.trans);
    const uint64_t h0 = N[0];
    const uint32_t m = (uint32_t)(h0 & 0xFFFF), W = (uint32_t)(h0 >> 16) & 0xFF, nvar = (uint32_t)(h0 >> 24) & 0xFFFF;
    const uint8_t* var_of = (const uint8_t*)(N + 1);
    const uint64_t* ACC = N + MXP_NFA_HDR_WORDS;
    const uint64_t* CL = ACC + (uint64_t)(H.ncls - 1) * W;
    const uint64_t* CLS = CL + (uint64_t)m * nvar * W;
    const uint16_t* asc = S.ascii + H.ascii;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t act = __ballot(1);
    const uint32_t leader = (uint32_t)__builtin_ctzll(act);
    uint32_t slot = 0;
    if (lane == leader) {
        uint32_t i = (blockIdx.x * 97u + (threadIdx.x >> 6) * 31u) % S.nfa_nslots;
        while (atomicCAS(S.nfa_busy + i, 0u, 1u) != 0u) i = i + 1u == S.nfa_nslots ? 0u : i + 1u;
        slot = i;
    }
    slot = (uint32_t)__shfl((int)slot, (int)leader, 64);
    uint64_t* U = S.nfa_scratch + (uint64_t)slot * MXP_NFA_SLOT_WORDS(S.nfa_wmax) + lane;
    uint64_t* C = U + (uint64_t)S.nfa_wmax * 64u;
    for (uint32_t w = 0; w < W; w++) U[w * 64u] = 0;
    bool result = false, begin = true, prev_nl = false, prev_word = false;
    uint32_t i = 0;
    for (;;) {
        const bool end = i >= n;
        uint32_t r = 0, width = 1, cls = 0;
        if (!end) {
            const uint32_t c0 = s[i];
            if (c0 < 0x80) {
                r = c0;
                cls = asc[c0];
            } else {
                r = mxp_decode_hi(s, i, n, c0, &width);
                cls = mxp_hi_class(S, H, r);
            }
        }
        uint32_t f = 0;
        if (begin) f |= 4u | 1u;
        if (prev_nl) f |= 1u;
        if (end) f |= 8u | 2u;
        if (!end && r == '\n') f |= 2u;
        f |= (prev_word != (!end && mxp_rx_word(r))) ? 16u : 32u;
        const uint32_t v = var_of[f];
        for (uint32_t w = 0; w < W; w++) C[w * 64u] = CLS[(uint64_t)v * W + w];
        for (uint32_t w = 0; w < W; w++) {
            uint64_t bits = U[w * 64u];
            while (bits) {
                const uint32_t j = w * 64u + (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                const uint64_t* q = CL + ((uint64_t)j * nvar + v) * W;
                for (uint32_t x = 0; x < W; x++) C[x * 64u] |= q[x];
            }
        }
        if ((C[(m >> 6) * 64u] >> (m & 63)) & 1u) {
            result = true;
            break;
        }
        if (end) break;
        const uint64_t* a = ACC + (uint64_t)cls * W;
        for (uint32_t w = 0; w < W; w++) U[w * 64u] = C[w * 64u] & a[w];
        begin = false;
        prev_nl = r == '\n';
        prev_word = mxp_rx_word(r);
        i += width;
    }
    // (every lane that came in is here again) the slot goes back
    __threadfence();
    if (lane == leader) atomicExch(S.nfa_busy + slot, 0u);
    return result;
}

__device__ __forceinline__ bool mxp_nfa_run(const mxp_dfa_set& S, const mxp_dfa_hdr& H, const uint8_t* s, uint32_t n) {
    const uint64_t* N = (const uint64_t*)(S.trans + H.trans);
    const uint64_t h0 = N[0];
    const uint32_t m = (uint32_t)(h0 & 0xFFFF), W = (uint32_t)(h0 >> 16) & 0xFF, nvar = (uint32_t)(h0 >> 24) & 0xFFFF;
    if (W > MXP_NFA_WIDE_WORDS) return mxp_nfa_run_global(S, H, s, n);
    if (W > MXP_NFA_MAX_WORDS) return mxp_nfa_run_wide(S, H, s, n);
    const uint8_t* var_of = (const uint8_t*)(N + 1);
    const uint64_t* ACC = N + MXP_NFA_HDR_WORDS;
    const uint64_t* CL = ACC + (uint64_t)(H.ncls - 1) * W;
    const uint64_t* CLS = CL + (uint64_t)m * nvar * W;
    const uint16_t* asc = S.ascii + H.ascii;
    uint64_t U[MXP_NFA_MAX_WORDS] = {0, 0, 0, 0};
    bool begin = true, prev_nl = false, prev_word = false;
    uint32_t i = 0;
    for (;;) {
        const bool end = i >= n;
        uint32_t r = 0, width = 1, cls = 0;
        if (!end) {
            const uint32_t c0 = s[i];
            if (c0 < 0x80) {
                r = c0;
                cls = asc[c0];
            } else {
                r = mxp_decode_hi(s, i, n, c0, &width);
                cls = mxp_hi_class(S, H, r);
            }
        }
        // syntax.EmptyOp flags: BEGIN_LINE 1, END_LINE 2, BEGIN_TEXT 4, END_TEXT 8, WORD_B 16, NO_WORD_B 32
        uint32_t f = 0;
        if (begin) f |= 4u | 1u;
        if (prev_nl) f |= 1u;
        if (end) f |= 8u | 2u;
        if (!end && r == '\n') f |= 2u;
        f |= (prev_word != (!end && mxp_rx_word(r))) ? 16u : 32u;
        const uint32_t v = var_of[f];
        uint64_t C[MXP_NFA_MAX_WORDS];
#pragma unroll
        for (uint32_t w = 0; w < MXP_NFA_MAX_WORDS; w++) C[w] = w < W ? CLS[(uint64_t)v * W + w] : 0;
#pragma unroll
        for (uint32_t w = 0; w < MXP_NFA_MAX_WORDS; w++) {
            uint64_t bits = U[w];
            while (bits) {
                const uint32_t j = w * 64u + (uint32_t)__builtin_ctzll(bits);
                bits &= bits - 1;
                const uint64_t* q = CL + ((uint64_t)j * nvar + v) * W;
#pragma unroll
                for (uint32_t x = 0; x < MXP_NFA_MAX_WORDS; x++)
                    if (x < W) C[x] |= q[x];
            }
        }
        uint64_t mw = 0;
#pragma unroll
        for (uint32_t w = 0; w < MXP_NFA_MAX_WORDS; w++)
            if (w == (m >> 6)) mw = C[w];
        if ((mw >> (m & 63)) & 1u) return true;
        if (end) return false;
        const uint64_t* a = ACC + (uint64_t)cls * W;
#pragma unroll
        for (uint32_t w = 0; w < MXP_NFA_MAX_WORDS; w++) U[w] = w < W ? (C[w] & a[w]) : 0;
        begin = false;
        prev_nl = r == '\n';
        prev_word = mxp_rx_word(r);
        i += width;
    }
}

// regexp.MatchString on one subject: decode runes the way Go's inputString does (utf8 rules; an
// invalid byte is U+FFFD of width 1), map each to its class, step; END column at the end.  A step
// into ACCEPT decides true, a step into REJECT (a state from which no match is reachable, folded at
// build time: regex.cpp fold_dead_states) decides false.
//
// kLds: the first K states' transition rows (TL, K * ncls words) and the ASCII class map (AL) are
// staged in LDS by the caller; states >= K step from global memory.  Subset construction numbers
// states in BFS order from the start, so the staged rows are the shallow, hot part of the DFA.
// (DFA headers only: callers that may meet an NFA header use mxp_rx_run)
// u16 parts (MXP_RX_DFA16): rows of u16 transitions, in LDS too; their reject / accept codes widen to
// the u32 ones.
template <bool kLds>
__device__ __forceinline__ bool mxp_dfa_walk(const mxp_dfa_set& S, const mxp_dfa_hdr& H, const uint32_t* TL,
                                             const uint16_t* AL, uint32_t K, const uint8_t* s, uint32_t n) {
    const uint32_t* T = S.trans + H.trans;
    const bool w16 = H.kind == MXP_RX_DFA16;
    const uint16_t* T16 = (const uint16_t*)T;
    const uint16_t* TL16 = (const uint16_t*)TL;
    auto next = [&](uint64_t at, uint32_t st) -> uint32_t {
        if (w16) {
            const uint32_t v = (kLds && st < K) ? TL16[(uint32_t)at] : T16[at];
            return v >= 0xFFFEu ? v | 0xFFFF0000u : v;
        }
        if constexpr (kLds) return st < K ? TL[(uint32_t)at] : T[at];
        return T[at];
    };
    const uint16_t* asc = kLds ? AL : S.ascii + H.ascii;
    uint32_t st = H.start;
    uint32_t i = H.skip;
    if (i == MXP_DFA_DECIDED) return true;
    // ASCII bytes come out of the aligned 8-byte word that holds them: one subject load per 8 steps
    // (the pools and symbol blobs are readable to the aligned word past their end)
    uintptr_t wa = ((uintptr_t)(s + i)) & ~(uintptr_t)7;
    uint64_t win = *(const uint64_t*)wa;
    while (i < n) {
        const uintptr_t a = (uintptr_t)(s + i);
        if ((a & ~(uintptr_t)7) != wa) {
            wa = a & ~(uintptr_t)7;
            win = *(const uint64_t*)wa;
        }
        const uint32_t c0 = (uint32_t)(win >> ((a & 7u) * 8u)) & 0xFFu;
        uint32_t cls;
        if (c0 < 0x80) {
            cls = asc[c0];
            i++;
        } else {
            const uint64_t w = mxp_ld8(s + i);  // bytes i .. i+7 (only those < n are used)
            const uint32_t left = n - i;
            const uint32_t b1 = (uint32_t)(w >> 8) & 0xFF, b2 = (uint32_t)(w >> 16) & 0xFF, b3 = (uint32_t)(w >> 24) & 0xFF;
            uint32_t r = 0xFFFD, width = 1;
            if (c0 >= 0xC2 && c0 <= 0xDF) {
                if (left >= 2 && b1 >= 0x80 && b1 <= 0xBF) {
                    r = ((c0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
                    width = 2;
                }
            } else if (c0 >= 0xE0 && c0 <= 0xEF) {
                const uint32_t lo = c0 == 0xE0 ? 0xA0 : 0x80, hi = c0 == 0xED ? 0x9F : 0xBF;
                if (left >= 3 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF) {
                    r = ((c0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
                    width = 3;
                }
            } else if (c0 >= 0xF0 && c0 <= 0xF4) {
                const uint32_t lo = c0 == 0xF0 ? 0x90 : 0x80, hi = c0 == 0xF4 ? 0x8F : 0xBF;
                if (left >= 4 && b1 >= lo && b1 <= hi && b2 >= 0x80 && b2 <= 0xBF && b3 >= 0x80 && b3 <= 0xBF) {
                    r = ((c0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
                    width = 4;
                }
            }
            i += width;
            // last range whose start <= r
            const uint32_t* lo = S.hilo + H.hi;
            int a = 0, b = (int)H.hi_n - 1, k = 0;
            while (a <= b) {
                const int m = (a + b) >> 1;
                if (lo[m] <= r) {
                    k = m;
                    a = m + 1;
                } else {
                    b = m - 1;
                }
            }
            cls = S.hicls[H.hi + k];
        }
        st = next((uint64_t)st * H.ncls + cls, st);
        if (st >= 0xFFFFFFFEu) return st == 0xFFFFFFFFu;
    }
    return next((uint64_t)st * H.ncls + H.ncls - 1, st) == 0xFFFFFFFFu;
}

__device__ __forceinline__ bool mxp_dfa_run(const mxp_dfa_set& S, uint32_t dfa, const uint8_t* s, uint32_t n) {
    const mxp_dfa_hdr H = S.hdr[dfa];
    return mxp_dfa_walk<false>(S, H, nullptr, nullptr, 0u, s, n);
}

// a DFA or an NFA header
__device__ __forceinline__ bool mxp_rx_run(const mxp_dfa_set& S, uint32_t dfa, const uint8_t* s, uint32_t n) {
    const mxp_dfa_hdr H = S.hdr[dfa];
    if (H.kind == MXP_RX_NFA) return mxp_nfa_run(S, H, s, n);
    return mxp_dfa_run(S, dfa, s, n);
}

#endif
