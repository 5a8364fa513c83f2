// resolve.hip -- gfx950 kernels of the batched runtime.resolver (resolver.cpp).
//
// Reference: resolver.Resolve / filterActions (mixer/pkg/runtime/resolver.go:110-238).  Per
// request, the rules of the default namespace and then those of the request's own namespace are
// walked in order; a rule counts only if it has an action for the variety and its TCP flag equals
// the request's; an empty match selects it unconditionally; the first predicate error fails the
// whole request (no actions); otherwise every rule whose predicate is true is selected.
//
// Rules of a namespace are contiguous in the engine's rule order (mxp_resolver_set checks), so
// each namespace is a rule range and the walk reads the predicate bitmaps word by word: lane =
// request, one coalesced load per bitmap word, the variety/TCP applicability and empty-match masks
// are per-word constants.  Pass 1 counts selected rules and finds the first error; the host scans
// the counts; pass 2 writes the selected rule ids.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pack_args.h"
#include "resolve_args.h"

namespace {

// bits of word w that fall in the rule range [lo, hi)
__device__ __forceinline__ uint32_t range_bits(uint32_t w, uint32_t lo, uint32_t hi) {
    const uint32_t b0 = w * 32u;
    const uint32_t a = lo > b0 ? lo - b0 : 0u;
    const uint32_t b = hi - b0 >= 32u ? 32u : hi - b0;
    const uint32_t upto = b >= 32u ? 0xFFFFFFFFu : ((1u << b) - 1u);
    return upto & ~((1u << a) - 1u);
}

constexpr uint32_t kWords = 8;

// a request's walk state: selected count, write position, the first four selected rules (stash)
struct WalkState {
    uint32_t cnt;
    uint64_t pos;
    uint32_t st4[4];
};

// Words [lo >> 5, (hi - 1) >> 5] of the rule range [lo, hi): false when the request fails there
// (pass 1 records the error).  kWords bitmap words are loaded before any is used, so a lane's loads
// are in flight together.  kUni: the range is the same for every lane (the default namespace's,
// a kernel-wide constant), so the masks are scalar loads (both TCP rows, selected per lane) and the
// bitmap loads depend on no vector load.
template <bool kWrite, bool kUni>
__device__ __forceinline__ bool walk_range(const mxp_resolve_args& A, uint32_t q, uint32_t tcp, uint32_t lo, uint32_t hi,
                                           WalkState& S) {
    const uint32_t wl = (hi - 1) >> 5;
    const uint32_t* __restrict__ am_lane = A.amask + (uint64_t)tcp * A.n_words;
    for (uint32_t w0 = lo >> 5; w0 <= wl; w0 += kWords) {
        uint32_t mv[kWords], ev[kWords], ap[kWords], emv[kWords];
        // (the masks of all kWords words first, then all their bitmap loads: a load issued after
        // another cannot be waited for alone, so interleaving them serialised the bitmap loads)
#pragma unroll
        for (uint32_t j = 0; j < kWords; j++) {
            const uint32_t w = w0 + j;
            const uint32_t wc = w <= wl ? w : wl;  // (clamped in range)
            if constexpr (kUni) {
                const uint32_t a0 = A.amask[wc], a1 = A.amask[A.n_words + wc];
                ap[j] = w <= wl ? ((tcp ? a1 : a0) & range_bits(w, lo, hi)) : 0u;
            } else {
                ap[j] = w <= wl ? (am_lane[wc] & range_bits(w, lo, hi)) : 0u;
            }
            emv[j] = A.empty[wc];
        }
#pragma unroll
        for (uint32_t j = 0; j < kWords; j++) {
            const uint64_t at = (uint64_t)(w0 + j) * A.n + q;
            mv[j] = ap[j] ? A.match[at] : 0u;
            ev[j] = ap[j] && A.err ? A.err[at] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < kWords; j++) {
            const uint32_t w = w0 + j;
            const uint32_t appl = ap[j];
            if (!appl) continue;
            const uint32_t em = emv[j];
            const uint32_t err = ev[j] & appl & ~em;
            if (err) {  // the first predicate error fails the request
                if (!kWrite) {
                    A.status[q] = MXP_RESOLVE_PRED_ERROR;
                    A.err_rule[q] = w * 32u + __builtin_ctz(err);
                    A.count[q] = 0;
                }
                return false;
            }
            const uint32_t sel = (mv[j] | em) & appl;
            if (kWrite) {
                if (A.ids16) {
                    uint16_t* out = (uint16_t*)A.sel_rules;
                    for (uint32_t b = sel; b; b &= b - 1) out[S.pos++] = (uint16_t)(w * 32u + __builtin_ctz(b));
                } else {
                    for (uint32_t b = sel; b; b &= b - 1) A.sel_rules[S.pos++] = w * 32u + __builtin_ctz(b);
                }
            } else {
                for (uint32_t b = sel, k = S.cnt; b && k < 4u; b &= b - 1, k++) {
                    const uint32_t r = w * 32u + __builtin_ctz(b);
                    S.st4[0] = k == 0u ? r : S.st4[0];  // (selects: no dynamically indexed registers)
                    S.st4[1] = k == 1u ? r : S.st4[1];
                    S.st4[2] = k == 2u ? r : S.st4[2];
                    S.st4[3] = k == 3u ? r : S.st4[3];
                }
                S.cnt += __builtin_popcount(sel);
            }
        }
    }
    return true;
}

// Pass 1 (count): the request's status, first erroring rule and number of selected rules (returned);
// pass 2 (write): its selected rule ids at sel_off[q].
template <bool kWrite>
__device__ __forceinline__ uint32_t walk(const mxp_resolve_args& A, uint32_t q) {
    const uint32_t info = A.nsinfo[q];
    if (info == MXP_NS_MISSING || info == MXP_NS_NOTSTRING) {
        if (!kWrite) {
            A.status[q] = info == MXP_NS_MISSING ? MXP_RESOLVE_NO_IDENTITY : MXP_RESOLVE_BAD_IDENTITY;
            A.err_rule[q] = 0xFFFFFFFFu;
            A.count[q] = 0;
        }
        return 0;
    }
    const uint32_t ns = info & 0x7FFFFFFFu;
    // compact mode: the first applicable error in resolution order is known (error records): its
    // rule, or its rank in the resolution order (default namespace's rules, then the request's own)
    if (!kWrite && A.err_in) {
        const uint32_t er = A.err_in[q];
        if (er != 0xFFFFFFFFu) {
            uint32_t rule = er;
            if (A.err_rank) {
                const bool def = A.default_id != MXP_NS_NONE;
                const uint32_t dlo = def ? A.ns_lo[A.default_id] : 0u, dlen = def ? A.ns_hi[A.default_id] - dlo : 0u;
                rule = er < dlen ? dlo + er : A.ns_lo[ns] + (er - dlen);
            }
            A.status[q] = MXP_RESOLVE_PRED_ERROR;
            A.err_rule[q] = rule;
            A.count[q] = 0;
            return 0;
        }
    }
    const uint32_t tcp = info >> 31;
    WalkState S{0u, kWrite ? A.sel_off[q] : 0ull, {0u, 0u, 0u, 0u}};
    if (A.default_id != MXP_NS_NONE) {
        const uint32_t lo = __builtin_amdgcn_readfirstlane(A.ns_lo[A.default_id]);
        const uint32_t hi = __builtin_amdgcn_readfirstlane(A.ns_hi[A.default_id]);
        if (lo < hi && !walk_range<kWrite, true>(A, q, tcp, lo, hi, S)) return 0;
    }
    if (ns != MXP_NS_NONE && ns != A.default_id) {
        const uint32_t lo = A.ns_lo[ns], hi = A.ns_hi[ns];
        if (lo < hi && !walk_range<kWrite, false>(A, q, tcp, lo, hi, S)) return 0;
    }
    if (!kWrite) {
        A.status[q] = MXP_RESOLVE_OK;
        A.err_rule[q] = 0xFFFFFFFFu;
        A.count[q] = S.cnt;
        if (A.stash) A.stash[q] = make_uint4(S.st4[0], S.st4[1], S.st4[2], S.st4[3]);
    }
    return S.cnt;
}

// sum of v over the 256-thread block (every thread gets it)
__device__ __forceinline__ uint64_t block_sum256(uint64_t v) {
    __shared__ uint64_t part[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint64_t t = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    return t;
}

// exclusive prefix of v over the 256-thread block; *total = the block's sum
__device__ __forceinline__ uint64_t block_excl256(uint64_t v, uint64_t* total) {
    __shared__ uint64_t part[4];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (uint32_t off = 1; off < 64u; off <<= 1) {
        const uint64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63u) part[wave] = x;
    __syncthreads();
    uint64_t before = 0;
    for (uint32_t k = 0; k < wave; k++) before += part[k];
    *total = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
    return before + x - v;
}

// namespace name [p, p + n) -> id (MXP_NS_NONE when no rule namespace has it)
__device__ __forceinline__ uint32_t ns_lookup(const mxp_ns_args& A, const uint8_t* p, uint32_t n) {
    const uint64_t h = mxp_item_hash(p, n);
    const uint32_t tag = (uint32_t)(h >> 32);
    for (uint32_t slot = (uint32_t)h & A.ns_mask;; slot = (slot + 1u) & A.ns_mask) {
        const unsigned long long t = A.ns_tab[slot];
        if (!t) return MXP_NS_NONE;
        if ((uint32_t)(t >> 32) != tag) continue;
        const uint32_t id = (uint32_t)t - 1u;
        const uint64_t d = A.ns_desc[id];
        if ((uint32_t)(d & 0xFFFFFFu) != n) continue;
        const uint8_t* e = A.ns_blob + (d >> 24);
        bool eq = true;
        for (uint32_t i = 0; i < n && eq; i++) eq = e[i] == p[i];
        if (eq) return id;
    }
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_count_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    const uint32_t c = q < A.n ? walk<false>(A, q) : 0u;
    if (A.block_sum) {  // (uniform per launch)
        const uint64_t t = block_sum256(c);
        if (threadIdx.x == 0) A.block_sum[blockIdx.x] = t;
    }
}

// exclusive scan of the count kernel's block sums, in place (one 1024-thread block; nb <= 1024 * 64)
extern "C" __global__ __launch_bounds__(1024) void mxp_resolve_scan_blocks_kernel(uint64_t* bs, uint32_t nb) {
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nb + 1023u) / 1024u;
    uint64_t sum = 0;
    for (uint32_t i = t * per; i < min(nb, (t + 1) * per); i++) sum += bs[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {  // Hillis-Steele over the 1024 partial sums
        const uint64_t y = t >= off ? part[t - off] : 0ull;
        __syncthreads();
        part[t] += y;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;  // exclusive
    for (uint32_t i = t * per; i < min(nb, (t + 1) * per); i++) {
        const uint64_t v = bs[i];
        bs[i] = run;
        run += v;
    }
}

// sel_off[q] = block prefix + the block's own exclusive scan of the counts; sel_off[n] = the total
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_offsets_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    const uint64_t c = q < A.n ? A.count[q] : 0u;
    uint64_t total;
    const uint64_t ex = block_excl256(c, &total);
    const uint64_t base = A.block_sum[blockIdx.x];
    if (q < A.n) A.sel_off_out[q] = base + ex;
    if (blockIdx.x == gridDim.x - 1u && threadIdx.x == 0) A.sel_off_out[A.n] = base + total;
}

// (a guarded write pass: the ids do not fit the capacity they were enqueued for)
__device__ __forceinline__ bool ids_over_cap(const mxp_resolve_args& A) {
    return A.sel_cap_dev && A.sel_off[A.n] > A.sel_cap_dev;
}

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_write_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= A.n || A.status[q] != MXP_RESOLVE_OK || ids_over_cap(A)) return;
    const uint32_t c = A.count[q];
    if (A.stash && c <= 4u) {  // the count pass kept them: no second walk of the bitmaps
        if (!c) return;
        const uint4 v = A.stash[q];
        const uint64_t pos = A.sel_off[q];
        const uint32_t r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t k = 0; k < 4u; k++)
            if (k < c) {
                if (A.ids16) ((uint16_t*)A.sel_rules)[pos + k] = (uint16_t)r[k];
                else A.sel_rules[pos + k] = r[k];
            }
        return;
    }
    walk<true>(A, q);
}

extern "C" __global__ __launch_bounds__(256) void mxp_ns_kernel(mxp_ns_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= A.n) return;
    const uint32_t k = A.id_kind ? A.id_kind[q] : (uint32_t)MXP_ABSENT;
    if (k == MXP_ABSENT) {
        A.nsinfo[q] = MXP_NS_MISSING;
        return;
    }
    if (k != MXP_STRING) {
        A.nsinfo[q] = MXP_NS_NOTSTRING;
        return;
    }
    // strings.SplitN(dest, ".", 3): ns = splits[1] when there is at least one '.', else ""
    const uint64_t s = A.id_val[q];
    const uint8_t* p = A.sbytes + A.soff[s];
    const uint32_t n = (uint32_t)(A.soff[s + 1] - A.soff[s]);
    uint32_t a = n, b = n;  // ns = p[a, b): "" without a '.'
    for (uint32_t i = 0; i < n; i++)
        if (p[i] == '.') {
            a = i + 1u;
            break;
        }
    for (uint32_t i = a; i < n; i++)
        if (p[i] == '.') {
            b = i;
            break;
        }
    const uint32_t id = ns_lookup(A, p + a, b - a);
    // tcp := attrs.Get("context.protocol") == "tcp" (an interface compare: a string "tcp" only)
    bool tcp = false;
    if (A.pr_kind && A.pr_kind[q] == MXP_STRING) {
        const uint64_t t = A.pr_val[q];
        const uint8_t* tp = A.sbytes + A.soff[t];
        tcp = A.soff[t + 1] - A.soff[t] == 3u && tp[0] == 't' && tp[1] == 'c' && tp[2] == 'p';
    }
    A.nsinfo[q] = id | (tcp ? 0x80000000u : 0u);
}

// write: 0 count (+ block sums), 1 write, 2 the device scan of the counts into sel_off_out
// Tiled walk of the default namespace's range (every request's first range, the same for all):
// a workgroup takes 64 requests; per chunk of 64 bitmap words the four waves load the 64 x 64 tile
// with one 256-byte row load per word (coalesced, rows in flight together) into LDS, then each wave
// walks 16 of the tile's requests with lane = word: a popcount and a wave prefix sum give every
// lane its ids' positions, so a request's ids of the chunk go out as one contiguous run (the
// per-lane walk wrote two bytes per lane into 64 different lines per store: C4's 730 MB of action
// lists took 5.2 ms).  The request's own namespace (after the default one in resolution order)
// and the outputs are per-lane work of wave 0 afterwards (walk_range).  kWrite 0: counts, first
// errors (error bitmap), stash; kWrite 1: ids of requests with more than 4 (the stash has the rest).
template <bool kWrite>
__device__ __forceinline__ void resolve_tile(const mxp_resolve_args& A) {
    __shared__ uint32_t tm[64][65];  // match words [word of the chunk][request of the tile] (padded row)
    __shared__ uint32_t te[64][65];  // error words (A.err only)
    __shared__ uint64_t s_run[64];   // pass 1: selected so far; pass 2: next write position
    __shared__ uint32_t s_info[64];  // nsinfo
    __shared__ uint32_t s_skip[64];  // 1: the request is not walked (done, failed, or the stash has it)
    __shared__ uint32_t s_st4[64][4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t base = blockIdx.x * 64u;
    const uint32_t q = base + lane;
    const uint32_t dlo = __builtin_amdgcn_readfirstlane(A.ns_lo[A.default_id]);
    const uint32_t dhi = __builtin_amdgcn_readfirstlane(A.ns_hi[A.default_id]);
    if (wave == 0) {
        uint32_t info = 0u, skip = 1u;
        uint64_t run = 0;
        if (q < A.n) {
            const uint32_t in = A.nsinfo[q];
            if (!kWrite) {
                if (in == MXP_NS_MISSING || in == MXP_NS_NOTSTRING) {
                    A.status[q] = in == MXP_NS_MISSING ? MXP_RESOLVE_NO_IDENTITY : MXP_RESOLVE_BAD_IDENTITY;
                    A.err_rule[q] = 0xFFFFFFFFu;
                    A.count[q] = 0;
                } else if (A.err_in && A.err_in[q] != 0xFFFFFFFFu) {
                    uint32_t rule = A.err_in[q];
                    if (A.err_rank) {
                        const uint32_t dlen = dhi - dlo;
                        rule = rule < dlen ? dlo + rule : A.ns_lo[in & 0x7FFFFFFFu] + (rule - dlen);
                    }
                    A.status[q] = MXP_RESOLVE_PRED_ERROR;
                    A.err_rule[q] = rule;
                    A.count[q] = 0;
                } else {
                    info = in;
                    skip = 0u;
                }
            } else if (A.status[q] == MXP_RESOLVE_OK) {
                const uint32_t c = A.count[q];
                if (!A.stash || c > 4u) {
                    info = in;
                    skip = 0u;
                    run = A.sel_off[q];
                } else if (c) {  // the stash has them
                    const uint4 v = A.stash[q];
                    const uint64_t pos = A.sel_off[q];
                    const uint32_t r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++)
                        if (k < c) {
                            if (A.ids16) ((uint16_t*)A.sel_rules)[pos + k] = (uint16_t)r[k];
                            else A.sel_rules[pos + k] = r[k];
                        }
                }
            }
        }
        s_info[lane] = info;
        s_skip[lane] = skip;
        s_run[lane] = run;
        s_st4[lane][0] = s_st4[lane][1] = s_st4[lane][2] = s_st4[lane][3] = 0u;
    }
    __syncthreads();
    // (no request of the tile to walk -- every one failed, or the stash had it: no tile loads)
    bool any = false;
    if (wave == 0) any = __ballot(s_skip[lane] == 0u) != 0;
    __shared__ uint32_t s_any;
    if (tid == 0) s_any = any ? 1u : 0u;
    __syncthreads();
    const uint32_t wl = dhi > dlo ? (dhi - 1u) >> 5 : 0u;
    for (uint32_t c0 = dlo >> 5; s_any && dhi > dlo && c0 <= wl; c0 += 64u) {
        // the tile: row j of the chunk = word c0 + j of the 64 requests
        for (uint32_t j = wave; j < 64u; j += 4u) {
            const uint32_t w = c0 + j;
            const bool in = w <= wl && q < A.n;
            const uint64_t at = (uint64_t)w * A.n + q;
            tm[j][lane] = in ? A.match[at] : 0u;
            if (A.err) te[j][lane] = in ? A.err[at] : 0u;
        }
        __syncthreads();
        const uint32_t w = c0 + lane;
        const bool wv = w <= wl;
        const uint32_t wc = wv ? w : wl;
        const uint32_t a0 = A.amask[wc], a1 = A.amask[A.n_words + wc], em = A.empty[wc];
        const uint32_t rb = wv ? range_bits(w, dlo, dhi) : 0u;
        for (uint32_t i = 0; i < 16u; i++) {
            const uint32_t r = wave * 16u + i;
            if (s_skip[r]) continue;  // (the same for the whole wave)
            const uint32_t info = s_info[r];
            const uint32_t appl = ((info >> 31) ? a1 : a0) & rb;
            if (!kWrite && A.err) {
                const uint64_t eb = __ballot((te[lane][r] & appl & ~em) != 0u);
                if (eb) {  // the first predicate error fails the request
                    if (lane == (uint32_t)__builtin_ctzll(eb)) {
                        const uint32_t qq = base + r;
                        A.status[qq] = MXP_RESOLVE_PRED_ERROR;
                        A.err_rule[qq] = w * 32u + __builtin_ctz(te[lane][r] & appl & ~em);
                        A.count[qq] = 0;
                        s_skip[r] = 1u;
                    }
                    continue;
                }
            }
            const uint32_t sel = (tm[lane][r] | em) & appl;
            const uint32_t pc = __builtin_popcount(sel);
            uint32_t x = pc;  // inclusive scan over the lanes
#pragma unroll
            for (uint32_t off = 1; off < 64u; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            const uint32_t before = x - pc, total = __shfl(x, 63, 64);
            const uint64_t run = s_run[r];
            if (kWrite) {
                uint64_t pos = run + before;
                if (A.ids16) {
                    uint16_t* out = (uint16_t*)A.sel_rules;
                    for (uint32_t b = sel; b; b &= b - 1) out[pos++] = (uint16_t)(w * 32u + __builtin_ctz(b));
                } else {
                    for (uint32_t b = sel; b; b &= b - 1) A.sel_rules[pos++] = w * 32u + __builtin_ctz(b);
                }
            } else if (run < 4u) {  // the stash: the request's first four ids
                uint64_t k = run + before;
                for (uint32_t b = sel; b && k < 4u; b &= b - 1, k++) s_st4[r][k] = w * 32u + __builtin_ctz(b);
            }
            if (lane == 0) s_run[r] = run + total;
        }
        __syncthreads();
    }
    // the request's own namespace, then the outputs (pass 1)
    if (wave == 0 && q < A.n) {
        if (s_skip[lane]) return;
        const uint32_t info = s_info[lane];
        const uint32_t ns = info & 0x7FFFFFFFu;
        WalkState S{kWrite ? 0u : (uint32_t)s_run[lane], kWrite ? s_run[lane] : 0ull,
                    {s_st4[lane][0], s_st4[lane][1], s_st4[lane][2], s_st4[lane][3]}};
        if (ns != MXP_NS_NONE && ns != A.default_id) {
            const uint32_t lo = A.ns_lo[ns], hi = A.ns_hi[ns];
            if (lo < hi && !walk_range<kWrite, false>(A, q, info >> 31, lo, hi, S)) return;
        }
        if (!kWrite) {
            A.status[q] = MXP_RESOLVE_OK;
            A.err_rule[q] = 0xFFFFFFFFu;
            A.count[q] = S.cnt;
            if (A.stash) A.stash[q] = make_uint4(S.st4[0], S.st4[1], S.st4[2], S.st4[3]);
        }
    }
}

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_tile_count_kernel(mxp_resolve_args A) {
    resolve_tile<false>(A);
}
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_tile_write_kernel(mxp_resolve_args A) {
    if (ids_over_cap(A)) return;
    resolve_tile<true>(A);
}

// Count pass over the default namespace's range without an error bitmap (compact Resolve): a
// workgroup takes 1,024 requests, a thread the four requests t, t + 256, t + 512, t + 768, so the
// workgroup reads each bitmap word's row as one 4 KB run (the per-lane walk read 1 KB runs: 2 TB/s
// on C2's 1.25 GB); kCW words x 4 requests of loads are in flight per thread.  The request's own
// namespace and the outputs per request afterwards; block sums per 256 requests for the scan.
// kVec (the default when n % 4 == 0): a thread takes the four consecutive requests 4t .. 4t + 3
// and reads each word row's four values with one aligned 16-byte load -- a quarter of the load
// instructions: 362 -> 298 us on C2's 1.31 GB (profiles/r6_s21_kernel_stats_e2e_c2_{strided,vec}.csv).
template <bool kVec, uint32_t kCW = 8>  // (kCW word rows of loads in flight)
__device__ __forceinline__ void resolve_count4(const mxp_resolve_args& A) {
    const uint32_t t = threadIdx.x;
    const uint32_t base = blockIdx.x * 1024u;
    auto req = [&](uint32_t k) { return kVec ? base + 4u * t + k : base + t + 256u * k; };
    const uint32_t dlo = __builtin_amdgcn_readfirstlane(A.ns_lo[A.default_id]);
    const uint32_t dhi = __builtin_amdgcn_readfirstlane(A.ns_hi[A.default_id]);
    uint32_t info[4], cnt[4], st[4][4];
    bool act[4];
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t q = req(k);
        act[k] = false;
        info[k] = 0u;
        cnt[k] = 0u;
        st[k][0] = st[k][1] = st[k][2] = st[k][3] = 0u;
        if (q >= A.n) continue;
        const uint32_t in = A.nsinfo[q];
        if (in == MXP_NS_MISSING || in == MXP_NS_NOTSTRING) {
            A.status[q] = in == MXP_NS_MISSING ? MXP_RESOLVE_NO_IDENTITY : MXP_RESOLVE_BAD_IDENTITY;
            A.err_rule[q] = 0xFFFFFFFFu;
            A.count[q] = 0;
        } else if (A.err_in && A.err_in[q] != 0xFFFFFFFFu) {
            uint32_t rule = A.err_in[q];
            if (A.err_rank) {
                const uint32_t dlen = dhi - dlo;
                rule = rule < dlen ? dlo + rule : A.ns_lo[in & 0x7FFFFFFFu] + (rule - dlen);
            }
            A.status[q] = MXP_RESOLVE_PRED_ERROR;
            A.err_rule[q] = rule;
            A.count[q] = 0;
        } else {
            info[k] = in;
            act[k] = true;
        }
    }
    const uint32_t wl = dhi > dlo ? (dhi - 1u) >> 5 : 0u;
    for (uint32_t w0 = dlo >> 5; dhi > dlo && w0 <= wl; w0 += kCW) {
        uint32_t a0[kCW], a1[kCW], em[kCW], mv[kCW][4];
#pragma unroll
        for (uint32_t j = 0; j < kCW; j++) {  // (uniform: scalar loads)
            const uint32_t w = w0 + j, wc = w <= wl ? w : wl;
            const uint32_t rb = w <= wl ? range_bits(w, dlo, dhi) : 0u;
            a0[j] = A.amask[wc] & rb;
            a1[j] = A.amask[A.n_words + wc] & rb;
            em[j] = A.empty[wc];
        }
        if constexpr (kVec) {
            const bool any = act[0] || act[1] || act[2] || act[3];
#pragma unroll
            for (uint32_t j = 0; j < kCW; j++) {
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (any && (a0[j] | a1[j])) v = *(const uint4*)(A.match + (uint64_t)(w0 + j) * A.n + req(0));
                mv[j][0] = act[0] ? v.x : 0u;
                mv[j][1] = act[1] ? v.y : 0u;
                mv[j][2] = act[2] ? v.z : 0u;
                mv[j][3] = act[3] ? v.w : 0u;
            }
        } else {
#pragma unroll
            for (uint32_t j = 0; j < kCW; j++)
#pragma unroll
                for (uint32_t k = 0; k < 4u; k++) {
                    const uint32_t q = req(k);
                    mv[j][k] = act[k] && (a0[j] | a1[j]) ? A.match[(uint64_t)(w0 + j) * A.n + q] : 0u;
                }
        }
#pragma unroll
        for (uint32_t j = 0; j < kCW; j++)
#pragma unroll
            for (uint32_t k = 0; k < 4u; k++) {
                const uint32_t appl = (info[k] >> 31) ? a1[j] : a0[j];
                const uint32_t sel = act[k] ? (mv[j][k] | em[j]) & appl : 0u;
                for (uint32_t b = sel, kk = cnt[k]; b && kk < 4u; b &= b - 1, kk++) {
                    const uint32_t r = (w0 + j) * 32u + __builtin_ctz(b);
                    st[k][0] = kk == 0u ? r : st[k][0];  // (selects: no dynamically indexed registers)
                    st[k][1] = kk == 1u ? r : st[k][1];
                    st[k][2] = kk == 2u ? r : st[k][2];
                    st[k][3] = kk == 3u ? r : st[k][3];
                }
                cnt[k] += __builtin_popcount(sel);
            }
    }
    uint64_t csum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t q = req(k);
        uint32_t c = 0u;
        if (act[k]) {
            const uint32_t ns = info[k] & 0x7FFFFFFFu;
            WalkState S{cnt[k], 0ull, {st[k][0], st[k][1], st[k][2], st[k][3]}};
            bool ok = true;
            if (ns != MXP_NS_NONE && ns != A.default_id) {
                const uint32_t lo = A.ns_lo[ns], hi = A.ns_hi[ns];
                ok = lo >= hi || walk_range<false, false>(A, q, info[k] >> 31, lo, hi, S);
            }
            if (ok) {
                A.status[q] = MXP_RESOLVE_OK;
                A.err_rule[q] = 0xFFFFFFFFu;
                A.count[q] = S.cnt;
                if (A.stash) A.stash[q] = make_uint4(S.st4[0], S.st4[1], S.st4[2], S.st4[3]);
                c = S.cnt;
            }
        }
        if constexpr (kVec) {
            csum += c;
        } else if (A.block_sum) {  // (requests base + 256 k ...: block 4 * blockIdx.x + k of the scan)
            const uint64_t tot = block_sum256(c);
            if (t == 0 && base + 256u * k < A.n) A.block_sum[4u * blockIdx.x + k] = tot;
        }
    }
    if (kVec && A.block_sum) {  // (wave w holds requests base + 256 w ...: block 4 * blockIdx.x + w)
        uint64_t v = csum;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        const uint32_t w = t >> 6;
        if ((t & 63u) == 0 && base + 256u * w < A.n) A.block_sum[4u * blockIdx.x + w] = v;
    }
}
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_count4_kernel(mxp_resolve_args A) { resolve_count4<false>(A); }
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_count4v_kernel(mxp_resolve_args A) { resolve_count4<true>(A); }

// Pair Resolve (resolver.cpp): each request's selected rules straight from the evaluation's deferred
// index pairs.  When every word of the rule set is a plain fill chunk's, a word of the match bitmap
// is 0 but for its pairs (mxp_fill_dtp_kernel), so the pairs filed per (fill chunk, lane quad) by
// mxp_dtp_sort_kernel are the bitmap: the evaluation skips its stores (kargs.dtp_lazy) and these
// passes read a count byte per quad and chunk, and a 16-byte slot row where it is not 0 -- C2:
// ~20 chunks x 1 B per quad instead of 1.31 GB of bitmap written and read again.  A thread takes
// the quad of requests 4t .. 4t + 3 of its workgroup's 1,024, as the fill does.  A quad's entries
// sorted (group, plane, request, bit) give each request's rules of the chunk in ascending order
// with duplicates adjacent; the chunks ascend, so the rules of the default namespace arrive in
// resolution order and so do the request's own namespace's, which resolve after all of them
// (resolver.go:202-238).  Error-plane entries are skipped: a compact evaluation's first errors
// come from its error records (err_in), as in the bitmap passes.
namespace {

__device__ __forceinline__ void sort8r(uint32_t (&x)[8]) {
#define MXP_RCX(a, b)                         \
    {                                         \
        const uint32_t lo = min(x[a], x[b]);  \
        x[b] = max(x[a], x[b]);               \
        x[a] = lo;                            \
    }
    MXP_RCX(0, 1) MXP_RCX(2, 3) MXP_RCX(4, 5) MXP_RCX(6, 7) MXP_RCX(0, 2) MXP_RCX(1, 3) MXP_RCX(4, 6) MXP_RCX(5, 7)
    MXP_RCX(1, 2) MXP_RCX(5, 6) MXP_RCX(0, 4) MXP_RCX(1, 5) MXP_RCX(2, 6) MXP_RCX(3, 7) MXP_RCX(2, 4) MXP_RCX(3, 5)
    MXP_RCX(1, 2) MXP_RCX(3, 4) MXP_RCX(5, 6)
#undef MXP_RCX
}

// kWrite 0: status, first error, count, stash and block sums (as resolve_count4); 1: the ids of the
// requests the stash does not hold, default namespace first (pass 0), then their own (pass 1)
template <bool kWrite>
__device__ __forceinline__ void resolve_pairs(const mxp_resolve_args& A) {
    // the stash while counting: [(request of the quad) * 8 + j][thread], j < 4 the default
    // namespace's first rules, 4 + j the own namespace's (columns per thread: no bank conflicts)
    __shared__ uint32_t s_st[kWrite ? 1 : 32 * 256];
    const uint32_t t = threadIdx.x;
    const uint32_t q0 = blockIdx.x * 1024u + 4u * t;
    const bool has_def = A.default_id != MXP_NS_NONE;
    const uint32_t dlo = has_def ? __builtin_amdgcn_readfirstlane(A.ns_lo[A.default_id]) : 0u;
    const uint32_t dhi = has_def ? __builtin_amdgcn_readfirstlane(A.ns_hi[A.default_id]) : 0u;
    uint32_t info[4], olo[4], ohi[4], cd[4], co[4];
    uint64_t pos[4];
    bool act[4];
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t q = q0 + k;
        act[k] = false;
        info[k] = olo[k] = ohi[k] = cd[k] = co[k] = 0u;
        pos[k] = 0ull;
        if (q >= A.n) continue;
        const uint32_t in = A.nsinfo[q];
        if (!kWrite) {
            if (in == MXP_NS_MISSING || in == MXP_NS_NOTSTRING) {
                A.status[q] = in == MXP_NS_MISSING ? MXP_RESOLVE_NO_IDENTITY : MXP_RESOLVE_BAD_IDENTITY;
                A.err_rule[q] = 0xFFFFFFFFu;
                A.count[q] = 0;
                continue;
            }
            if (A.err_in && A.err_in[q] != 0xFFFFFFFFu) {
                uint32_t rule = A.err_in[q];
                if (A.err_rank) {
                    const uint32_t dlen = dhi - dlo;
                    rule = rule < dlen ? dlo + rule : A.ns_lo[in & 0x7FFFFFFFu] + (rule - dlen);
                }
                A.status[q] = MXP_RESOLVE_PRED_ERROR;
                A.err_rule[q] = rule;
                A.count[q] = 0;
                continue;
            }
            act[k] = true;
        } else {
            if (A.status[q] != MXP_RESOLVE_OK) continue;
            const uint32_t c = A.count[q];
            pos[k] = A.sel_off[q];
            if (A.stash && c <= 4u) {  // the stash has them
                const uint4 v = A.stash[q];
                const uint32_t r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (uint32_t j = 0; j < 4u; j++)
                    if (j < c) {
                        if (A.ids16) ((uint16_t*)A.sel_rules)[pos[k] + j] = (uint16_t)r[j];
                        else A.sel_rules[pos[k] + j] = r[j];
                    }
                continue;
            }
            act[k] = c != 0u;
        }
        info[k] = in;
        const uint32_t ns = in & 0x7FFFFFFFu;
        if (act[k] && ns != MXP_NS_NONE && ns != A.default_id) {
            olo[k] = A.ns_lo[ns];
            ohi[k] = A.ns_hi[ns];
        }
    }
    const bool mine = act[0] || act[1] || act[2] || act[3];
    const bool own = olo[0] < ohi[0] || olo[1] < ohi[1] || olo[2] < ohi[2] || olo[3] < ohi[3];
    constexpr uint32_t kPasses = kWrite ? 2u : 1u;
    for (uint32_t pass = 0; pass < kPasses; pass++) {
        // (kWrite: pass 0 the default namespace's rules, pass 1 the own namespace's; a wave without
        // such requests skips the pass)
        if (!__ballot(mine && (pass == 0u || own))) continue;
        // (the count bytes of kPre chunks loaded together: the walk is a chain of mostly-zero counts)
        constexpr uint32_t kPre = 8;
        for (uint32_t c0 = 0; c0 < A.pr_nch; c0 += kPre) {
            uint32_t kns[kPre];
#pragma unroll
            for (uint32_t j = 0; j < kPre; j++)
                kns[j] = mine && c0 + j < A.pr_nch ? A.pr_qn[(uint64_t)(c0 + j) * A.pr_row + (q0 >> 2)] : 0u;
#pragma unroll
            for (uint32_t jc = 0; jc < kPre; jc++) {
                const uint32_t kn = kns[jc];
                if (!__ballot(kn != 0u)) continue;
                const uint32_t c = c0 + jc;
                const uint32_t g0 = __builtin_amdgcn_readfirstlane(A.pr_fills[8u * c + 2u]);
                const uint64_t qi = (uint64_t)c * A.pr_row + (q0 >> 2);
                if (!kn) continue;
                const uint4 sl = *(const uint4*)(A.pr_slots + qi * 8u);
                const uint32_t h[4] = {sl.x, sl.y, sl.z, sl.w};
                uint32_t x[8];
#pragma unroll
                for (uint32_t i = 0; i < 8u; i++) x[i] = i < kn ? (h[i >> 1] >> (16u * (i & 1u))) & 0xFFFFu : 0xFFFFu;
                if (kn > 1u) sort8r(x);
                uint32_t prev = 0xFFFFFFFFu;
#pragma unroll
                for (uint32_t i = 0; i < 8u; i++) {
                    const uint32_t e = x[i];
                    const bool skip = e == 0xFFFFu || e == prev || (e & 128u);
                    prev = e;
                    if (skip) continue;
                    const uint32_t r = (e >> 5) & 3u, rule = (g0 + (e >> 8)) * 32u + (e & 31u);
#pragma unroll
                    for (uint32_t k = 0; k < 4u; k++) {
                        if (k != r || !act[k]) continue;
                        const uint32_t tcp = info[k] >> 31;
                        if (!((A.amask[tcp * A.n_words + (rule >> 5)] >> (rule & 31u)) & 1u)) continue;
                        const bool def = rule >= dlo && rule < dhi;
                        if (!def && !(rule >= olo[k] && rule < ohi[k])) continue;
                        if (kWrite) {
                            if (def != (pass == 0u)) continue;
                            if (A.ids16) ((uint16_t*)A.sel_rules)[pos[k]++] = (uint16_t)rule;
                            else A.sel_rules[pos[k]++] = rule;
                        } else if (def) {
                            if (cd[k] < 4u) s_st[(k * 8u + cd[k]) * 256u + t] = rule;
                            cd[k]++;
                        } else {
                            if (co[k] < 4u) s_st[(k * 8u + 4u + co[k]) * 256u + t] = rule;
                            co[k]++;
                        }
                    }
                }
            }
        }
    }
    if (kWrite) return;
    uint64_t csum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) {
        const uint32_t q = q0 + k;
        if (!act[k]) continue;
        const uint32_t c = cd[k] + co[k];
        A.status[q] = MXP_RESOLVE_OK;
        A.err_rule[q] = 0xFFFFFFFFu;
        A.count[q] = c;
        if (A.stash) {
            uint32_t st[4];
#pragma unroll
            for (uint32_t j = 0; j < 4u; j++) {
                const uint32_t jo = j - cd[k];  // (own rules follow the default namespace's)
                st[j] = j < cd[k] ? s_st[(k * 8u + j) * 256u + t]
                        : jo < co[k] ? s_st[(k * 8u + 4u + jo) * 256u + t] : 0u;
            }
            A.stash[q] = make_uint4(st[0], st[1], st[2], st[3]);
        }
        csum += c;
    }
    if (A.block_sum) {  // (wave w holds requests base + 256 w ...: block 4 * blockIdx.x + w of the scan)
        uint64_t v = csum;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        const uint32_t w = t >> 6;
        if ((t & 63u) == 0 && blockIdx.x * 1024u + 256u * w < A.n) A.block_sum[4u * blockIdx.x + w] = v;
    }
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_pairs_count_kernel(mxp_resolve_args A) { resolve_pairs<false>(A); }
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_pairs_write_kernel(mxp_resolve_args A) {
    if (ids_over_cap(A)) return;
    resolve_pairs<true>(A);
}



// the count pass's block sums from the counts (the tiled count kernel's blocks are 64 requests)
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_bsum_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    const uint64_t t = block_sum256(q < A.n ? A.count[q] : 0u);
    if (threadIdx.x == 0) A.block_sum[blockIdx.x] = t;
}

// write 0: counts (+ block sums); 1: ids; 2: the scan of the counts; 3 / 4: 0 / 1 tiled (the
// default namespace's range walked by resolve_tile; needs default_id != MXP_NS_NONE); 5 / 6: 0 / 1
// from the deferred pairs (pair Resolve)
extern "C" hipError_t mxp_launch_resolve(const mxp_resolve_args* a, int write, hipStream_t s) {
    const uint32_t grid = (a->n + 255u) / 256u;
    if (write == 1) {
        hipLaunchKernelGGL(mxp_resolve_write_kernel, dim3(grid), dim3(256), 0, s, *a);
    } else if (write == 2) {
        hipLaunchKernelGGL(mxp_resolve_scan_blocks_kernel, dim3(1), dim3(1024), 0, s, a->block_sum, grid);
        hipLaunchKernelGGL(mxp_resolve_offsets_kernel, dim3(grid), dim3(256), 0, s, *a);
    } else if (write == 3) {
        if (!a->err) {  // (compact: the four-request count kernel; with an error bitmap the tiled one)
            // (MXP_RESOLVE_VEC=0: the strided four-request kernel, A/B)
            static const bool vec = !getenv("MXP_RESOLVE_VEC") || atoi(getenv("MXP_RESOLVE_VEC")) != 0;
            // (16 word rows in flight: 146 VGPRs, 3 waves/SIMD, 342 against 298 us on C2,
            // profiles/r6_s22_kernel_stats_e2e_c2_cw{8,16}.csv)
            hipLaunchKernelGGL(vec && (a->n & 3u) == 0u ? mxp_resolve_count4v_kernel : mxp_resolve_count4_kernel,
                               dim3((a->n + 1023u) / 1024u), dim3(256), 0, s, *a);
        } else {
            hipLaunchKernelGGL(mxp_resolve_tile_count_kernel, dim3((a->n + 63u) / 64u), dim3(256), 0, s, *a);
            if (a->block_sum) hipLaunchKernelGGL(mxp_resolve_bsum_kernel, dim3(grid), dim3(256), 0, s, *a);
        }
    } else if (write == 4) {
        hipLaunchKernelGGL(mxp_resolve_tile_write_kernel, dim3((a->n + 63u) / 64u), dim3(256), 0, s, *a);
    } else if (write == 5 || write == 6) {  // pair Resolve: count / ids
        hipLaunchKernelGGL(write == 5 ? mxp_resolve_pairs_count_kernel : mxp_resolve_pairs_write_kernel,
                           dim3((a->n + 1023u) / 1024u), dim3(256), 0, s, *a);
    } else {
        hipLaunchKernelGGL(mxp_resolve_count_kernel, dim3(grid), dim3(256), 0, s, *a);
    }
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_ns(const mxp_ns_args* a, hipStream_t s) {
    hipLaunchKernelGGL(mxp_ns_kernel, dim3((a->n + 255u) / 256u), dim3(256), 0, s, *a);
    return hipGetLastError();
}

// compact Resolve: err_in[q] = rule for each (q, rule) pair of the host's first-error pass
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_scatter_kernel(const uint32_t* pairs, uint32_t m,
                                                                             uint32_t* err_in) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < m) err_in[pairs[2u * i]] = pairs[2u * i + 1u];
}

extern "C" hipError_t mxp_launch_resolve_scatter(const uint32_t* pairs, uint32_t m, uint32_t* err_in, hipStream_t s) {
    if (m) hipLaunchKernelGGL(mxp_resolve_scatter_kernel, dim3((m + 255u) / 256u), dim3(256), 0, s, pairs, m, err_in);
    return hipGetLastError();
}

// compact Resolve: each error record (request, rule) that filterActions would meet -- an applicable
// rule (variety, tcp) with a non-empty match in the request's resolution ranges -- lowers the
// request's first-error rank (err_in, ~0 = none) to the rule's position in the resolution order
extern "C" __global__ __launch_bounds__(256) void mxp_resolve_first_err_kernel(mxp_resolve_args A, const uint4* recs,
                                                                               uint32_t m) {
    const bool def = A.default_id != MXP_NS_NONE;
    const uint32_t dlo = def ? A.ns_lo[A.default_id] : 0u, dhi = def ? A.ns_hi[A.default_id] : 0u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < m; i += gridDim.x * 256u) {
        const uint4 rec = recs[i];
        const uint32_t q = rec.x, r = rec.y;
        if (q >= A.n || r >= A.n_words * 32u) continue;
        const uint32_t info = A.nsinfo[q];
        if (info == MXP_NS_MISSING || info == MXP_NS_NOTSTRING) continue;
        const uint32_t tcp = info >> 31, ns = info & 0x7FFFFFFFu, w = r >> 5, bit = 1u << (r & 31u);
        if ((A.empty[w] & bit) || !(A.amask[(uint64_t)tcp * A.n_words + w] & bit)) continue;
        uint32_t rank;
        if (def && r >= dlo && r < dhi) {
            rank = r - dlo;
        } else if (ns != MXP_NS_NONE && ns != A.default_id && r >= A.ns_lo[ns] && r < A.ns_hi[ns]) {
            rank = (dhi - dlo) + (r - A.ns_lo[ns]);
        } else {
            continue;
        }
        atomicMin((unsigned int*)A.err_in + q, rank);
    }
}

extern "C" hipError_t mxp_launch_resolve_first_err(const mxp_resolve_args* a, const void* recs, uint32_t m,
                                                   hipStream_t s) {
    if (m) {
        const uint32_t need = (m + 255u) / 256u;
        hipLaunchKernelGGL(mxp_resolve_first_err_kernel, dim3(need < 4096u ? need : 4096u), dim3(256), 0, s, *a,
                           (const uint4*)recs, m);
    }
    return hipGetLastError();
}

// Device -> pinned host memory by the shader instead of the copy engine: `dst` is the device
// address of mapped pinned host memory.  On the MI355X box a DMA download runs at ~30 GB/s; 16-byte
// stores from a kernel reach the link's ~54 GB/s (tools/pcie_probe.hip).  When dst
// and src share their alignment mod 16 the body moves in 16-byte words (the head and tail bytewise);
// otherwise bytewise.
__device__ __forceinline__ void d2h_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n) {
    const uint64_t tid = blockIdx.x * 256ull + threadIdx.x, stride = (uint64_t)gridDim.x * 256ull;
    const uint64_t mis = (uint64_t)(uintptr_t)dst & 15u;
    if (mis != ((uint64_t)(uintptr_t)src & 15u)) {
        for (uint64_t i = tid; i < n; i += stride) dst[i] = src[i];
        return;
    }
    const uint64_t head = mis ? (16u - mis < n ? 16u - mis : n) : 0u;
    const uint64_t words = (n - head) >> 4;
    if (tid < head) dst[tid] = src[tid];
    uint4* __restrict__ d16 = (uint4*)(dst + head);
    const uint4* __restrict__ s16 = (const uint4*)(src + head);
    for (uint64_t i = tid; i < words; i += stride) d16[i] = s16[i];
    const uint64_t done = head + (words << 4);
    if (tid < n - done) dst[done + tid] = src[done + tid];
}

extern "C" __global__ __launch_bounds__(256) void mxp_d2h_copy_kernel(uint8_t* __restrict__ dst,
                                                                      const uint8_t* __restrict__ src, uint64_t n) {
    d2h_copy(dst, src, n);
}

// the Resolve's ids, *count of them (isz bytes each), enqueued before the host knows the count: none
// when they exceed cap (the guarded write pass wrote none either)
extern "C" __global__ __launch_bounds__(256) void mxp_d2h_copy_ids_kernel(uint8_t* __restrict__ dst,
                                                                          const uint8_t* __restrict__ src,
                                                                          const uint64_t* count, uint32_t isz, uint64_t cap) {
    const uint64_t c = *count;
    if (c <= cap) d2h_copy(dst, src, c * isz);
}

extern "C" hipError_t mxp_launch_d2h_copy_ids(void* dst, const void* src, const uint64_t* count, uint32_t isz, uint64_t cap,
                                              hipStream_t s) {
    const uint64_t need = (cap * isz / 16u + 255u) / 256u;
    const uint32_t grid = (uint32_t)(need < 1024u ? (need ? need : 1u) : 1024u);
    hipLaunchKernelGGL(mxp_d2h_copy_ids_kernel, dim3(grid), dim3(256), 0, s, (uint8_t*)dst, (const uint8_t*)src, count,
                       isz, cap);
    return hipGetLastError();
}

extern "C" hipError_t mxp_launch_d2h_copy(void* dst, const void* src, uint64_t n, hipStream_t s) {
    if (n) {
        const uint64_t need = (n / 16u + 255u) / 256u;
        const uint32_t grid = (uint32_t)(need < 1024u ? (need ? need : 1u) : 1024u);
        hipLaunchKernelGGL(mxp_d2h_copy_kernel, dim3(grid), dim3(256), 0, s, (uint8_t*)dst, (const uint8_t*)src, n);
    }
    return hipGetLastError();
}
