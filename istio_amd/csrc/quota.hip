// quota.hip -- batched memquota (mixer/adapter/memquota) on the GPU.
//
// HandleQuota (memquota.go:107-117) per request, in arrival order per key: alloc (:119-171) and
// free (:173-214) against a non-expiring cell (ValidDuration 0) or a rolling window
// (rollingWindow.go: ticksPerSecond 10, one slot per tick).  Requests for different keys are
// independent; those for one key are sequential.  So: a stable radix sort of (key, arrival index)
// groups each key's requests in order (hipCUB), then one wavefront per key replays them against the key's
// state in HBM, a run of requests at a time (mxp_quota_kernel).  Per-key granted deltas (alloc -
// free) come out for the all-reduce across GPUs.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <limits>

#include "quota_args.h"

namespace {

// loads of per-key state the kernel also writes: relaxed atomics keep them on the vector memory path
// (a uniform address would otherwise invite a scalar-cache load that cannot see the vector stores)
__device__ __forceinline__ int64_t vload(const int64_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

__device__ __forceinline__ int64_t rfl64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)(uint64_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// lane moves through DPP (row shifts and row broadcasts of gfx9-family CDNA), no LDS
template <int kCtrl>
__device__ __forceinline__ int32_t dpp(int32_t v) {
    return __builtin_amdgcn_update_dpp(0, v, kCtrl, 0xF, 0xF, false);
}
template <int kCtrl>
__device__ __forceinline__ int64_t dpp(int64_t v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(uint64_t)v, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), kCtrl, 0xF, 0xF, false);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int32_t readlane(int32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int64_t readlane(int64_t v, uint32_t l) { return readlane64(v, l); }

// inclusive prefix sum over the 64 lanes: row_shr 1, 2, 4, 8 within each row of 16, then
// row_bcast:15 and row_bcast:31 carry the rows' totals forward
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v, uint32_t lane) {
    const uint32_t rl = lane & 15u;
    T t = dpp<0x111>(v);
    if (rl >= 1u) v += t;
    t = dpp<0x112>(v);
    if (rl >= 2u) v += t;
    t = dpp<0x114>(v);
    if (rl >= 4u) v += t;
    t = dpp<0x118>(v);
    if (rl >= 8u) v += t;
    t = dpp<0x142>(v);
    if ((lane & 31u) >= 16u) v += t;
    t = dpp<0x143>(v);
    if (lane >= 32u) v += t;
    return v;
}

// minimum over the 64 lanes, the same DPP pattern (the fill of lanes a shift leaves empty never
// enters: those lanes keep their own value)
template <typename T>
__device__ __forceinline__ T wave_min(T v, uint32_t lane) {
    const uint32_t rl = lane & 15u;
    T t = dpp<0x111>(v);
    if (rl >= 1u && t < v) v = t;
    t = dpp<0x112>(v);
    if (rl >= 2u && t < v) v = t;
    t = dpp<0x114>(v);
    if (rl >= 4u && t < v) v = t;
    t = dpp<0x118>(v);
    if (rl >= 8u && t < v) v = t;
    t = dpp<0x142>(v);
    if ((lane & 31u) >= 16u && t < v) v = t;
    t = dpp<0x143>(v);
    if (lane >= 32u && t < v) v = t;
    return readlane(v, 63);
}

// A key's quota state reduces to one number, the units in use u (a cell's inUse; a rolling window's
// sum of slots = limit - avail): an alloc of a grants a when u + a <= limit (else 0, or the room
// when best effort) and a free of r grants min(r, u) -- the window's release walk takes min(r, sum
// of slots).  A window also has its current slot (allocations land there, releases take from it
// first) and the older slots the releases reach past it: the current slot follows x -> x + g on an
// alloc and x -> max(x - g, 0) on a free, so over any stretch of requests it is x -> qt + max(x, c)
// (a Slot function, composed as the stretch grows); the older slots give max(x, c) - x, taken in
// one backward walk at the end (older slots only shrink within a batch, so the walks compose).
struct Slot {
    int64_t qt;  // the stretch's signed grants
    int64_t c;   // the clamp (INT64_MIN: no free)
};

__device__ __forceinline__ int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

// F then (qt2, c2): qt2 + max(F.qt + max(x, F.c), c2) = F.qt + qt2 + max(x, F.c, c2 - F.qt)
__device__ __forceinline__ void slot_then(Slot& F, int64_t qt2, int64_t c2) {
    if (c2 != INT64_MIN) {
        const int64_t c = wadd(c2, -F.qt);
        F.c = c > F.c ? c : F.c;
    }
    F.qt = wadd(F.qt, qt2);
}

// The reference's step for one request (memquota.go:119-214, rollingWindow.go:49-96), any amount
// (the arithmetic wraps as Go's does for amounts near the int64 limits).  Returns the grant.
__device__ __forceinline__ int64_t quota_step(int64_t m, int64_t& u, Slot& F, int64_t amount, bool be) {
    if (amount > 0) {
        const int64_t room = wadd(m, -u);
        int64_t g = amount;
        if (g > room) g = be ? room : 0;
        u = wadd(u, g);
        slot_then(F, g, INT64_MIN);
        return g;
    }
    const int64_t r = (int64_t)(0ull - (uint64_t)amount);  // args.QuotaAmount = -args.QuotaAmount
    const int64_t g = r >= u ? u : r;
    u = wadd(u, -g);
    slot_then(F, wadd(0, -g), g);  // max(x - g, 0) = -g + max(x, g)
    return g;
}

// One chunk of a key's requests (lane i: amt, best effort bef; lanes >= cnt hold 0), replayed a
// run at a time on the units in use u alone (limit m).  T is int32_t when the limit, u and the
// amounts are small enough for 32-bit prefix sums (|m|, |u| < 2^28, |amounts| < 2^20), else
// int64_t (|m|, |u| <= 2^61, |amounts| <= 2^55).  Per step, wave-uniform:
//   * skip to the next request that can change the state -- an alloc that fits the room, a best-
//     effort alloc while the room is not 0, a free while units are in use; those skipped grant 0;
//   * from there (t), with P the chunk's inclusive prefix sum of the amounts, request j would
//     leave u + P_j - P_{t-1} in use if all of [t, j] were granted in full: the first j where that
//     is past the limit (an alloc) or below 0 (a free) is p; [t, p) is granted in full;
//   * p alone: an alloc past the room grants the room when best effort (u = m) else 0; a free of
//     more than is in use grants everything in use (u = 0).
// Returns each lane's grant.
template <typename T>
__device__ __forceinline__ T replay_runs(T amt, uint32_t bef, uint32_t lane, uint32_t cnt, T m, T& u, uint32_t& steps) {
    const uint64_t frees = __ballot(amt < 0), allocs = __ballot(amt > 0), bes = __ballot(bef != 0u);
    const T P = wave_incl_sum(amt, lane);
    uint64_t zero = 0, viol = 0;  // lanes granted 0 by a skip; lanes stepped alone (grant in vg)
    T vg = 0;
    uint32_t t = 0;
    while (t < cnt) {
        const T r = m - u;
        const uint64_t from_t = ~0ull << t;
        const uint64_t live = ((allocs & (__ballot(amt <= r) | (r != 0 ? bes : 0ull))) | (u != 0 ? frees : 0ull)) & from_t;
        const uint32_t s = live ? (uint32_t)__builtin_ctzll(live) : 64u;
        if (s >= cnt) {
            zero |= from_t;
            break;
        }
        zero |= from_t & ~(~0ull << s);
        t = s;
        const T P0 = t ? readlane(P, t - 1u) : (T)0;
        const T hi = P0 + r, lo = P0 - u;
        const uint64_t bad = ((allocs & __ballot(P > hi)) | (frees & __ballot(P < lo))) & (~0ull << t);
        steps++;
        if (!bad) {
            u += readlane(P, cnt - 1u) - P0;
            break;
        }
        const uint32_t p = (uint32_t)__builtin_ctzll(bad);
        if (p > t) u += readlane(P, p - 1u) - P0;
        T g;
        if ((allocs >> p) & 1u) {
            const bool be = (bes >> p) & 1u;
            g = be ? m - u : (T)0;
            u = be ? m : u;
        } else {
            g = u;
            u = 0;
        }
        viol |= 1ull << p;
        vg = lane == p ? g : vg;
        t = p + 1u;
    }
    const T full = amt < 0 ? -amt : amt;
    return ((zero >> lane) & 1u) ? (T)0 : ((viol >> lane) & 1u) ? vg : full;
}

// The current slot over a replayed chunk: with Q the prefix sum of the signed grants, the chunk is
// x -> Q_T + max(x, -min over the frees of Q_j)
template <typename T>
__device__ __forceinline__ void slot_chunk(T amt, T res, uint32_t lane, Slot& F) {
    const T sg = amt < 0 ? -res : res;
    const T Q = wave_incl_sum(sg, lane);
    const int64_t QT = readlane(Q, 63u);
    int64_t c = INT64_MIN;
    if (__ballot(amt < 0)) c = -(int64_t)wave_min(amt < 0 ? Q : std::numeric_limits<T>::max(), lane);
    slot_then(F, QT, c);
}

// Long keys are cut into pieces of kPiece requests replayed by waves of their own.  A piece's true
// starting state is unknown until the piece before it is replayed, but it lies in [0, limit], and
// interval arithmetic over the requests narrows that: a free maps [lo, hi] to [max(lo - r, 0),
// max(hi - r, 0)], a best-effort alloc to [min(lo + a, m), min(hi + a, m)] (both monotone), a plain
// alloc (u + a if it fits, else u) to bounds on its two branches.  Where lo == hi the state is
// known whatever it was at the piece's start (a saturated key gets there within a few hundred
// requests: every best-effort alloc past the room lands on the limit).  sync_point finds that
// point in [from, to): returns the first request index after it (the exact state in u), or kNone.
constexpr uint32_t kPiece = 2048;
constexpr uint32_t kSyncMax = 2048;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int64_t kBig = 1ll << 55, kLim = 1ll << 61, kSmall = 1ll << 28;

// Limits of 2^28 and more: request by request on the scalar unit, the hull of a plain alloc's two
// branches.  (An amount past 2^55 ends the walk: no sync point.)
__device__ uint32_t sync_walk64(const mxp_quota_args& A, uint32_t from, uint32_t to, int64_t m, uint32_t lane, int64_t& u) {
    int64_t lo = 0, hi = m;
    for (uint32_t base = from; base < to; base += 64u) {
        const uint32_t j = base + lane;
        const bool in = j < to;
        const int64_t amt = in ? A.samt[j] : 0;
        const uint64_t bes = __ballot(in && A.sbe[j] != 0);
        if (__ballot(amt > kBig || amt < -kBig)) return kNone;
        const uint32_t cnt = min(64u, to - base);
        for (uint32_t t = 0; t < cnt; t++) {
            const int64_t a = readlane64(amt, t);
            if (a < 0) {
                lo = lo + a > 0 ? lo + a : 0;
                hi = hi + a > 0 ? hi + a : 0;
            } else if (a > 0) {
                if ((bes >> t) & 1u) {
                    lo = lo + a < m ? lo + a : m;
                    hi = hi + a < m ? hi + a : m;
                } else {
                    const int64_t edge = m - a;  // states above it do not fit
                    const bool fit = lo <= edge, over = hi > edge;
                    const int64_t nlo = !fit ? lo : !over ? lo + a : min(lo + a, max(lo, edge + 1));
                    const int64_t nhi = !over ? hi + a : fit ? m : hi;
                    lo = nlo;
                    hi = nhi;
                }
            }
            if (lo == hi) {
                u = lo;
                return base + t + 1u;
            }
        }
    }
    return kNone;
}

// Limits below 2^28 (amounts below 2^20, else no sync point): 64 requests at a time, lane-parallel.
// Bound lo and hi separately, each by a clamped add x -> min(max(x + s, L), H): a free of r is
// (-r, 0, inf) for both, a best-effort alloc of a (a, -inf, m); a plain alloc is (a, -inf, m - a + 1)
// for lo (those that fit land at most there, those that do not stay above m - a) and (a, -inf, m)
// for hi (states never exceed the limit).  Clamped adds compose -- f then g is (s1 + s2,
// max(L1 + s2, L2), min(max(H1 + s2, L2), H2)) -- so a prefix scan over the lanes gives every
// request's bounds at once; the first lane where they meet is the sync point.
struct ClampAdd {
    int32_t s, L, H;
};

__device__ __forceinline__ ClampAdd ca_then(ClampAdd f, ClampAdd g) {
    return ClampAdd{f.s + g.s, max(f.L + g.s, g.L), min(max(f.H + g.s, g.L), g.H)};
}

template <int kCtrl>
__device__ __forceinline__ void ca_step(ClampAdd& lo, ClampAdd& hi, bool take) {
    const ClampAdd plo{dpp<kCtrl>(lo.s), dpp<kCtrl>(lo.L), dpp<kCtrl>(lo.H)};
    const ClampAdd phi{plo.s, dpp<kCtrl>(hi.L), dpp<kCtrl>(hi.H)};
    if (take) {
        lo = ca_then(plo, lo);
        hi = ca_then(phi, hi);
    }
}

__device__ uint32_t sync_walk32(const mxp_quota_args& A, uint32_t from, uint32_t to, int32_t m, uint32_t lane, int64_t& u) {
    constexpr int32_t kInf = 1 << 30;
    int32_t lo = 0, hi = m;
    for (uint32_t base = from; base < to; base += 64u) {
        const uint32_t j = base + lane;
        const bool in = j < to;
        const int64_t a64 = in ? A.samt[j] : 0;
        const bool be = in && A.sbe[j] != 0;
        if (__ballot(a64 >= (1 << 20) || a64 <= -(1 << 20))) return kNone;
        const int32_t a = (int32_t)a64;
        ClampAdd flo{a, a < 0 ? 0 : -kInf, a > 0 ? (be ? m : m - a + 1) : kInf};
        ClampAdd fhi{a, a < 0 ? 0 : -kInf, a > 0 ? m : kInf};
        const uint32_t rl = lane & 15u;
        ca_step<0x111>(flo, fhi, rl >= 1u);
        ca_step<0x112>(flo, fhi, rl >= 2u);
        ca_step<0x114>(flo, fhi, rl >= 4u);
        ca_step<0x118>(flo, fhi, rl >= 8u);
        ca_step<0x142>(flo, fhi, (lane & 31u) >= 16u);
        ca_step<0x143>(flo, fhi, lane >= 32u);
        const int32_t vlo = min(max(lo + flo.s, flo.L), flo.H);
        const int32_t vhi = min(max(hi + fhi.s, fhi.L), fhi.H);
        const uint64_t met = __ballot(in && vlo == vhi);
        if (met) {
            const uint32_t t = (uint32_t)__builtin_ctzll(met);
            u = readlane(vlo, t);
            return base + t + 1u;
        }
        lo = readlane(vlo, 63u);  // (lanes past the end are the identity)
        hi = readlane(vhi, 63u);
    }
    return kNone;
}

__device__ __forceinline__ uint32_t sync_point(const mxp_quota_args& A, uint32_t from, uint32_t to, int64_t m, uint32_t lane,
                                               int64_t& u) {
    if (m == 0) {  // in sync from the start
        u = 0;
        return from;
    }
    return m < kSmall ? sync_walk32(A, from, to, (int32_t)m, lane, u) : sync_walk64(A, from, to, m, lane, u);
}

}  // namespace

// One wavefront per (key, piece).  Waves 0 .. n_keys take piece 0 of key w (key n_keys collects
// out-of-range ids: granted 0); wave n_keys + beta (beta >= 1) takes the piece starting at sorted
// position beta * kPiece when that falls strictly inside a key's requests.  A piece's wave replays
// from its sync point (piece 0: from the key's first request, with the state in HBM) up to the next
// piece's sync point (or the key's end), so every request is replayed exactly once from its true
// state.  Single-piece keys finish in place; the waves of a long key leave a record each, and the
// last to finish (a counter per key) composes their Slot functions, walks the older slots and
// writes the key's state.
extern "C" __global__ __launch_bounds__(256) void mxp_quota_kernel(mxp_quota_args A) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    uint32_t k, pstart;
    if (w <= A.n_keys) {
        k = w;
        pstart = A.seg_start[k];
    } else {
        pstart = (w - A.n_keys) * kPiece;
        if (pstart >= A.n) return;
        k = __builtin_amdgcn_readfirstlane(A.skeys[pstart]);
        if (pstart == A.seg_start[k]) return;  // a key's first request: its piece 0
    }
    const uint32_t b = A.seg_start[k], e = A.seg_start[k + 1];
    if (b == e) return;
    if (k == A.n_keys) {  // key ids >= n_keys (mxp_quota_clamp): no state to grant from
        if (pstart == b)
            for (uint32_t j = b + lane; j < e; j += 64u) A.granted[A.order[j]] = 0;
        return;
    }
    const uint32_t p = pstart == b ? 0u : pstart / kPiece - b / kPiece;
    const uint32_t n_pieces = 1u + ((e - 1u) / kPiece - b / kPiece);
    const int64_t maxv = rfl64(A.max_amount[k]);
    const uint32_t len = A.ticks[k];
    const bool window = len != 0;
    int64_t* slots = window ? A.slots + A.slot_off[k] : nullptr;
    // the state in HBM (every wave reads it before any writes it: the writes come after all of the
    // key's waves have finished)
    int64_t avail = 0, u;
    uint32_t cur = 0;
    if (!window) {
        u = rfl64(vload(A.cells + k));
    } else {
        avail = rfl64(vload(A.avail + k));
        cur = __builtin_amdgcn_readfirstlane((uint32_t)__atomic_load_n(A.win_cur + k, __ATOMIC_RELAXED));
        u = maxv - avail;
    }
    // (amounts past 2^55 -- mxp_quota_gather flags their keys -- could wrap the state out of [0, limit])
    const bool pieced = n_pieces > 1u && maxv >= 0 && maxv <= kLim && u >= 0 && u <= maxv && A.big[k] == 0u;
    if (p > 0 && !pieced) return;  // piece 0 replays the whole key
    const bool prof = A.prof != nullptr;
    const int64_t t_start = prof ? (int64_t)wall_clock64() : 0, c_start = prof ? (int64_t)clock64() : 0;
    int64_t c_replay = 0;
    uint32_t iters = 0;
    // [start, end): from this piece's sync point to the next piece's (or the key's end)
    uint32_t start = b, end = e;
    if (p > 0) {
        start = sync_point(A, pstart, min(min(pstart + kPiece, e), pstart + kSyncMax), maxv, lane, u);
        if (start == kNone) start = end = pstart;  // no sync point: the waves before replay this piece
    }
    if (pieced && start != end) {
        for (uint32_t q = p + 1u; q < n_pieces; q++) {
            const uint32_t qs = (b / kPiece + q) * kPiece;
            int64_t uq;
            const uint32_t s = sync_point(A, qs, min(min(qs + kPiece, e), qs + kSyncMax), maxv, lane, uq);
            if (s != kNone) {
                end = s;
                break;
            }
        }
    }
    int64_t u_start = u;  // (piece 0: after the roll)
    Slot F{0, INT64_MIN};
    int64_t x0 = 0;  // piece 0: the current slot after the roll
    bool rolled = false;
    const bool small_limit = maxv <= kLim && maxv >= -kLim;
    // The requests in sorted order (mxp_quota_gather: contiguous), a group of kG chunks at a time: a
    // group's loads go into registers one group ahead and are copied into this wave's LDS stage at
    // the group boundary, and the chunk replays read only LDS -- so no wait on global memory falls
    // inside the serial replay
    constexpr uint32_t kG = 4;
    __shared__ uint32_t st_i[4][kG * 64u];
    __shared__ int64_t st_a[4][kG * 64u];
    __shared__ uint32_t st_b[4][kG * 64u];
    const uint32_t wv = threadIdx.x >> 6;
    uint32_t ni[kG], nb[kG];
    int64_t na[kG];
#pragma unroll
    for (uint32_t c = 0; c < kG; c++) {
        const uint32_t j = start + c * 64u + lane;
        ni[c] = j < end ? A.order[j] : 0u;
        na[c] = j < end ? A.samt[j] : 0;
        nb[c] = j < end ? (uint32_t)A.sbe[j] : 0u;
    }
    for (uint32_t gb = start; gb < end; gb += kG * 64u) {
#pragma unroll
    for (uint32_t c = 0; c < kG; c++) {
        st_i[wv][c * 64u + lane] = ni[c];
        st_a[wv][c * 64u + lane] = na[c];
        st_b[wv][c * 64u + lane] = nb[c];
        const uint32_t jn = gb + (kG + c) * 64u + lane;
        ni[c] = jn < end ? A.order[jn] : 0u;
        na[c] = jn < end ? A.samt[jn] : 0;
        nb[c] = jn < end ? (uint32_t)A.sbe[jn] : 0u;
    }
    __asm__ volatile("" ::: "memory");  // (keeps the next group's loads issued here, ahead of the replay)
    for (uint32_t c = 0; c < kG; c++) {
        const uint32_t base = gb + c * 64u;
        if (base >= end) break;
        const uint32_t j = base + lane;
        const bool act = j < end;
        const uint32_t i = st_i[wv][c * 64u + lane];
        const int64_t amt = act ? st_a[wv][c * 64u + lane] : 0;
        const uint32_t bef = st_b[wv][c * 64u + lane];
        int64_t res = 0;
        const uint32_t cnt = min(64u, end - base);
        if (window && p == 0 && !rolled && __ballot(amt != 0)) {
            // rollingWindow.roll(currentTick) at the key's first non-zero request (the batch has one
            // tick: later rolls are no-ops; it is always in piece 0's stretch, as a sync point needs
            // a non-zero request before it): release the slots that fell out of the window
            rolled = true;
            int64_t behind = A.tick - rfl64(vload(A.win_tick + k));
            if (behind > (int64_t)len) behind = len;
            if (behind < 0) behind = 0;  // batch times are non-decreasing (the reference would index out of range)
            int64_t freed = 0;
            for (int64_t c = 0; c < behind; c += 64) {
                int64_t v = 0;
                if (c + lane < behind) {
                    int64_t* sp = slots + (uint32_t)((cur + 1 + c + lane) % len);
                    v = vload(sp);
                    __atomic_store_n(sp, (int64_t)0, __ATOMIC_RELAXED);
                }
                for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
                freed += readlane64(v, 0);
            }
            avail += freed;
            // the new current slot is one of those just released (behind > 0) or unchanged
            x0 = behind > 0 ? 0 : readlane64(vload(slots + cur), 0);
            cur = (uint32_t)((cur + behind) % len);
            u = maxv - avail;
            u_start = u;
            __threadfence_block();
        }
        const bool huge = !small_limit || u > kLim || u < -kLim || __ballot(amt > kBig || amt < -kBig) != 0;
        if (huge) {
            for (uint32_t t = 0; t < cnt; t++) {
                const int64_t a = readlane64(amt, t);
                if (a == 0) continue;  // HandleQuota: neither alloc nor free
                const int64_t g = quota_step(maxv, u, F, a, __builtin_amdgcn_readlane(bef, t) != 0);
                res = lane == t ? g : res;
            }
        } else if (maxv < kSmall && maxv > -kSmall && u < kSmall && u > -kSmall &&
                   !__ballot(amt >= (1 << 20) || amt <= -(1 << 20))) {
            const int64_t c0 = prof ? (int64_t)clock64() : 0;
            int32_t u32 = (int32_t)u;
            const int32_t r32 = replay_runs<int32_t>((int32_t)amt, bef, lane, cnt, (int32_t)maxv, u32, iters);
            u = u32;
            res = r32;
            if (window) slot_chunk<int32_t>((int32_t)amt, r32, lane, F);
            if (prof) c_replay += (int64_t)clock64() - c0;
        } else {
            res = replay_runs<int64_t>(amt, bef, lane, cnt, maxv, u, iters);
            if (window) slot_chunk<int64_t>(amt, res, lane, F);
        }
        if (act) A.granted[i] = res;
    }
    }
    int64_t u_end = u;
    bool last = true;
    if (pieced) {
        // leave this piece's record; the key's last wave to finish composes them
        int64_t* R = A.prec + 6ull * (p == 0 ? k : A.n_keys + pstart / kPiece);
        if (lane == 0) {
            R[0] = F.qt;
            R[1] = F.c;
            R[2] = u;
            R[3] = u_start;
            R[4] = x0;
            R[5] = (int64_t)(((uint64_t)cur << 32) | (rolled ? 2u : 0u) | (end == e && start != end ? 1u : 0u));
        }
        __threadfence();
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd(A.done + k, 1u);
        old = __builtin_amdgcn_readfirstlane(old);
        last = old == n_pieces - 1u;
        if (last) {
            __threadfence();
            if (lane == 0) A.done[k] = 0;  // (ready for the next batch)
            F = Slot{0, INT64_MIN};
            for (uint32_t q = 0; q < n_pieces; q++) {
                const int64_t* Rq = A.prec + 6ull * (q == 0 ? k : A.n_keys + (b / kPiece + q));
                const uint64_t fl = (uint64_t)rfl64(vload(Rq + 5));
                if (q == 0) {
                    u_start = rfl64(vload(Rq + 3));
                    x0 = rfl64(vload(Rq + 4));
                    rolled = (fl & 2u) != 0;
                    cur = (uint32_t)(fl >> 32);
                }
                if (fl & 1u) u_end = rfl64(vload(Rq + 2));
                slot_then(F, rfl64(vload(Rq + 0)), rfl64(vload(Rq + 1)));
            }
        }
    }
    if (prof && lane == 0) {  // (debug: MXP_QUOTA_PROF) per wave: time (100 MHz ticks), run steps,
        A.prof[4 * w] = (int64_t)wall_clock64() - t_start;  // shader clocks in all and in the 32-bit
        A.prof[4 * w + 1] = iters;                           // replays
        A.prof[4 * w + 2] = (int64_t)clock64() - c_start;
        A.prof[4 * w + 3] = c_replay;
    }
    if (!last) return;
    const int64_t delta = u_end - u_start;
    const int64_t lift = F.c > x0 ? F.c : x0;
    const int64_t older = lift - x0;  // what the releases took from the older slots
    if (window && rolled && older != 0) {
        // from cur - 1 backwards, each slot giving min(its units, what is still to take) -- lane l
        // holds slot cur - c - l, an inclusive prefix sum over the lanes says what every slot before
        // it gives
        int64_t amount = older;
        for (uint32_t c = 1; c < len && amount > 0; c += 64u) {
            const bool in = c + lane < len;
            const uint32_t idx = (cur + len - ((c + lane) % len)) % len;
            const int64_t av = in ? vload(slots + idx) : 0;
            const int64_t incl = wave_incl_sum(av, lane);
            const int64_t before = incl - av, want = amount - before;
            const int64_t give = want <= 0 ? 0 : want < av ? want : av;
            if (in && give > 0) __atomic_store_n(slots + idx, av - give, __ATOMIC_RELAXED);
            __threadfence_block();
            const int64_t chunk = readlane64(incl, 63);
            amount -= chunk < amount ? chunk : amount;
        }
    }
    if (lane == 0) {
        if (!window) {
            A.cells[k] = u_end;
        } else if (rolled) {
            A.avail[k] = maxv - u_end;
            A.win_cur[k] = cur;
            A.win_tick[k] = A.tick;
            __atomic_store_n(slots + cur, wadd(F.qt, lift), __ATOMIC_RELAXED);
        }
        if (A.delta) A.delta[k] += delta;
    }
}

// the requests' amounts and best-effort flags in key-sorted order, for the replay's contiguous loads
// (and flags the keys holding amounts past +-2^55: those are never cut into pieces)
extern "C" __global__ void mxp_quota_gather(const uint32_t* order, const uint32_t* skeys, const int64_t* amount,
                                            const uint8_t* be, uint32_t n, int64_t* samt, uint8_t* sbe, uint32_t* big) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = order[j];
    const int64_t a = amount[i];
    samt[j] = a;
    sbe[j] = be[i];
    if (a > kBig || a < -kBig) big[skeys[j]] = 1u;
}

extern "C" __global__ void mxp_quota_iota(uint32_t* v, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) v[i] = i;
}

// segment starts of the sorted keys: seg_start[k] = first position with key >= k
extern "C" __global__ void mxp_quota_segments(const uint32_t* skeys, uint32_t n, uint32_t n_keys, uint32_t* seg_start) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i > n) return;
    const uint32_t prev = i == 0 ? 0u : skeys[i - 1] + 1u;
    const uint32_t cur = i == n ? n_keys : skeys[i];
    for (uint32_t k = prev; k <= cur && k <= n_keys; k++) seg_start[k] = i;
}

// key ids outside [0, n_keys) become the sentinel n_keys: the radix sort only looks at the low bits
// of n_keys, so an out-of-range id would otherwise sort as another key and replay against its state
extern "C" __global__ void mxp_quota_clamp(const uint32_t* key, uint32_t n, uint32_t n_keys, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) out[i] = min(key[i], n_keys);
}

// sorts the clamped keys (keys_in is scratch of n entries, overwritten with the clamped copy)
extern "C" hipError_t mxp_quota_sort(void* tmp, size_t* tmp_bytes, const uint32_t* key, uint32_t n_keys,
                                     uint32_t* keys_in, uint32_t* keys_out, uint32_t* idx_in, uint32_t* idx_out,
                                     uint32_t n, int bits, hipStream_t s) {
    if (tmp) {
        hipLaunchKernelGGL(mxp_quota_clamp, dim3((n + 255) / 256), dim3(256), 0, s, key, n, n_keys, keys_in);
        hipLaunchKernelGGL(mxp_quota_iota, dim3((n + 255) / 256), dim3(256), 0, s, idx_in, n);
    }
    return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys_in, keys_out, idx_in, idx_out, (int)n, 0, bits, s);
}

// ---- bucketing the requests by key (up to kMaxBins - 1 keys): a stable counting sort in three
// passes, in place of a radix sort (whose passes all see the whole batch) plus the gather and segment
// kernels.  Tiles of kTile requests in arrival order, one wave each:
//   mxp_quota_hist     each tile's count per key (LDS), into H[key][tile]
//   mxp_quota_binscan  one wave per key: exclusive prefix over the tiles (in place), the key's total
//   mxp_quota_scatter  each tile: the keys' segment starts (exclusive prefix of the totals; tile 0
//                      stores seg_start) + the tile's prefix = where its requests of each key go;
//                      64 requests at a time, a request's rank among its key's in the 64 from the
//                      key's bits (one ballot per bit: the lanes agreeing on all bits share its key)
//                      -- arrival order kept within a key -- and the group's first lane moves the
//                      key's position past the group.  Writes order, skeys, the amounts and
//                      best-effort flags in sorted order, and flags keys with amounts past 2^55.
constexpr uint32_t kTile = 1024;  // (same-box: 2048 0.259 / 0.260 ms, 1024 0.253 / 0.255, 512 0.270 / 0.272; profiles/r3_v16_quota_tiles.log)

extern "C" __global__ __launch_bounds__(64) void mxp_quota_hist(const uint32_t* key, uint32_t n, uint32_t n_keys,
                                                                uint32_t tiles, uint32_t* H) {
    extern __shared__ uint32_t h[];
    const uint32_t bins = n_keys + 1u, t = blockIdx.x, lane = threadIdx.x;
    for (uint32_t b = lane; b < bins; b += 64u) h[b] = 0;
    __syncthreads();
    const uint32_t j1 = min(t * kTile + kTile, n);
    for (uint32_t j = t * kTile + lane; j < j1; j += 64u) atomicAdd(&h[min(key[j], n_keys)], 1u);
    __syncthreads();
    for (uint32_t b = lane; b < bins; b += 64u) H[(size_t)b * tiles + t] = h[b];
}

extern "C" __global__ void mxp_quota_binscan(uint32_t* H, uint32_t tiles, uint32_t bins, uint32_t* tot) {
    const uint32_t b = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (b >= bins) return;
    uint32_t* row = H + (size_t)b * tiles;
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < tiles; t0 += 64u) {
        const uint32_t t = t0 + lane;
        const int32_t v = t < tiles ? (int32_t)row[t] : 0;
        const int32_t incl = wave_incl_sum(v, lane);
        if (t < tiles) row[t] = carry + (uint32_t)(incl - v);
        carry += (uint32_t)readlane(incl, 63u);
    }
    if (lane == 0) tot[b] = carry;
}

extern "C" __global__ __launch_bounds__(64) void mxp_quota_scatter(const uint32_t* key, const int64_t* amount,
                                                                   const uint8_t* be, uint32_t n, uint32_t n_keys,
                                                                   uint32_t tiles, const uint32_t* H, const uint32_t* tot,
                                                                   uint32_t* order, uint32_t* skeys, int64_t* samt,
                                                                   uint8_t* sbe, uint32_t* big, uint32_t* seg_start) {
    extern __shared__ uint32_t pos[];
    const uint32_t bins = n_keys + 1u, t = blockIdx.x, lane = threadIdx.x;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < bins; b0 += 64u) {
        const uint32_t b = b0 + lane;
        const int32_t v = b < bins ? (int32_t)tot[b] : 0;
        const int32_t incl = wave_incl_sum(v, lane);
        const uint32_t start = carry + (uint32_t)(incl - v);
        if (b < bins) {
            pos[b] = start + H[(size_t)b * tiles + t];
            if (t == 0) seg_start[b] = start;
        }
        carry += (uint32_t)readlane(incl, 63u);
    }
    if (t == 0 && lane == 0) seg_start[bins] = carry;
    __syncthreads();
    const uint32_t bits = n_keys ? 32u - (uint32_t)__builtin_clz(n_keys) : 0u;
    const uint32_t j1 = min(t * kTile + kTile, n);
    for (uint32_t j0 = t * kTile; j0 < j1; j0 += 64u) {
        const uint32_t j = j0 + lane;
        const bool in = j < j1;
        const uint32_t k = in ? min(key[j], n_keys) : 0u;
        uint64_t peers = __ballot(in);
        for (uint32_t bit = 0; bit < bits; bit++) {
            const bool on = (k >> bit) & 1u;
            const uint64_t m = __ballot(on);
            peers &= on ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__builtin_popcountll(peers & ((1ull << lane) - 1ull));
        const uint32_t p = in ? pos[k] + rank : 0u;  // (every lane reads before any first lane writes)
        if (in && rank == 0) pos[k] = p + (uint32_t)__builtin_popcountll(peers);
        if (in) {
            const int64_t a = amount[j];
            order[p] = j;
            skeys[p] = k;
            samt[p] = a;
            sbe[p] = be[j];
            if (a > kBig || a < -kBig) big[k] = 1u;
        }
    }
}

extern "C" size_t mxp_quota_bucket_words(uint32_t n, uint32_t n_keys) {
    const size_t tiles = (n + kTile - 1) / kTile;
    return ((size_t)n_keys + 1) * (tiles + 1);
}

// the waves beyond the keys' first pieces (positions kPiece, 2 kPiece, ... below n), and the
// piece records the kernel needs (6 words each, n_keys + 1 + that many)
extern "C" uint32_t mxp_quota_piece_waves(uint32_t n) { return n ? (n - 1u) / kPiece : 0u; }

// bucketed == nullptr: the requests were radix sorted (mxp_quota_sort) -- segments and gather
// here; else bucketed is the scratch of mxp_quota_bucket_words words and the keys are bucketed here
extern "C" hipError_t mxp_launch_quota(const mxp_quota_args* a, uint32_t* bucketed, hipStream_t s) {
    const uint32_t bins = a->n_keys + 1u;  // the sentinel key n_keys collects the out-of-range ids (granted 0)
    hipError_t e = hipMemsetAsync(a->big, 0, (size_t)bins * 4, s);
    if (e != hipSuccess) return e;
    if (bucketed) {
        const uint32_t tiles = (a->n + kTile - 1) / kTile;
        uint32_t* H = bucketed;
        uint32_t* tot = bucketed + (size_t)bins * tiles;
        hipLaunchKernelGGL(mxp_quota_hist, dim3(tiles), dim3(64), bins * 4, s, a->key, a->n, a->n_keys, tiles, H);
        hipLaunchKernelGGL(mxp_quota_binscan, dim3((bins + 3) / 4), dim3(256), 0, s, H, tiles, bins, tot);
        hipLaunchKernelGGL(mxp_quota_scatter, dim3(tiles), dim3(64), bins * 4, s, a->key, a->amount, a->best_effort,
                           a->n, a->n_keys, tiles, (const uint32_t*)H, (const uint32_t*)tot, (uint32_t*)a->order,
                           (uint32_t*)a->skeys, a->samt, a->sbe, a->big, (uint32_t*)a->seg_start);
    } else {
        hipLaunchKernelGGL(mxp_quota_segments, dim3((a->n + 1 + 255) / 256), dim3(256), 0, s, a->skeys, a->n, bins,
                           (uint32_t*)a->seg_start);
        hipLaunchKernelGGL(mxp_quota_gather, dim3((a->n + 255) / 256), dim3(256), 0, s, a->order, a->skeys, a->amount,
                           a->best_effort, a->n, a->samt, a->sbe, a->big);
    }
    // waves: piece 0 of keys 0 .. n_keys, then one per kPiece-aligned sorted position
    const uint32_t waves = a->n_keys + 1u + mxp_quota_piece_waves(a->n);
    hipLaunchKernelGGL(mxp_quota_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, *a);
    return hipGetLastError();
}
