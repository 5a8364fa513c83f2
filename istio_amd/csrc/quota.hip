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

// 64-bit lane moves through DPP (row shifts and row broadcasts of gfx9-family CDNA), no LDS
template <int kCtrl>
__device__ __forceinline__ int64_t dpp64(int64_t v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(uint64_t)v, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)((uint64_t)v >> 32), kCtrl, 0xF, 0xF, false);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// inclusive prefix sum over the 64 lanes: row_shr 1, 2, 4, 8 within each row of 16, then
// row_bcast:15 and row_bcast:31 carry the rows' totals forward
__device__ __forceinline__ int64_t wave_incl_sum64(int64_t v, uint32_t lane) {
    const uint32_t rl = lane & 15u;
    int64_t t = dpp64<0x111>(v);
    if (rl >= 1u) v += t;
    t = dpp64<0x112>(v);
    if (rl >= 2u) v += t;
    t = dpp64<0x114>(v);
    if (rl >= 4u) v += t;
    t = dpp64<0x118>(v);
    if (rl >= 8u) v += t;
    t = dpp64<0x142>(v);
    if ((lane & 31u) >= 16u) v += t;
    t = dpp64<0x143>(v);
    if (lane >= 32u) v += t;
    return v;
}

__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int64_t o = (int64_t)__shfl_xor((long long)v, off, 64);
        v = o < v ? o : v;
    }
    return rfl64(v);
}

// a key's quota state, wave-uniform (scalar registers).  The reference's sequential semantics
// reduce to one number: the units in use u (a cell's inUse; a rolling window's sum of slots =
// limit - avail), since an alloc of a grants a when u + a <= limit (else 0, or the room when best
// effort) and a free of r grants min(r, u) -- the window's release walk takes min(r, sum of slots).
// A window also tracks its current slot (allocations land there, releases take from it first) and
// the total the releases took from the older slots (applied in one backward walk at the end: older
// slots only ever shrink within a batch, so the walks of all the batch's releases compose).
struct KeyState {
    int64_t m;      // MaxAmount
    int64_t u;      // units in use
    int64_t cur;    // window: current slot's units
    int64_t older;  // window: units the releases took from the older slots
};

// The reference's step for one request (memquota.go:119-214, rollingWindow.go:49-96), any amount
// (the arithmetic wraps as Go's does for amounts near the int64 limits).  Returns the grant.
__device__ __forceinline__ int64_t quota_step(KeyState& S, int64_t amount, bool be) {
    if (amount > 0) {
        const int64_t room = S.m - S.u;
        int64_t g = amount;
        if (g > room) g = be ? room : 0;
        S.u += g;
        S.cur += g;
        return g;
    }
    const int64_t r = (int64_t)(0ull - (uint64_t)amount);  // args.QuotaAmount = -args.QuotaAmount
    const int64_t g = r >= S.u ? S.u : r;
    const int64_t take = S.cur < g ? S.cur : g;
    S.cur -= take;
    S.older += g - take;
    S.u -= g;
    return g;
}

}  // namespace

// One wavefront per key, its requests (sorted by key, in arrival order) 64 at a time; the grants
// are the reference's sequential replay, computed a run at a time instead of a request at a time:
//   * from position t, an inclusive prefix sum S of the amounts over the lanes gives every
//     request's units in use if all of them were granted in full; the first request where that is
//     impossible (an alloc past the limit, a free of more than is in use) is p;
//   * requests [t, p) are granted in full at once (lane-parallel); p is stepped alone (rejected,
//     clamped to the room when best effort, or a free of everything in use); t = p + 1;
//   * with no room left, every alloc up to the next free is granted 0 in one step (ballot); with
//     nothing in use, every free up to the next alloc.
// A saturated key (the Zipf head: ~160k requests per 1M, a limit of a few thousand) needs about one
// such step per 7 requests instead of one per request.  A window's current slot follows the same
// runs: allocs add, frees clamp at 0 -- x -> max(x + S, ...) composes, so its value after a run is
// S_T + max(cur, -min over the run's frees of S_j).  Chunks holding amounts beyond +-2^55 (prefix
// sums could overflow) are stepped request by request (quota_step).
extern "C" __global__ __launch_bounds__(256) void mxp_quota_kernel(mxp_quota_args A) {
    const uint32_t lane = threadIdx.x & 63u;
    // the key and its state are wave-uniform: scalar registers and branches for the whole replay
    const uint32_t k = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (k > A.n_keys) return;
    const uint32_t b = A.seg_start[k], e = A.seg_start[k + 1];
    if (b == e) return;
    if (k == A.n_keys) {  // key ids >= n_keys (mxp_quota_clamp): no state to grant from
        for (uint32_t j = b + lane; j < e; j += 64u) A.granted[A.order[j]] = 0;
        return;
    }
    const int64_t maxv = rfl64(A.max_amount[k]);
    const uint32_t len = A.ticks[k];
    const bool window = len != 0;
    int64_t* slots = window ? A.slots + A.slot_off[k] : nullptr;
    KeyState S{maxv, 0, 0, 0};
    int64_t avail = 0;
    uint32_t cur = 0;
    bool rolled = false;
    if (!window) {
        S.u = rfl64(vload(A.cells + k));
    } else {
        avail = rfl64(vload(A.avail + k));
        cur = __builtin_amdgcn_readfirstlane((uint32_t)__atomic_load_n(A.win_cur + k, __ATOMIC_RELAXED));
        S.u = maxv - avail;
    }
    int64_t u_start = S.u;
    // (prefix sums stay exact while |amounts| <= 2^55 and the limit <= 2^61)
    const int64_t kBig = 1ll << 55;
    const bool small_limit = maxv <= (1ll << 61) && maxv >= -(1ll << 61);
    // The key's requests in sorted order (mxp_quota_gather: contiguous), a group of kG chunks at a
    // time: a group's loads go into registers one group ahead and are copied into this wave's LDS
    // stage at the group boundary, and the chunk replays read only LDS -- so no wait on global
    // memory falls inside the serial replay (rotating prefetched registers chunk by chunk made every
    // chunk wait for its loads: s_waitcnt vmcnt(0) at the loop head, ~5 us per chunk)
    constexpr uint32_t kG = 4;
    __shared__ uint32_t st_i[4][kG * 64u];
    __shared__ int64_t st_a[4][kG * 64u];
    __shared__ uint32_t st_b[4][kG * 64u];
    const uint32_t wv = threadIdx.x >> 6;
    uint32_t ni[kG], nb[kG];
    int64_t na[kG];
#pragma unroll
    for (uint32_t c = 0; c < kG; c++) {
        const uint32_t j = b + c * 64u + lane;
        ni[c] = j < e ? A.order[j] : 0u;
        na[c] = j < e ? A.samt[j] : 0;
        nb[c] = j < e ? (uint32_t)A.sbe[j] : 0u;
    }
    for (uint32_t gb = b; gb < e; gb += kG * 64u) {
#pragma unroll
    for (uint32_t c = 0; c < kG; c++) {
        st_i[wv][c * 64u + lane] = ni[c];
        st_a[wv][c * 64u + lane] = na[c];
        st_b[wv][c * 64u + lane] = nb[c];
        const uint32_t jn = gb + (kG + c) * 64u + lane;
        ni[c] = jn < e ? A.order[jn] : 0u;
        na[c] = jn < e ? A.samt[jn] : 0;
        nb[c] = jn < e ? (uint32_t)A.sbe[jn] : 0u;
    }
    __asm__ volatile("" ::: "memory");  // (keeps the next group's loads issued here, ahead of the replay)
    for (uint32_t c = 0; c < kG; c++) {
        const uint32_t base = gb + c * 64u;
        if (base >= e) break;
        const uint32_t j = base + lane;
        const bool act = j < e;
        const uint32_t i = st_i[wv][c * 64u + lane];
        const int64_t amt = act ? st_a[wv][c * 64u + lane] : 0;
        const uint32_t bef = st_b[wv][c * 64u + lane];
        int64_t res = 0;
        const uint32_t cnt = min(64u, e - base);
        if (window && !rolled && __ballot(amt != 0)) {
            // rollingWindow.roll(currentTick) at the key's first non-zero request (the batch has one
            // tick: later rolls are no-ops): release the slots that fell out of the window
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
            S.cur = behind > 0 ? 0 : readlane64(vload(slots + cur), 0);
            cur = (uint32_t)((cur + behind) % len);
            S.u = maxv - avail;
            u_start = S.u;
            __threadfence_block();
        }
        const bool huge = !small_limit || __ballot(amt > kBig || amt < -kBig) != 0;
        if (huge) {
            for (uint32_t t = 0; t < cnt; t++) {
                const int64_t a = readlane64(amt, t);
                if (a == 0) continue;  // HandleQuota: neither alloc nor free
                const int64_t g = quota_step(S, a, __builtin_amdgcn_readlane(bef, t) != 0);
                res = lane == t ? g : res;
            }
        } else {
            const uint64_t frees = __ballot(amt < 0), allocs = __ballot(amt > 0);
            // one inclusive prefix sum of the chunk's amounts; a run from t with u in use reads the
            // units in use after lane i as u + P_i - P_{t-1}
            const int64_t P = wave_incl_sum64(amt, lane);
            uint32_t t = 0;
            while (t < cnt) {
                const uint64_t from_t = ~0ull << t;
                if (S.u == S.m) {  // no room: allocs grant 0 up to the next free
                    const uint64_t f = frees & from_t;
                    t = f ? (uint32_t)__builtin_ctzll(f) : cnt;
                    if (t >= cnt) break;
                }
                if (S.u == 0) {  // nothing in use: frees grant 0 up to the next alloc
                    const uint64_t f = allocs & from_t;
                    t = f ? (uint32_t)__builtin_ctzll(f) : cnt;
                    if (t >= cnt) break;
                    if (S.u == S.m) continue;
                }
                const int64_t P0 = t ? readlane64(P, t - 1u) : 0;
                const int64_t o = S.u - P0;
                const bool mine = lane >= t;
                const bool bad = mine && ((amt > 0 && o + P > S.m) || (amt < 0 && o + P < 0));
                const uint64_t badm = __ballot(bad);
                const uint32_t p = badm ? (uint32_t)__builtin_ctzll(badm) : cnt;
                // [t, p): granted in full
                if (mine && lane < p) res = amt > 0 ? amt : -amt;
                if (p > t) {
                    const int64_t ST = readlane64(P, p - 1u) - P0;
                    const uint64_t run = from_t & (p >= 64u ? ~0ull : ~(~0ull << p));
                    if (window && (frees & run)) {
                        const int64_t mf = wave_min64(((run >> lane) & 1u) && amt < 0 ? P : INT64_MAX) - P0;
                        const int64_t lift = -mf > S.cur ? -mf : S.cur;  // max(cur, -min S_j)
                        S.older += lift - S.cur;
                        S.cur = ST + lift;
                    } else {
                        S.cur += ST;
                    }
                    S.u += ST;
                }
                if (p >= cnt) break;
                // p alone: an alloc past the limit (rejected, or clamped to the room when best
                // effort) or a free of more than is in use (grants everything in use)
                const int64_t g = quota_step(S, readlane64(amt, p), __builtin_amdgcn_readlane(bef, p) != 0);
                res = lane == p ? g : res;
                t = p + 1;
            }
        }
        if (act) A.granted[i] = res;
    }
    }
    const int64_t delta = S.u - u_start;
    if (window && rolled && S.older != 0) {
        // the releases' share of the older slots: from cur - 1 backwards, each slot giving
        // min(its units, what is still to take) -- lane l holds slot cur - c - l, an inclusive
        // prefix sum over the lanes says what every slot before it gives
        int64_t amount = S.older;
        for (uint32_t c = 1; c < len && amount > 0; c += 64u) {
            const bool in = c + lane < len;
            const uint32_t idx = (cur + len - ((c + lane) % len)) % len;
            const int64_t av = in ? vload(slots + idx) : 0;
            const int64_t incl = wave_incl_sum64(av, lane);
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
            A.cells[k] = S.u;
        } else if (rolled) {
            A.avail[k] = maxv - S.u;
            A.win_cur[k] = cur;
            A.win_tick[k] = A.tick;
            __atomic_store_n(slots + cur, S.cur, __ATOMIC_RELAXED);
        }
        if (A.delta) A.delta[k] += delta;
    }
}

// the requests' amounts and best-effort flags in key-sorted order, for the replay's contiguous loads
extern "C" __global__ void mxp_quota_gather(const uint32_t* order, const int64_t* amount, const uint8_t* be, uint32_t n,
                                            int64_t* samt, uint8_t* sbe) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = order[j];
    samt[j] = amount[i];
    sbe[j] = be[i];
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

extern "C" hipError_t mxp_launch_quota(const mxp_quota_args* a, const uint32_t* skeys, uint32_t* seg_start,
                                       hipStream_t s) {
    // n_keys + 1 segments: the sentinel key n_keys collects the out-of-range ids (granted 0)
    hipLaunchKernelGGL(mxp_quota_segments, dim3((a->n + 1 + 255) / 256), dim3(256), 0, s, skeys, a->n, a->n_keys + 1,
                       seg_start);
    hipLaunchKernelGGL(mxp_quota_gather, dim3((a->n + 255) / 256), dim3(256), 0, s, a->order, a->amount, a->best_effort,
                       a->n, a->samt, a->sbe);
    hipLaunchKernelGGL(mxp_quota_kernel, dim3((a->n_keys + 1 + 3) / 4), dim3(256), 0, s, *a);
    return hipGetLastError();
}
