// quota.hip -- batched memquota (mixer/adapter/memquota) on the GPU.
//
// HandleQuota (memquota.go:107-117) per request, in arrival order per key: alloc (:119-171) and
// free (:173-214) against a non-expiring cell (ValidDuration 0) or a rolling window
// (rollingWindow.go: ticksPerSecond 10, one slot per tick).  Requests for different keys are
// independent; those for one key are sequential.  So: a stable radix sort of (key, arrival index)
// groups each key's requests in order (hipCUB), then one lane per key replays them against the key's
// state in HBM.  Per-key granted deltas (alloc - free) come out for the all-reduce across GPUs.
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


}  // namespace

// One wavefront per key.  A key's requests are sequential (each grant depends on the state the
// previous one left), so the wave streams them 64 at a time -- order / amount / best-effort loaded
// lane-parallel -- and replays them in order in scalar registers, the key's state (cell in-use, or
// window avail + current slot) held in registers for the whole batch; granted amounts are written
// back lane-parallel.  Window slots other than the current one are touched only by releases that
// walk back past it.  The batch has one tick, so the window rolls once, at the key's first non-zero
// request (later rolls in the batch are no-ops: rollingWindow.roll with behind == 0).
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
    const int64_t maxv = A.max_amount[k];
    const uint32_t len = A.ticks[k];
    const bool window = len != 0;
    int64_t* slots = window ? A.slots + A.slot_off[k] : nullptr;
    int64_t in_use = 0, avail = 0, cur_val = 0;
    uint32_t cur = 0;
    bool rolled = false;
    if (!window) {
        in_use = rfl64(vload(A.cells + k));
    } else {
        avail = rfl64(vload(A.avail + k));
        cur = __builtin_amdgcn_readfirstlane((uint32_t)__atomic_load_n(A.win_cur + k, __ATOMIC_RELAXED));
    }
    int64_t delta = 0;
    // the next 64 requests' (order, amount, best effort) gathers are issued before this batch's
    // replay, so their latency hides behind it
    uint32_t i_n = 0, bef_n = 0;
    int64_t amt_n = 0;
    if (b + lane < e) {
        i_n = A.order[b + lane];
        amt_n = A.amount[i_n];
        bef_n = (uint32_t)A.best_effort[i_n];
    }
    for (uint32_t base = b; base < e; base += 64u) {
        const uint32_t j = base + lane;
        const bool act = j < e;
        const uint32_t i = i_n;
        const int64_t amt = amt_n;
        const uint32_t bef = bef_n;
        if (base + 64u + lane < e) {
            i_n = A.order[base + 64u + lane];
            amt_n = A.amount[i_n];
            bef_n = (uint32_t)A.best_effort[i_n];
        }
        int64_t res = 0;
        const uint32_t cnt = min(64u, e - base);
        for (uint32_t t = 0; t < cnt; t++) {
            int64_t amount = readlane64(amt, t);
            if (amount == 0) continue;  // HandleQuota: neither alloc nor free
            if (window && !rolled) {
                // rollingWindow.roll(currentTick): release the slots that fell out of the window
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
                cur_val = behind > 0 ? 0 : readlane64(vload(slots + cur), 0);
                cur = (uint32_t)((cur + behind) % len);
                __threadfence_block();  // the walk below re-reads released slots from lane 0
            }
            const bool be = __builtin_amdgcn_readlane(bef, t) != 0;
            int64_t result;
            if (amount > 0) {  // alloc (memquota.go:119-171)
                result = amount;
                const int64_t room = window ? avail : maxv - in_use;
                if (result > room) {
                    if (!be) {
                        res = lane == t ? 0 : res;
                        continue;
                    }
                    result = room;  // best effort: grab what is left
                }
                if (window) {
                    cur_val += result;
                    avail -= result;
                } else {
                    in_use += result;
                }
                delta += result;
            } else {  // free (memquota.go:173-214)
                amount = -amount;
                if (!window) {
                    result = amount >= in_use ? in_use : amount;  // a cell freed entirely is deleted: same as empty
                    in_use -= result;
                } else {
                    // rollingWindow.release: from the current slot backwards, each slot giving
                    // min(its amount, what is still to release).  The current slot is in a register;
                    // the older ones go 64 at a time: lane l holds slot cur - c - l, and an inclusive
                    // prefix sum over the lanes says how much every slot before it gives, so the
                    // chunk's slots are updated at once instead of one dependent step per slot
                    int64_t total = cur_val < amount ? cur_val : amount;
                    cur_val -= total;
                    amount -= total;
                    for (uint32_t c = 1; c < len && amount > 0; c += 64u) {
                        const bool in = c + lane < len;
                        const uint32_t idx = (cur + len - ((c + lane) % len)) % len;
                        const int64_t av = in ? vload(slots + idx) : 0;
                        int64_t incl = av;
#pragma unroll
                        for (uint32_t off = 1; off < 64u; off <<= 1) {
                            const int64_t up = (int64_t)__shfl_up((long long)incl, off, 64);
                            if (lane >= off) incl += up;
                        }
                        const int64_t before = incl - av, want = amount - before;
                        const int64_t give = want <= 0 ? 0 : want < av ? want : av;
                        if (in && give > 0) __atomic_store_n(slots + idx, av - give, __ATOMIC_RELAXED);
                        __threadfence_block();
                        const int64_t chunk = readlane64(incl, 63);
                        const int64_t took = chunk < amount ? chunk : amount;
                        total += took;
                        amount -= took;
                    }
                    avail += total;
                    result = total;
                }
                delta -= result;
            }
            res = lane == t ? result : res;
        }
        if (act) A.granted[i] = res;
    }
    if (lane == 0) {
        if (!window) {
            A.cells[k] = in_use;
        } else if (rolled) {
            A.avail[k] = avail;
            A.win_cur[k] = cur;
            A.win_tick[k] = A.tick;
            __atomic_store_n(slots + cur, cur_val, __ATOMIC_RELAXED);
        }
        if (A.delta) A.delta[k] += delta;
    }
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
    hipLaunchKernelGGL(mxp_quota_kernel, dim3((a->n_keys + 1 + 3) / 4), dim3(256), 0, s, *a);
    return hipGetLastError();
}
