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

__device__ void roll(const mxp_quota_args& A, uint32_t k, int64_t tick) {
    const uint32_t len = A.ticks[k];
    int64_t* slots = A.slots + A.slot_off[k];
    int64_t behind = tick - A.win_tick[k];
    if (behind > (int64_t)len) behind = len;
    if (behind < 0) behind = 0;  // batch times are non-decreasing (the reference would index out of range)
    uint32_t cur = A.win_cur[k];
    for (int64_t i = 0; i < behind; i++) {
        const uint32_t idx = (uint32_t)((cur + 1 + i) % len);
        A.avail[k] += slots[idx];
        slots[idx] = 0;
    }
    A.win_cur[k] = (uint32_t)((cur + behind) % len);
    A.win_tick[k] = tick;
}

}  // namespace

// one lane per key: replay the key's requests (sorted by arrival) against its state
extern "C" __global__ __launch_bounds__(256) void mxp_quota_kernel(mxp_quota_args A) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= A.n_keys) return;
    const uint32_t b = A.seg_start[k], e = A.seg_start[k + 1];
    const int64_t maxv = A.max_amount[k];
    const bool window = A.ticks[k] != 0;
    int64_t delta = 0;
    for (uint32_t j = b; j < e; j++) {
        const uint32_t i = A.order[j];
        int64_t amount = A.amount[i];
        const bool be = A.best_effort[i] != 0;
        int64_t result = 0;
        if (amount > 0) {  // alloc
            result = amount;
            if (!window) {
                const int64_t in_use = A.cells[k];
                if (result > maxv - in_use) {
                    if (!be) {
                        result = 0;
                        A.granted[i] = 0;
                        continue;
                    }
                    result = maxv - in_use;  // grab as much as we can
                }
                A.cells[k] = in_use + result;
            } else {
                roll(A, k, A.tick);
                if (result > A.avail[k]) {
                    if (!be) {
                        A.granted[i] = 0;
                        continue;
                    }
                    result = A.avail[k];
                }
                A.slots[A.slot_off[k] + A.win_cur[k]] += result;
                A.avail[k] -= result;
            }
            delta += result;
        } else if (amount < 0) {  // free
            amount = -amount;
            result = amount;
            if (!window) {
                const int64_t in_use = A.cells[k];
                if (result >= in_use) {
                    A.cells[k] = 0;  // the cell is deleted: same as an empty one
                    result = in_use;
                } else {
                    A.cells[k] = in_use - result;
                }
            } else {
                // release from the leading edge of the window backwards (rollingWindow.release)
                roll(A, k, A.tick);
                const uint32_t len = A.ticks[k];
                int64_t* slots = A.slots + A.slot_off[k];
                int64_t total = 0;
                int64_t idx = A.win_cur[k];
                for (uint32_t s = 0; s < len; s++) {
                    const int64_t av = slots[idx];
                    if (av >= amount) {
                        slots[idx] -= amount;
                        total += amount;
                        break;
                    }
                    slots[idx] = 0;
                    total += av;
                    amount -= av;
                    idx = idx == 0 ? (int64_t)len - 1 : idx - 1;
                }
                A.avail[k] += total;
                result = total;
            }
            delta -= result;
        }
        A.granted[i] = result;
    }
    if (A.delta) A.delta[k] += delta;
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

extern "C" hipError_t mxp_quota_sort(void* tmp, size_t* tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                                     uint32_t* idx_in, uint32_t* idx_out, uint32_t n, int bits, hipStream_t s) {
    if (tmp) hipLaunchKernelGGL(mxp_quota_iota, dim3((n + 255) / 256), dim3(256), 0, s, idx_in, n);
    return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys_in, keys_out, idx_in, idx_out, (int)n, 0, bits, s);
}

extern "C" hipError_t mxp_launch_quota(const mxp_quota_args* a, const uint32_t* skeys, uint32_t* seg_start,
                                       hipStream_t s) {
    hipLaunchKernelGGL(mxp_quota_segments, dim3((a->n + 1 + 255) / 256), dim3(256), 0, s, skeys, a->n, a->n_keys,
                       seg_start);
    hipLaunchKernelGGL(mxp_quota_kernel, dim3((a->n_keys + 255) / 256), dim3(256), 0, s, *a);
    return hipGetLastError();
}
