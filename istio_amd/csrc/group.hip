// group.hip -- the device half of a group step's counter fold (group.cpp mxp_group_reduce).
//
// After the step's all-reduce each member's step buffer holds the group-wide sums of hits[R] ++
// quota_delta[K]; one pass adds them into the running totals and zeroes the step buffer for the next
// step's fused counters (a few tens of KB: one launch of 16-byte vectors, no second pass to clear).
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ __launch_bounds__(256) void mxp_group_fold_kernel(long long* __restrict__ total,
                                                                         long long* __restrict__ step, uint32_t n) {
    const uint32_t pairs = n / 2u;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < pairs; i += gridDim.x * 256u) {
        longlong2 s = reinterpret_cast<const longlong2*>(step)[i];
        longlong2 t = reinterpret_cast<const longlong2*>(total)[i];
        t.x += s.x;
        t.y += s.y;
        reinterpret_cast<longlong2*>(total)[i] = t;
        reinterpret_cast<longlong2*>(step)[i] = make_longlong2(0, 0);
    }
    if ((n & 1u) && blockIdx.x == 0 && threadIdx.x == 0) {
        total[n - 1] += step[n - 1];
        step[n - 1] = 0;
    }
}

// total / step: 16-byte aligned device buffers of n int64 counters (hipMalloc blocks)
extern "C" hipError_t mxp_launch_group_fold(long long* total, long long* step, uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = (uint32_t)((n / 2u + 255u) / 256u);
    hipLaunchKernelGGL(mxp_group_fold_kernel, dim3(grid ? grid : 1u), dim3(256), 0, s, total, step, n);
    return hipGetLastError();
}
