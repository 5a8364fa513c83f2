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

template <bool kWrite>
__device__ __forceinline__ void walk(const mxp_resolve_args& A, uint32_t q) {
    const uint32_t info = A.nsinfo[q];
    if (info == MXP_NS_MISSING || info == MXP_NS_NOTSTRING) {
        if (!kWrite) {
            A.status[q] = info == MXP_NS_MISSING ? MXP_RESOLVE_NO_IDENTITY : MXP_RESOLVE_BAD_IDENTITY;
            A.err_rule[q] = 0xFFFFFFFFu;
            A.count[q] = 0;
        }
        return;
    }
    const uint32_t ns = info & 0x7FFFFFFFu;
    const uint32_t tcp = info >> 31;
    const uint32_t* amask = A.amask + (uint64_t)tcp * A.n_words;
    uint32_t ranges[2][2];
    uint32_t nr = 0;
    if (A.default_id != MXP_NS_NONE) {
        ranges[nr][0] = A.ns_lo[A.default_id];
        ranges[nr][1] = A.ns_hi[A.default_id];
        nr++;
    }
    if (ns != MXP_NS_NONE && ns != A.default_id) {
        ranges[nr][0] = A.ns_lo[ns];
        ranges[nr][1] = A.ns_hi[ns];
        nr++;
    }
    uint32_t cnt = 0;
    uint64_t pos = kWrite ? A.sel_off[q] : 0;
    for (uint32_t k = 0; k < nr; k++) {
        const uint32_t lo = ranges[k][0], hi = ranges[k][1];
        if (lo >= hi) continue;
        for (uint32_t w = lo >> 5; w <= (hi - 1) >> 5; w++) {
            const uint32_t appl = amask[w] & range_bits(w, lo, hi);
            if (!appl) continue;
            const uint64_t at = (uint64_t)w * A.n + q;
            const uint32_t em = A.empty[w];
            const uint32_t err = A.err[at] & appl & ~em;
            if (err) {  // the first predicate error fails the request
                if (!kWrite) {
                    A.status[q] = MXP_RESOLVE_PRED_ERROR;
                    A.err_rule[q] = w * 32u + __builtin_ctz(err);
                    A.count[q] = 0;
                }
                return;
            }
            const uint32_t sel = (A.match[at] | em) & appl;
            if (kWrite) {
                for (uint32_t b = sel; b; b &= b - 1) A.sel_rules[pos++] = w * 32u + __builtin_ctz(b);
            } else {
                cnt += __builtin_popcount(sel);
            }
        }
    }
    if (!kWrite) {
        A.status[q] = MXP_RESOLVE_OK;
        A.err_rule[q] = 0xFFFFFFFFu;
        A.count[q] = cnt;
    }
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_count_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q < A.n) walk<false>(A, q);
}

extern "C" __global__ __launch_bounds__(256) void mxp_resolve_write_kernel(mxp_resolve_args A) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q < A.n && A.status[q] == MXP_RESOLVE_OK) walk<true>(A, q);
}

extern "C" hipError_t mxp_launch_resolve(const mxp_resolve_args* a, int write, hipStream_t s) {
    const uint32_t grid = (a->n + 255u) / 256u;
    if (write)
        hipLaunchKernelGGL(mxp_resolve_write_kernel, dim3(grid), dim3(256), 0, s, *a);
    else
        hipLaunchKernelGGL(mxp_resolve_count_kernel, dim3(grid), dim3(256), 0, s, *a);
    return hipGetLastError();
}
