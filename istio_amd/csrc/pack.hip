// pack.hip -- the device packer's kernels (pack_args.h; driven by pack_device.cpp).
#include <hip/hip_runtime.h>

#include "../../include/mxp_batch.h"
#include "netparse.h"
#include "pack_args.h"
#include "timeparse.h"
#include "kargs.h"
#include "vm.h"

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kNoValue = ~0ull;

__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }

// the bytes of item `idx` of interning kind `kind` (buf: room for synthesized 16-byte forms)
__device__ __forceinline__ bool item_of(const mxp_pack_args& A, uint32_t kind, uint64_t idx, const uint8_t** p,
                                        uint32_t* n, uint8_t* buf) {
    if (kind == MXP_IK_TIME) {
        if (idx < A.nt) {
            mxp_time_key(A.tsec[idx], A.tnsec[idx], buf);
        } else {
            const uint64_t q = idx - A.nt;
            if (!A.pts_ok[q]) return false;
            mxp_time_key(A.pts_sec[q], A.pts_nsec[q], buf);
        }
        *p = buf;
        *n = 12;
        return true;
    }
    if (idx < A.ns) {
        if (kind != MXP_IK_STR && !(A.use[idx] & 1u)) return false;
        const uint64_t o = A.soff[idx];
        *p = A.sbytes + o;
        *n = (uint32_t)(A.soff[idx + 1] - o);
        if (kind == MXP_IK_CANON && *n == 4) {  // net.IP.Equal: a 4-byte address is its v4-mapped form
            for (int k = 0; k < 10; k++) buf[k] = 0;
            buf[10] = buf[11] = 0xFF;
            for (int k = 0; k < 4; k++) buf[12 + k] = (*p)[k];
            *p = buf;
            *n = 16;
        }
        return true;
    }
    const uint64_t q = idx - A.ns;  // a parsed ip() value (16 bytes; its own canonical form)
    if (!A.pip_ok[q]) return false;
    *p = A.pip + 16 * q;
    *n = 16;
    return true;
}

__device__ __forceinline__ void pool_item(const mxp_pool_view& P, uint32_t kind, uint32_t id, const uint8_t** p,
                                          uint32_t* n, uint8_t* buf) {
    if (kind == MXP_IK_TIME) {
        mxp_time_key(P.tsec[id], P.tnsec[id], buf);
        *p = buf;
        *n = 12;
        return;
    }
    const uint64_t d = P.desc[id];
    *p = P.blob + (d >> 24);
    *n = (uint32_t)(d & 0xFFFFFFu);
}

__device__ __forceinline__ bool same(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb) {
    if (na != nb) return false;
    for (uint32_t k = 0; k < na; k++)
        if (a[k] != b[k]) return false;
    return true;
}

}  // namespace

// BYTES values mark their batch strings (raw / canonical interning covers only those)
extern "C" __global__ __launch_bounds__(256) void mxp_pack_mark_kernel(mxp_pack_args A) {
    for (uint64_t i = gtid(); i < (uint64_t)A.ncol * A.n; i += gstride()) {
        const uint32_t c = (uint32_t)(i / A.n), r = (uint32_t)(i % A.n);
        if (!A.ck[c] || A.vkey[c] != kNone) continue;
        if (A.ck[c][r] == MXP_BYTES) {
            const uint64_t v = A.cv[c][r];
            if (v < A.ns) A.use[v] = 1;
        }
    }
}

// Interning of items [i0, i1) of one kind: the rule-set pool's table first (id = pool id), else
// the batch table -- a CAS on an empty slot makes the item its content's representative; an
// occupied slot with the same hash tag is compared byte by byte (the items are immutable input,
// so a winner's content is readable without further ordering).  id = base + representative.
extern "C" __global__ __launch_bounds__(256) void mxp_pack_intern_kernel(mxp_pack_args A) {
    uint8_t buf[16], pbuf[16];
    for (uint64_t idx = A.i0 + gtid(); idx < A.i1; idx += gstride()) {
        const uint8_t* p;
        uint32_t n;
        if (!item_of(A, A.kind, idx, &p, &n, buf)) {
            A.out[idx] = kNone;
            continue;
        }
        if (A.kind == MXP_IK_STR && A.max_len_out) atomicMax(A.max_len_out, n);
        const uint64_t h = mxp_item_hash(p, n);
        const uint64_t tag = h >> 32;
        uint32_t id = kNone;
        if (A.pool.n) {
            for (uint32_t s = (uint32_t)h & A.pool.mask;; s = (s + 1u) & A.pool.mask) {
                const unsigned long long e = A.pool.ht[s];
                if (!e) break;
                if ((e >> 32) != tag) continue;
                const uint8_t* q;
                uint32_t m;
                pool_item(A.pool, A.kind, (uint32_t)e - 1u, &q, &m, pbuf);
                if (same(p, n, q, m)) {
                    id = (uint32_t)e - 1u;
                    break;
                }
            }
        }
        if (id == kNone) {
            const unsigned long long key = (tag << 32) | (idx + 1u);
            for (uint32_t s = (uint32_t)h & A.bmask;; s = (s + 1u) & A.bmask) {
                unsigned long long e = __hip_atomic_load(A.btab + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!e) {
                    e = atomicCAS(A.btab + s, 0ull, key);
                    if (!e) {
                        id = A.base + (uint32_t)idx;
                        break;
                    }
                }
                if ((e >> 32) != tag) continue;
                const uint64_t other = (uint32_t)e - 1u;
                const uint8_t* q;
                uint32_t m;
                item_of(A, A.kind, other, &q, &m, pbuf);
                if (same(p, n, q, m)) {
                    id = A.base + (uint32_t)other;
                    break;
                }
            }
        }
        A.out[idx] = id;
    }
}

// The engine's columns: kinds / values through the id maps (strings, byte strings, timestamps);
// virtual map[key] columns: the entry whose key is the column's key (interned ids compare).
extern "C" __global__ __launch_bounds__(256) void mxp_pack_gather_kernel(mxp_pack_args A) {
    for (uint64_t i = gtid(); i < (uint64_t)A.ncol * A.n; i += gstride()) {
        const uint32_t c = (uint32_t)(i / A.n), r = (uint32_t)(i % A.n);
        uint8_t k = 0;
        uint64_t v = 0;
        if (A.ck[c]) {
            const uint8_t bk = A.ck[c][r];
            const uint64_t bv = A.cv[c][r];
            if (A.vkey[c] == kNone) {
                k = bk;
                v = bv;
                if (bk == MXP_STRING || bk == MXP_OTHER) v = A.sid[bv];
                else if (bk == MXP_BYTES) v = MXP_BYTES_ID(A.bcan[bv], A.braw[bv]);
                else if (bk == MXP_TIMESTAMP) v = A.tid[bv];
            } else if (bk == MXP_ABSENT) {
                k = VC_ABSENT;
            } else if (bk != MXP_STRING_MAP) {
                k = VC_NOTMAP;
            } else {
                k = VC_VALUE;
                v = A.empty_sid;
                for (uint64_t e = A.moff[bv]; e < A.moff[bv + 1]; e++)
                    if (A.sid[A.mkey[e]] == A.vkey[c]) {
                        v = A.sid[A.mval[e]];
                        break;
                    }
            }
        }
        A.kinds[(uint64_t)c * A.n + r] = k;
        A.vals[(uint64_t)c * A.n + r] = v;
    }
}

// string-map CSR in engine ids
extern "C" __global__ __launch_bounds__(256) void mxp_pack_maps_kernel(mxp_pack_args A) {
    for (uint64_t e = gtid(); e < A.n_entries; e += gstride()) {
        A.omkey[e] = A.sid[A.mkey[e]];
        A.omval[e] = A.sid[A.mval[e]];
    }
    for (uint64_t m = gtid(); m <= A.nm; m += gstride()) A.omoff[m] = (uint32_t)A.moff[m];
}

// aligned overlay pool: exclusive scan of the 8-aligned lengths (block sums, a one-block scan of
// them, add back), then one thread per string copies its bytes
#define MXP_SCAN_B 1024u
extern "C" __global__ __launch_bounds__(1024) void mxp_pack_scan1_kernel(mxp_pack_args A) {
    __shared__ uint64_t sh[MXP_SCAN_B];
    const uint64_t i = (uint64_t)blockIdx.x * MXP_SCAN_B + threadIdx.x;
    const uint64_t len = i < A.ns ? ((A.soff[i + 1] - A.soff[i] + 7u) & ~7ull) : 0;
    sh[threadIdx.x] = len;
    __syncthreads();
    for (uint32_t o = 1; o < MXP_SCAN_B; o <<= 1) {
        const uint64_t x = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
        __syncthreads();
        sh[threadIdx.x] += x;
        __syncthreads();
    }
    if (i < A.ns) A.scan[i] = sh[threadIdx.x] - len;  // exclusive within the block
    if (threadIdx.x == MXP_SCAN_B - 1) A.scan_blocks[blockIdx.x] = sh[threadIdx.x];
}
extern "C" __global__ __launch_bounds__(1024) void mxp_pack_scan2_kernel(mxp_pack_args A, uint32_t nblocks) {
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nblocks; b0 += MXP_SCAN_B) {
        __shared__ uint64_t sh[MXP_SCAN_B];
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t x = b < nblocks ? A.scan_blocks[b] : 0;
        sh[threadIdx.x] = x;
        __syncthreads();
        for (uint32_t o = 1; o < MXP_SCAN_B; o <<= 1) {
            const uint64_t y = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += y;
            __syncthreads();
        }
        const uint64_t c = carry;
        if (b < nblocks) A.scan_blocks[b] = c + sh[threadIdx.x] - x;
        __syncthreads();
        if (threadIdx.x == MXP_SCAN_B - 1) carry = c + sh[threadIdx.x];
        __syncthreads();
    }
    if (threadIdx.x == 0) A.scan[A.ns] = carry;  // total
}
extern "C" __global__ __launch_bounds__(256) void mxp_pack_copy_kernel(mxp_pack_args A) {
    for (uint64_t i = gtid(); i < A.ns; i += gstride()) {
        const uint64_t o = A.scan[i] + A.scan_blocks[i / MXP_SCAN_B];
        const uint64_t s0 = A.soff[i], n = A.soff[i + 1] - s0;
        A.bdesc[i] = (o << 24) | n;
        for (uint64_t k = 0; k < ((n + 7u) & ~7ull); k++) A.bblob[o + k] = k < n ? A.sbytes[s0 + k] : 0;
    }
}

// value classes: distinct string ids (bitmap over [0, S]) and other kinds of each candidate column.
// Zipf-hot values put most requests on a few bitmap words, so a request only reaches the global
// bitmap when nothing cheaper has seen its id: a per-workgroup LDS table of recently marked ids
// (direct-mapped; racy stores only cost a redundant mark), then a plain load of the word (a set bit
// is final, so a stale copy only costs a redundant atomic), then up to eight rounds of in-wave pooling
// (the lanes whose ids share the first needing lane's word OR their bits into one atomic) before the
// remaining lanes' own atomicOr.
#define MXP_VT_MARK_LDS 2048u
extern "C" __global__ __launch_bounds__(256) void mxp_pack_vt_mark_kernel(mxp_pack_args A) {
    __shared__ uint32_t seen[MXP_VT_MARK_LDS];
    const uint32_t a = blockIdx.y;
    const uint32_t c = A.vt_col[a];
    unsigned long long* bits = A.vt_bits + (uint64_t)a * (A.S / 64 + 1);
    for (uint32_t i = threadIdx.x; i < MXP_VT_MARK_LDS; i += 256u) seen[i] = 0xFFFFFFFFu;
    __syncthreads();
    uint32_t km = 0;
    // (uniform trip count per wave: the ballots below need every lane)
    const uint64_t stride = gstride();
    for (uint64_t r0 = gtid() & ~63ull; r0 < A.n; r0 += stride) {
        const uint64_t r = r0 + (threadIdx.x & 63u);
        bool need = false;
        uint32_t x = 0;
        if (r < A.n) {
            const uint8_t k = A.kinds[(uint64_t)c * A.n + r];
            if (k == 1u) {
                const uint64_t v = A.vals[(uint64_t)c * A.n + r];
                x = (uint32_t)(v < A.S ? v : A.S);
                const uint32_t slot = (x * 0x9E3779B1u) >> (32 - 11);
                if (seen[slot] != x) {
                    seen[slot] = x;
                    need = !(bits[x >> 6] & (1ull << (x & 63u)));
                }
            } else {
                km |= 1u << (k & 31u);
            }
        }
        // the lanes sharing the first needing lane's bitmap WORD pool their bits (consecutive
        // interned ids -- a column of mostly distinct values -- put a whole wave on one word)
        for (int round = 0; round < 8; round++) {
            const uint64_t m = __ballot(need);
            if (!m) break;
            const uint32_t lead = (uint32_t)__builtin_ctzll(m);
            const uint32_t w0 = (uint32_t)__shfl((int)(x >> 6), (int)lead, 64);
            const bool same = need && (x >> 6) == w0;
            uint32_t lo = same && (x & 63u) < 32u ? 1u << (x & 31u) : 0u;
            uint32_t hi = same && (x & 63u) >= 32u ? 1u << (x & 31u) : 0u;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                lo |= (uint32_t)__shfl_xor((int)lo, off, 64);
                hi |= (uint32_t)__shfl_xor((int)hi, off, 64);
            }
            if ((threadIdx.x & 63u) == lead) atomicOr(bits + w0, (unsigned long long)hi << 32 | lo);
            if (same) need = false;
        }
        if (need) atomicOr(bits + (x >> 6), 1ull << (x & 63u));
    }
    if (km) atomicOr(A.vt_kmask + a, km);
}
extern "C" __global__ __launch_bounds__(256) void mxp_pack_vt_count_kernel(mxp_pack_args A) {
    const uint32_t a = blockIdx.y;
    const unsigned long long* bits = A.vt_bits + (uint64_t)a * (A.S / 64 + 1);
    uint32_t cnt = 0;
    for (uint64_t w = gtid(); w < A.S / 64 + 1; w += gstride()) cnt += (uint32_t)__builtin_popcountll(bits[w]);
    for (int off = 32; off > 0; off >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, off, 64);
    if ((threadIdx.x & 63u) == 0 && cnt) atomicAdd(A.vt_count + a, (unsigned long long)cnt);
}

// ip() / timestamp() of every string id: the rule-set pool's strings, then the batch's
__device__ __forceinline__ void text_of_id(const mxp_pack_args& A, uint64_t id, const uint8_t** p, uint32_t* n) {
    if (id < A.G) {
        const uint64_t d = A.gdesc[id];
        *p = A.gblob + (d >> 24);
        *n = (uint32_t)(d & 0xFFFFFFu);
    } else {
        const uint64_t s = id - A.G, o = A.soff[s];
        *p = A.sbytes + o;
        *n = (uint32_t)(A.soff[s + 1] - o);
    }
}
extern "C" __global__ __launch_bounds__(256) void mxp_pack_parse_kernel(mxp_pack_args A, uint32_t what) {
    for (uint64_t id = gtid(); id < A.S; id += gstride()) {
        const uint8_t* p;
        uint32_t n;
        text_of_id(A, id, &p, &n);
        if (what == 0) {
            uint8_t ip[16];
            const bool ok = mxpnet::parse_ip(p, n, ip);
            A.pip_ok[id] = ok ? 1 : 0;
            if (ok)
                for (int k = 0; k < 16; k++) A.pip[16 * id + k] = ip[k];
        } else {
            int64_t sec = 0;
            int32_t ns = 0;
            const bool ok = mxptime::parse_rfc3339(p, n, &sec, &ns);
            A.pts_ok[id] = ok ? 1 : 0;
            A.pts_sec[id] = sec;
            A.pts_nsec[id] = ns;
        }
    }
}
// pre-table entries from the interned parsed values
extern "C" __global__ __launch_bounds__(256) void mxp_pack_pretable_kernel(mxp_pack_args A, uint32_t what) {
    for (uint64_t id = gtid(); id < A.S; id += gstride()) {
        if (what == 0)
            A.ipof[id] = A.pip_ok[id] ? MXP_FH(MXP_BYTES, MXP_BYTES_ID(A.bcan[A.ns + id], A.braw[A.ns + id])) : kNoValue;
        else
            A.tsof[id] = A.pts_ok[id] ? MXP_FH(MXP_TIMESTAMP, A.tid[A.nt + id]) : kNoValue;
    }
}

// run-time regexp patterns: the host's (batch string -> rxof) pairs, by interned id
extern "C" __global__ __launch_bounds__(256) void mxp_pack_rx_kernel(mxp_pack_args A) {
    for (uint64_t id = gtid(); id < A.S; id += gstride()) A.rxof[id] = MXP_RXOF_SYNTAX;
}
extern "C" __global__ __launch_bounds__(256) void mxp_pack_rx_scatter_kernel(mxp_pack_args A) {
    for (uint64_t i = gtid(); i < A.n_rx; i += gstride()) {
        const uint32_t k = A.rx_s[i];
        A.rxof[k & 0x80000000u ? k & 0x7FFFFFFFu : A.sid[k]] = A.rx_v[i];
    }
}

// ------------------------------------------------------------------------------------ launchers
namespace {
uint32_t grid_for(uint64_t work) {
    const uint64_t g = (work + 255) / 256;
    return (uint32_t)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}
}  // namespace

extern "C" hipError_t mxp_launch_pack(const mxp_pack_args* a, uint32_t step, uint32_t arg, hipStream_t s) {
    switch (step) {
    case 0: hipLaunchKernelGGL(mxp_pack_mark_kernel, dim3(grid_for((uint64_t)a->ncol * a->n)), dim3(256), 0, s, *a); break;
    case 1: hipLaunchKernelGGL(mxp_pack_intern_kernel, dim3(grid_for(a->i1 - a->i0)), dim3(256), 0, s, *a); break;
    case 2: hipLaunchKernelGGL(mxp_pack_gather_kernel, dim3(grid_for((uint64_t)a->ncol * a->n)), dim3(256), 0, s, *a); break;
    case 3: hipLaunchKernelGGL(mxp_pack_maps_kernel, dim3(grid_for(a->n_entries + a->nm + 1)), dim3(256), 0, s, *a); break;
    case 4: {
        const uint32_t nb = (a->ns + MXP_SCAN_B - 1) / MXP_SCAN_B;
        if (!nb) break;
        hipLaunchKernelGGL(mxp_pack_scan1_kernel, dim3(nb), dim3(MXP_SCAN_B), 0, s, *a);
        hipLaunchKernelGGL(mxp_pack_scan2_kernel, dim3(1), dim3(MXP_SCAN_B), 0, s, *a, nb);
        hipLaunchKernelGGL(mxp_pack_copy_kernel, dim3(grid_for(a->ns)), dim3(256), 0, s, *a);
        break;
    }
    case 5:
        hipLaunchKernelGGL(mxp_pack_vt_mark_kernel, dim3(grid_for(a->n) < 1024 ? grid_for(a->n) : 1024, a->n_vt_cand), dim3(256), 0, s, *a);
        hipLaunchKernelGGL(mxp_pack_vt_count_kernel, dim3(grid_for(a->S / 64 + 1), a->n_vt_cand), dim3(256), 0, s, *a);
        break;
    case 6: hipLaunchKernelGGL(mxp_pack_parse_kernel, dim3(grid_for(a->S)), dim3(256), 0, s, *a, arg); break;
    case 7: hipLaunchKernelGGL(mxp_pack_pretable_kernel, dim3(grid_for(a->S)), dim3(256), 0, s, *a, arg); break;
    case 8:
        hipLaunchKernelGGL(mxp_pack_rx_kernel, dim3(grid_for(a->S)), dim3(256), 0, s, *a);
        if (a->n_rx) hipLaunchKernelGGL(mxp_pack_rx_scatter_kernel, dim3(grid_for(a->n_rx)), dim3(256), 0, s, *a);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
