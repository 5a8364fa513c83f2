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
    const uint32_t c = blockIdx.y;  // (grid: requests x columns)
    if (!A.ck[c] || A.vkey[c] != kNone) return;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < A.n; r += (uint64_t)gridDim.x * blockDim.x) {
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
// Strings (MXP_IK_STR) hash and compare 8 bytes at a time (the batch blob and the pools carry 16
// bytes of slack).  (The longest string comes from the scan kernels: an atomic max per wave here --
// 28k waves on one address for C2's 1.8M strings, ~11 ns each -- was 0.33 ms of this pass.)
__device__ __forceinline__ uint64_t ld8_any(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7) * 8u;
    const uint64_t lo = q[0];
    return sh == 0 ? lo : (lo >> sh) | (q[1] << (64u - sh));
}
__device__ __forceinline__ uint64_t str_hash_words(const uint8_t* p, uint32_t n) {
    uint64_t h = 0;
    for (uint32_t i = 0; i < n; i += 8) {
        const uint32_t r = n - i;
        const uint64_t w = ld8_any(p + i) & (r >= 8u ? ~0ull : (1ull << (8u * r)) - 1ull);
        h ^= w;
        h *= 0x9E3779B97F4A7C15ull;
        h ^= h >> 31;
    }
    h ^= (uint64_t)n * 0xC2B2AE3D27D4EB4Full;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}
__device__ __forceinline__ bool same_words(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb) {
    if (na != nb) return false;
    for (uint32_t i = 0; i < na; i += 8) {
        const uint32_t r = na - i;
        const uint64_t m = r >= 8u ? ~0ull : (1ull << (8u * r)) - 1ull;
        if ((ld8_any(a + i) ^ ld8_any(b + i)) & m) return false;
    }
    return true;
}

// (kWords: the string pass -- its items are the batch strings as given, so it needs no buffers for
// synthesized forms and no scratch)
template <bool kWords>
__device__ __forceinline__ void intern_body(const mxp_pack_args& A) {
    uint8_t buf[kWords ? 1 : 16], pbuf[kWords ? 1 : 16];
    constexpr bool words = kWords;
    for (uint64_t idx = A.i0 + gtid(); idx < A.i1; idx += gstride()) {
        const uint8_t* p;
        uint32_t n;
        if constexpr (kWords) {
            const uint64_t o = A.soff[idx];
            p = A.sbytes + o;
            n = (uint32_t)(A.soff[idx + 1] - o);
        } else if (!item_of(A, A.kind, idx, &p, &n, buf)) {
            A.out[idx] = kNone;
            continue;
        }
        const uint64_t h = words ? str_hash_words(p, n) : mxp_item_hash(p, n);
        const uint64_t tag = h >> 32;
        uint32_t id = kNone;
        if (A.pool.n) {
            for (uint32_t s = (uint32_t)h & A.pool.mask;; s = (s + 1u) & A.pool.mask) {
                const unsigned long long e = A.pool.ht[s];
                if (!e) break;
                if ((e >> 32) != tag) continue;
                const uint8_t* q;
                uint32_t m;
                if constexpr (kWords) {
                    const uint64_t d = A.pool.desc[(uint32_t)e - 1u];
                    q = A.pool.blob + (d >> 24);
                    m = (uint32_t)(d & 0xFFFFFFu);
                } else {
                    pool_item(A.pool, A.kind, (uint32_t)e - 1u, &q, &m, pbuf);
                }
                if (words ? same_words(p, n, q, m) : same(p, n, q, m)) {
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
                if constexpr (kWords) {
                    const uint64_t o = A.soff[other];
                    q = A.sbytes + o;
                    m = (uint32_t)(A.soff[other + 1] - o);
                } else {
                    item_of(A, A.kind, other, &q, &m, pbuf);
                }
                if (words ? same_words(p, n, q, m) : same(p, n, q, m)) {
                    id = A.base + (uint32_t)other;
                    break;
                }
            }
        }
        A.out[idx] = id;
    }
}
extern "C" __global__ __launch_bounds__(256) void mxp_pack_intern_kernel(mxp_pack_args A) { intern_body<false>(A); }
extern "C" __global__ __launch_bounds__(256) void mxp_pack_intern_str_kernel(mxp_pack_args A) { intern_body<true>(A); }

// The engine's columns: kinds / values through the id maps (strings, byte strings, timestamps);
// virtual map[key] columns: the entry whose key is the column's key (interned ids compare).
// (grid: requests x columns, blockIdx.y = column -- no 64-bit division per element)
extern "C" __global__ __launch_bounds__(256) void mxp_pack_gather_kernel(mxp_pack_args A) {
    const uint32_t c = blockIdx.y;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < A.n; r += (uint64_t)gridDim.x * blockDim.x) {
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
// them, add back), then one thread per string copies its bytes.  The scans also find the longest
// string (block maxima, reduced by the one-block scan).
#define MXP_SCAN_B 1024u
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, off, 64));
    return x;
}
extern "C" __global__ __launch_bounds__(1024) void mxp_pack_scan1_kernel(mxp_pack_args A) {
    __shared__ uint64_t sh[MXP_SCAN_B];
    __shared__ uint32_t bmax;
    const uint64_t i = (uint64_t)blockIdx.x * MXP_SCAN_B + threadIdx.x;
    const uint64_t raw = i < A.ns ? A.soff[i + 1] - A.soff[i] : 0;
    const uint64_t len = (raw + 7u) & ~7ull;
    if (threadIdx.x == 0) bmax = 0u;
    sh[threadIdx.x] = len;
    __syncthreads();
    {
        const uint32_t m = wave_max_u32((uint32_t)min(raw, (uint64_t)0xFFFFFFFFu));
        if ((threadIdx.x & 63u) == 0) atomicMax(&bmax, m);  // (LDS: 16 per block)
    }
    for (uint32_t o = 1; o < MXP_SCAN_B; o <<= 1) {
        const uint64_t x = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
        __syncthreads();
        sh[threadIdx.x] += x;
        __syncthreads();
    }
    if (i < A.ns) A.scan[i] = sh[threadIdx.x] - len;  // exclusive within the block
    if (threadIdx.x == MXP_SCAN_B - 1) A.scan_blocks[blockIdx.x] = sh[threadIdx.x];
    if (threadIdx.x == 0) A.scan_max[blockIdx.x] = bmax;  // (bmax final: the scan loop's barriers)
}
extern "C" __global__ __launch_bounds__(1024) void mxp_pack_scan2_kernel(mxp_pack_args A, uint32_t nblocks) {
    __shared__ uint64_t carry;
    __shared__ uint32_t lmax;
    if (threadIdx.x == 0) {
        carry = 0;
        lmax = 0u;
    }
    __syncthreads();
    {
        uint32_t m = 0;
        for (uint32_t b = threadIdx.x; b < nblocks; b += MXP_SCAN_B) m = max(m, A.scan_max[b]);
        m = wave_max_u32(m);
        if ((threadIdx.x & 63u) == 0) atomicMax(&lmax, m);
    }
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
    if (threadIdx.x == 0) {
        A.scan[A.ns] = carry;  // total
        if (A.max_len_out) *A.max_len_out = lmax;  // (lmax final: the loop's barriers)
    }
}
// (8 bytes at a time: the destination is 8-aligned, the source is read through ld8_any -- the batch
// blob carries 16 bytes of slack -- and the last word is zero past the string)
extern "C" __global__ __launch_bounds__(256) void mxp_pack_copy_kernel(mxp_pack_args A) {
    for (uint64_t i = gtid(); i < A.ns; i += gstride()) {
        const uint64_t o = A.scan[i] + A.scan_blocks[i / MXP_SCAN_B];
        const uint64_t s0 = A.soff[i], n = A.soff[i + 1] - s0;
        A.bdesc[i] = (o << 24) | n;
        uint64_t* dst = (uint64_t*)(A.bblob + o);
        for (uint64_t k = 0; k < n; k += 8u) {
            const uint64_t r = n - k;
            dst[k / 8u] = ld8_any(A.sbytes + s0 + k) & (r >= 8u ? ~0ull : (1ull << (8u * r)) - 1ull);
        }
    }
}

// Value classes: the class dictionary of every candidate column, in two levels so that no hot key
// meets more than MXP_VTD_MERGE global atomics (a column's few Zipf-hot values would otherwise take
// one probe and one count atomic from every tile).
// Level 1 (grid: tiles of MXP_VTD_TILE requests x candidate columns): the tile's distinct keys in an
// LDS table -- each request adds 1 to its key's count (LDS atomics; a per-wave ballot loop over the
// distinct keys cost ~1,500 scalar instructions per wave on C4) -- then written out as the tile's
// list, from the slots the inserting lanes listed (not a scan of the whole table).
#define MXP_VTD_LCAP 2048u
extern "C" __global__ __launch_bounds__(256) void mxp_pack_vtd_local_kernel(mxp_pack_args A) {
    __shared__ unsigned long long lkey[MXP_VTD_LCAP];
    __shared__ uint32_t lcnt[MXP_VTD_LCAP], lrep[MXP_VTD_LCAP];
    __shared__ uint16_t lslot[MXP_VTD_TILE];  // the occupied slots, in insertion order
    __shared__ uint32_t nins;
    const uint32_t tid = threadIdx.x, a = blockIdx.y, t = blockIdx.x;
    const uint32_t c = A.vt_col[a];
    for (uint32_t i = tid; i < MXP_VTD_LCAP; i += 256u) {
        lkey[i] = ~0ull;
        lcnt[i] = 0u;
    }
    if (tid == 0) nins = 0u;
    __syncthreads();
    const uint64_t base = (uint64_t)t * MXP_VTD_TILE;
#pragma unroll
    for (uint32_t r = 0; r < MXP_VTD_TILE / 256u; r++) {
        const uint64_t req = base + tid + 256u * r;
        if (req >= A.n) continue;
        const unsigned long long key = mxp_vt_key(A.kinds[(uint64_t)c * A.n + req], A.vals[(uint64_t)c * A.n + req]);
        uint32_t h = (uint32_t)mxp_hash64(key) & (MXP_VTD_LCAP - 1u);
        for (;;) {
            const unsigned long long cur = lkey[h];
            if (cur == key) break;
            if (cur == ~0ull) {
                const unsigned long long old = atomicCAS(&lkey[h], ~0ull, key);
                if (old == ~0ull) {
                    lrep[h] = (uint32_t)req;
                    lslot[atomicAdd(&nins, 1u)] = (uint16_t)h;
                    break;
                }
                if (old == key) break;
            }
            h = (h + 1u) & (MXP_VTD_LCAP - 1u);
        }
        atomicAdd(&lcnt[h], 1u);
    }
    __syncthreads();
    const uint64_t lo = ((uint64_t)a * A.vtd_tiles + t) * MXP_VTD_TILE;
    const uint32_t k = nins;
    for (uint32_t i = tid; i < k; i += 256u) {
        const uint32_t h = lslot[i];
        A.vtd_lkey[lo + i] = lkey[h];
        A.vtd_lcr[lo + i] = make_uint2(lcnt[h], lrep[h]);
    }
    if (tid == 0) A.vtd_ln[(uint64_t)a * A.vtd_tiles + t] = k;
}

// Level 2 (grid: MXP_VTD_MERGE x candidate columns): a workgroup merges its share of the tile
// lists in an LDS table (128 KB: one workgroup per CU), then adds its distinct keys to the column's
// provisional table (compare-and-swap; counts added; the first inserter's representative kept) and
// counts the new keys.  Past MXP_VTD_MAXD distinct keys -- in LDS or in the table -- the column is
// marked overflowed and the merge stops (a column of mostly distinct values is no value-class
// column).
extern "C" __global__ __launch_bounds__(256) void mxp_pack_vtd_merge_kernel(mxp_pack_args A) {
    __shared__ unsigned long long tkey[MXP_VTD_CAP];
    __shared__ uint32_t tcnt[MXP_VTD_CAP], trep[MXP_VTD_CAP];
    __shared__ uint32_t tn, over;
    const uint32_t tid = threadIdx.x, a = blockIdx.y;
    uint32_t* meta = A.vtd_meta + 2u * a;
    for (uint32_t i = tid; i < MXP_VTD_CAP; i += 256u) {
        tkey[i] = ~0ull;
        tcnt[i] = 0u;
    }
    if (tid == 0) {
        tn = 0u;
        over = __hip_atomic_load(meta + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const uint32_t per = (A.vtd_tiles + MXP_VTD_MERGE - 1u) / MXP_VTD_MERGE;
    const uint32_t t0 = blockIdx.x * per, t1 = min(t0 + per, A.vtd_tiles);
    for (uint32_t t = t0; t < t1 && !over; t++) {
        const uint64_t lo = ((uint64_t)a * A.vtd_tiles + t) * MXP_VTD_TILE;
        const uint32_t k = A.vtd_ln[(uint64_t)a * A.vtd_tiles + t];
        for (uint32_t e = tid; e < k; e += 256u) {
            const unsigned long long key = A.vtd_lkey[lo + e];
            const uint2 cr = A.vtd_lcr[lo + e];
            uint32_t h = (uint32_t)mxp_hash64(key) & (MXP_VTD_CAP - 1u);
            for (;;) {
                const unsigned long long cur = tkey[h];
                if (cur == key) break;
                if (cur == ~0ull) {
                    const unsigned long long old = atomicCAS(&tkey[h], ~0ull, key);
                    if (old == ~0ull) {
                        trep[h] = cr.y;
                        if (atomicAdd(&tn, 1u) >= MXP_VTD_MAXD) over = 1u;
                        break;
                    }
                    if (old == key) break;
                }
                h = (h + 1u) & (MXP_VTD_CAP - 1u);
            }
            atomicAdd(&tcnt[h], cr.x);
        }
        __syncthreads();  // (over: read by every thread before the next tile)
    }
    if (over) {
        if (tid == 0) __hip_atomic_store(meta + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    unsigned long long* T = A.vtd_tkey + (uint64_t)a * MXP_VTD_CAP;
    uint2* CR = A.vtd_tcr + (uint64_t)a * MXP_VTD_CAP;
    for (uint32_t i = tid; i < MXP_VTD_CAP; i += 256u) {
        const unsigned long long key = tkey[i];
        if (key == ~0ull) continue;
        uint32_t h = (uint32_t)mxp_hash64(key) & (MXP_VTD_CAP - 1u);
        for (;;) {
            unsigned long long old = __hip_atomic_load(T + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == ~0ull) {
                old = atomicCAS(T + h, ~0ull, key);
                if (old == ~0ull) {
                    CR[h].y = trep[i];
                    if (atomicAdd(meta, 1u) >= MXP_VTD_MAXD) __hip_atomic_store(meta + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            if (old == key) break;
            h = (h + 1u) & (MXP_VTD_CAP - 1u);
            if (__hip_atomic_load(meta + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;  // (a full table)
        }
        atomicAdd(&CR[h].x, tcnt[i]);
    }
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
    case 0:
        if (a->ncol) hipLaunchKernelGGL(mxp_pack_mark_kernel, dim3(grid_for(a->n), a->ncol), dim3(256), 0, s, *a);
        break;
    case 1:
        if (a->kind == MXP_IK_STR)
            hipLaunchKernelGGL(mxp_pack_intern_str_kernel, dim3(grid_for(a->i1 - a->i0)), dim3(256), 0, s, *a);
        else
            hipLaunchKernelGGL(mxp_pack_intern_kernel, dim3(grid_for(a->i1 - a->i0)), dim3(256), 0, s, *a);
        break;
    case 2:
        if (a->ncol) hipLaunchKernelGGL(mxp_pack_gather_kernel, dim3(grid_for(a->n), a->ncol), dim3(256), 0, s, *a);
        break;
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
        hipLaunchKernelGGL(mxp_pack_vtd_local_kernel, dim3(a->vtd_tiles, a->n_vt_cand), dim3(256), 0, s, *a);
        hipLaunchKernelGGL(mxp_pack_vtd_merge_kernel, dim3(MXP_VTD_MERGE, a->n_vt_cand), dim3(256), 0, s, *a);
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

// The narrow batch (mxp_batch_upload2): u32 values / offsets as copied, widened to the u64 layout
// the packer reads (zero extension; a grid-stride pass of 16-byte loads and 32-byte stores)
extern "C" __global__ __launch_bounds__(256) void mxp_widen_kernel(const uint32_t* __restrict__ in,
                                                                   uint64_t* __restrict__ out, uint64_t n) {
    const uint64_t n4 = n / 4u;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256ull) {
        const uint4 v = reinterpret_cast<const uint4*>(in)[i];
        reinterpret_cast<ulonglong2*>(out)[2 * i] = make_ulonglong2(v.x, v.y);
        reinterpret_cast<ulonglong2*>(out)[2 * i + 1] = make_ulonglong2(v.z, v.w);
    }
    const uint64_t t = 4 * n4 + blockIdx.x * 256ull + threadIdx.x;
    if (blockIdx.x == 0 && t < n) out[t] = in[t];
}

// in / out: 16-byte aligned device buffers (hipMalloc blocks)
extern "C" hipError_t mxp_launch_widen(const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t g = (n / 4u + 255u) / 256u;
    hipLaunchKernelGGL(mxp_widen_kernel, dim3((uint32_t)(g < 2048u ? (g ? g : 1u) : 2048u)), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}
