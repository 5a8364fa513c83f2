// pack_args.h -- kernel arguments of the device packer (pack.hip, driven by pack_device.cpp).
//
// mxp_batch_upload hands the caller's columnar batch (include/mxp_batch.h) to the device as is --
// the used columns' kinds / values, the batch string table, string-map CSR and timestamps -- and
// the packer turns it into the engine's device columns there: every batch string is interned
// against the rule set's pool (a device hash table keyed by the content hash) or, on a miss,
// deduplicated against the batch's other strings (a CAS-built table; id = G + the representative's
// batch index), byte strings likewise into raw and net.IP-canonical id spaces, timestamps into
// time ids; the columns are then gathered through those id maps, and the per-string ip() /
// timestamp() tables parsed on the device (netparse.h / timeparse.h).  Mirrors the host packer
// (engine.cpp pack_host) id space for id space; only the numbering of batch-local ids differs.
#pragma once

#include <stdint.h>

// interning kinds (item spaces)
enum {
    MXP_IK_STR = 0,    // batch strings [0, ns)
    MXP_IK_RAW = 1,    // byte strings: batch strings [0, ns) used as BYTES, then parsed ip() values [ns, ns + S)
    MXP_IK_CANON = 2,  // net.IP.Equal classes of the same items (4-byte -> v4-mapped 16 bytes)
    MXP_IK_TIME = 3    // batch timestamps [0, nt), then parsed timestamp() values [nt, nt + S)
};

// a rule-set interning pool on the device: entries' content + an open-addressing table of
// (hash >> 32) << 32 | (id + 1), 0 = empty, slot = hash & mask
typedef struct mxp_pool_view {
    const uint64_t* desc;           // offset << 24 | length into blob (strings, bytes, canonical bytes)
    const uint8_t* blob;
    const int64_t* tsec;            // times
    const int32_t* tnsec;
    const unsigned long long* ht;
    uint32_t mask;
    uint32_t n;
} mxp_pool_view;

#define MXP_PACK_MAXCOL 64
#define MXP_PACK_VTCAND 32  // value-class candidate columns sized per upload (engine kVtCandMax)
#define MXP_VTD_TILE 1024u  // requests per tile list of the dictionary's first level
#define MXP_VTD_CAP 8192u   // provisional table slots per candidate column
#define MXP_VTD_MAXD 4096u  // more distinct keys: the column is no value-class column (engine kVtMaxClasses)
#define MXP_VTD_MERGE 16u   // merge workgroups per candidate column

#if defined(__HIPCC__)
#define MXP_PHD __host__ __device__ inline
#else
#define MXP_PHD inline
#endif

// content hash of an interned item (pool tables are built on the host with the same function):
// little-endian 8-byte words, zero beyond the end
MXP_PHD uint64_t mxp_item_hash(const uint8_t* p, uint32_t n) {
    uint64_t h = 0;
    for (uint32_t i = 0; i < n; i += 8) {
        uint64_t w = 0;
        for (uint32_t k = 0; k < 8 && i + k < n; k++) w |= (uint64_t)p[i + k] << (8 * k);
        h ^= w;
        h *= 0x9E3779B97F4A7C15ull;
        h ^= h >> 31;
    }
    h ^= (uint64_t)n * 0xC2B2AE3D27D4EB4Full;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}

// the 12-byte key of a timestamp (seconds, nanoseconds; little-endian)
MXP_PHD void mxp_time_key(int64_t sec, int32_t nsec, uint8_t out[12]) {
    for (int k = 0; k < 8; k++) out[k] = (uint8_t)((uint64_t)sec >> (8 * k));
    for (int k = 0; k < 4; k++) out[8 + k] = (uint8_t)((uint32_t)nsec >> (8 * k));
}

typedef struct mxp_pack_args {
    // the caller's batch, uploaded as given
    const uint8_t* sbytes;          // batch string bytes
    const uint64_t* soff;           // [ns + 1]
    const int64_t* tsec;            // batch timestamps [nt]
    const int32_t* tnsec;
    const uint64_t* moff;           // string maps: [nm + 1] entry offsets
    const uint32_t* mkey;           // [E] key / value batch string indices
    const uint32_t* mval;
    uint32_t ns, nt, nm, n;         // strings, timestamps, maps, requests
    uint64_t n_entries;             // map entries E
    // the rule-set string pool (ids < G): the predicate kernels' own pool
    const uint64_t* gdesc;
    const uint8_t* gblob;
    uint32_t G;
    uint32_t pad0;
    uint64_t S;                     // string id space: G + ns
    // interning (one kind per launch)
    mxp_pool_view pool;
    unsigned long long* btab;       // batch dedup table (0 = empty)
    uint32_t bmask;
    uint32_t kind;
    uint32_t base;                  // id of a batch-local item = base + its representative's index
    uint32_t pad1;
    uint64_t i0, i1;                // item range of the launch
    uint32_t* out;                  // [items] interned ids (by item index)
    // parsed per string id [S]
    uint8_t* pip;                   // 16 bytes each
    uint8_t* pip_ok;
    int64_t* pts_sec;
    int32_t* pts_nsec;
    uint8_t* pts_ok;
    // uses: BYTES values mark their batch strings (1)
    uint8_t* use;
    // id maps (by item index): strings, raw / canonical byte ids, time ids
    const uint32_t* sid;
    const uint32_t* braw;
    const uint32_t* bcan;
    const uint32_t* tid;
    // gather: per engine column its batch column (kinds, values; null = absent), virtual map
    // columns' key ids (~0 for plain columns)
    const uint8_t* ck[MXP_PACK_MAXCOL];
    const uint64_t* cv[MXP_PACK_MAXCOL];
    uint32_t vkey[MXP_PACK_MAXCOL];
    uint32_t ncol;
    uint32_t empty_sid;
    uint8_t* kinds;                 // out [ncol][n]
    uint64_t* vals;
    // string-map CSR out (ids)
    uint32_t* omoff;
    uint32_t* omkey;
    uint32_t* omval;
    // aligned overlay pool of the batch strings (ids G + s)
    uint64_t* bdesc;                // [ns]
    uint8_t* bblob;
    uint64_t* scan;                 // [ns + 1] aligned lengths -> offsets
    uint64_t* scan_blocks;
    // pre-tables by string id [S]
    uint64_t* ipof;
    uint64_t* tsof;
    // value classes, the batch's class dictionary in two levels (pack.hip mxp_pack_vtd_*): per tile of
    // MXP_VTD_TILE requests and candidate column its distinct keys (mxp_vt_key) with counts and a
    // representative request, then per column those lists merged into a provisional table of
    // MXP_VTD_CAP slots -- distinct count and overflow (> MXP_VTD_MAXD keys) read back at the upload's
    // one synchronisation; the final tables are built from it (kernels.hip mxp_vtd_final_kernel)
    unsigned long long* vtd_lkey;   // [ncand][tiles][MXP_VTD_TILE] tile lists: keys
    uint2* vtd_lcr;                 // ... (count, representative)
    uint32_t* vtd_ln;               // [ncand][tiles] list lengths
    unsigned long long* vtd_tkey;   // [ncand][MXP_VTD_CAP] provisional tables (~0: empty)
    uint2* vtd_tcr;                 // ... (count, representative)
    uint32_t* vtd_meta;             // [ncand][2] distinct keys, overflow
    uint32_t vtd_tiles;
    uint32_t vt_col[MXP_PACK_VTCAND];
    uint32_t n_vt_cand;
    uint32_t* max_len_out;          // longest batch string (written by mxp_pack_scan2_kernel)
    uint32_t* scan_max;             // per scan block: its longest string
    // run-time regexp patterns: (batch string | 0x80000000 + engine id, rxof value) pairs scattered
    // by interned id
    const uint32_t* rx_s;
    const uint32_t* rx_v;
    uint32_t n_rx;
    uint32_t* rxof;
} mxp_pack_args;
