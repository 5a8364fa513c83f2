// lists.h -- list-adapter tables and kernel arguments shared by lists.cpp (host compile) and
// lists.hip (gfx950 check kernel).  Reference: mixer/adapter/list/{list,stringList,ipList}.go.
#pragma once

#include <stdint.h>

#include "dfa_dev.h"
#include "netparse.h"

// string hash table slot: hash tag (the hash's top 20 bits) << 44 | entry length << 32 | entry pool
// offset / 8, so a probe reads the entry's bytes with no descriptor load in between; an entry of
// MXP_LIST_LONG bytes or more keeps length MXP_LIST_LONG in the slot and its index into ent_desc in
// the low word.  Empty slot = ~0 (no real slot: lengths stop at MXP_LIST_LONG).
#define MXP_LIST_EMPTY 0xFFFFFFFFFFFFFFFFull
#define MXP_LIST_LONG 0xFFEu
#define MXP_LIST_SLOT(h, len, low) (((uint64_t)(h) >> 44) << 44 | (uint64_t)(len) << 32 | (uint64_t)(low))

// LDS staging of regex-list DFAs: transition words per workgroup (60 KB of the 160 KB of a CU, so
// two 1024-thread workgroups share a CU) and parts staged at most
#define MXP_LDS_DFA_WORDS 15360u
#define MXP_LDS_DFA_PARTS 8u
#define MXP_LIST_RX_THREADS 1024u

typedef struct mxp_list_args {
    uint32_t type;              // MXP_LIST_*
    uint32_t blacklist;
    uint32_t n;                 // symbols
    uint32_t hmask;             // string table size - 1
    const uint8_t* sym;         // symbol blob (>= 16 bytes of slack)
    const uint64_t* sym_off;    // [n + 1]
    const uint64_t* htab;       // string lists: open-addressing slots
    const uint64_t* ent_desc;   // entry offset << 24 | length (8-aligned pool)
    const uint8_t* ent_pool;
    const uint32_t* v4lo;       // IP lists: disjoint sorted IPv4 intervals
    const uint32_t* v4hi;
    const uint64_t* v6lo;       // disjoint sorted IPv6 intervals, [2 i] high / [2 i + 1] low 64 bits
    const uint64_t* v6hi;
    uint32_t n4, n6;
    mxp_dfa_set rx;             // REGEX lists: DFAs / NFAs 0 .. rx_n-1, each the union of a part of the patterns
    int32_t* codes;             // [n] google.rpc codes
    // fused listentry (mxp_listentry_check): symbols are the Eval results of one rule instead of
    // sym / sym_off -- a string id per request (vals[q * vstride], an interface handle when viface),
    // with the rule's error bit err_word[q] & err_bit; ids < n_gstr in the rule set's pool
    const uint64_t* vals;
    const uint32_t* err_word;
    uint32_t err_bit;
    uint32_t vstride;
    uint32_t viface;
    uint32_t rx_n;
    uint64_t n_gstr;
    const uint64_t* gstr_off;   // offset << 24 | length (8-aligned pools, 16 bytes of slack)
    const uint8_t* gstr;
    const uint64_t* bstr_off;
    const uint8_t* bstr;
    // REGEX lists, LDS staging (mxp_list_rx_kernel): parts k < lds_nparts have their first
    // lds_plan[k] transition rows copied to LDS word lds_plan[MXP_LDS_DFA_PARTS + k] (0 rows: the
    // part walks from global memory), plus their ASCII class maps.  (A device table, not a kernarg
    // array: a dynamically indexed by-value argument would be copied to scratch.)
    uint32_t lds_nparts;
    const uint32_t* lds_plan;
    uint32_t rx_nfa;            // REGEX lists with NFA parts: the *_nfa kernel instantiations
    uint32_t ip_split;          // IP lists: mxp_list_ip_kernel (address families in waves of their own)
    const uint32_t* v4dir;      // IP lists: [65537] v4dir[k] = intervals whose start is below k << 16
    uint32_t opt;               // MXP_LIST_OPT_* (A/B knobs, MXP_LIST_OPT; default all on)
    uint32_t pad_opt;
    // REGEX lists, literal-prefix dispatch (mxp_list_rxp_kernel; lists.cpp rxp_build): patterns
    // anchored on a literal prefix are found through a hash table of their prefixes, each checked by a
    // small tail automaton (MXP_RXP_* block) staged in the lane's LDS slot; the other patterns stay in
    // the union parts above
    const uint64_t* rxp_tab;    // slots: tag << 44 | prefix length << 38 | blocks << 32 | first block
    const uint8_t* rxp_blk;     // tail blocks, 16-byte units
    const uint32_t* rxp_lead;   // [MXP_RXP_LEAD] prefix-length masks by the hash of a prefix's first 3 bytes
    uint32_t rxp_mask;          // table slots - 1 (0: no dispatch)
    uint32_t rxp_short;         // prefix-length mask of the prefixes shorter than 3 bytes
} mxp_list_args;

// Tail block of one prefix-dispatched pattern (at most MXP_RXP_BLOCK bytes, 16-byte units):
//   [0] S tail states (0: the prefix alone matches)   [1] C classes (ASCII classes, then HI, END)
//   [2] L prefix length                                [3] the block's 16-byte units
//   [4 .. 4 + MXP_RXP_MAXPRE)   the prefix, zero padded
//   [32 .. 96)                  class of each ASCII byte, one nibble each (low nibble = even byte)
//   [96 .. 96 + S * C)          next state per (state, class): a state, MXP_RXP_ACC or MXP_RXP_REJ
// A byte >= 0x80 takes class C - 2 (HI): from every tail state all non-ASCII runes either reject or
// accept (the block is built only then), so the rune's first byte decides; C - 1 is END of text.
#define MXP_RXP_BLOCK 240u       // a block the LDS variant stages (larger ones it steps from global memory)
#define MXP_RXP_BLOCK_MAX 1024u  // any block (96 header bytes + S x C transition bytes)
#define MXP_RXP_STATES 96u       // tail states (u8 codes below MXP_RXP_ACC)
#define MXP_RXP_ROW 61u   // LDS words per lane (the block and one pad word: an odd stride)
#define MXP_RXP_MAXPRE 28u
#define MXP_RXP_TRANS 96u
#define MXP_RXP_ACC 0xFEu
#define MXP_RXP_REJ 0xFFu
#define MXP_RXP_LEAD 16384u  // (64 KB: ~0.5 leads a bucket at 10k patterns -- one or two probes a lookup)
#define MXP_RXP_THREADS 128u

// bucket of a prefix's first three bytes in rxp_lead
MXP_NHD uint32_t mxp_rxp_lead(uint32_t b0, uint32_t b1, uint32_t b2) {
    return ((b0 | b1 << 8 | b2 << 16) * 2654435761u) >> 18;  // (14 bits: MXP_RXP_LEAD)
}
#define MXP_LIST_OPT_V4REG 1u   // dotted quads of <= 15 bytes parsed from registers (one window load)
#define MXP_LIST_OPT_V4DIR 2u   // the IPv4 search starts from the /16 directory
#define MXP_LIST_OPT_STRREG 4u  // string symbols of <= 64 bytes loaded once into registers
#define MXP_LIST_OPT_RXP_LDS 8u // regex-list tails stepped from a per-lane LDS copy (else from global / L2)
// (ablations of the regex dispatch, results invalid: stop after the prefix-table probe / the header)
#define MXP_LIST_OPT_ABL_PROBE 32u
#define MXP_LIST_OPT_ABL_HDR 64u

// ASCII upper-casing of 8 packed bytes (bytes >= 0x80 untouched): strings.ToUpper of ASCII-only
// strings (any other string takes goupper.h's per-rune stream)
MXP_NHD uint64_t mxp_upper8(uint64_t x) {
    const uint64_t h = x & 0x7F7F7F7F7F7F7F7Full;
    const uint64_t ge_a = h + 0x1F1F1F1F1F1F1F1Full;  // high bit set where byte >= 'a'
    const uint64_t gt_z = h + 0x0505050505050505ull;  // high bit set where byte > 'z'
    const uint64_t lower = ge_a & ~gt_z & ~x & 0x8080808080808080ull;
    return x ^ (lower >> 2);
}

// word-at-a-time string hash; `w` is the next 8 bytes (little-endian, zero beyond the end)
MXP_NHD uint64_t mxp_hash_step(uint64_t h, uint64_t w) {
    h ^= w;
    h *= 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 31);
}
MXP_NHD uint64_t mxp_hash_final(uint64_t h, uint64_t len) {
    h ^= len * 0xC2B2AE3D27D4EB4Full;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}
