// resolve_args.h -- argument block of the batched-resolver kernels (resolve.hip).
#pragma once

#include <stdint.h>

#include "../../include/mxp.h"

#define MXP_NS_NONE 0x7FFFFFFDu      // namespace without rules (with the tcp bit it stays distinct from the two codes below)
#define MXP_NS_MISSING 0xFFFFFFFFu   // identity attribute absent
#define MXP_NS_NOTSTRING 0xFFFFFFFEu // identity attribute not a string

// destAndNamespace (resolver.go:180-199) + the tcp flag of filterActions (:208) on the device, per
// request, from the batch as uploaded (pack_device.cpp scratch: raw kinds / values of the identity
// and context.protocol columns, raw batch strings) and the configuration's namespace names
typedef struct mxp_ns_args {
    uint32_t n;
    uint32_t ns_mask;          // namespace table size - 1
    const uint8_t* id_kind;    // [n] identity column (nullptr: absent from the batch)
    const uint64_t* id_val;
    const uint8_t* pr_kind;    // [n] context.protocol column (nullptr: absent)
    const uint64_t* pr_val;
    const uint64_t* soff;      // raw batch strings (offsets [ns + 1], bytes with 16 B of slack)
    const uint8_t* sbytes;
    const unsigned long long* ns_tab;  // open addressing: hash hi 32 << 32 | namespace id + 1 (0: empty)
    const uint64_t* ns_desc;   // [namespaces] offset << 24 | length into ns_blob
    const uint8_t* ns_blob;
    uint32_t* nsinfo;          // [n] out: namespace id | tcp << 31, MXP_NS_NONE / MISSING / NOTSTRING
} mxp_ns_args;

#define MXP_RES_SCAN_TILE 256u  // requests per block of the count kernel's block sums

typedef struct mxp_resolve_args {
    uint32_t n;                // requests
    uint32_t n_words;          // ceil(rules / 32)
    const uint32_t* nsinfo;    // [n] namespace id | tcp << 31, or MXP_NS_MISSING / MXP_NS_NOTSTRING
    const uint32_t* ns_lo;     // rule range of each namespace
    const uint32_t* ns_hi;
    uint32_t default_id;       // namespace id of the default config namespace (MXP_NS_NONE: no rules)
    uint32_t pad;
    const uint32_t* amask;     // [2][n_words] rules with an action for the variety, per request tcp flag
    const uint32_t* empty;     // [n_words] rules with an empty match (selected without evaluation)
    const uint32_t* match;     // [n_words][n] predicate bitmaps of the batch
    const uint32_t* err;
    uint8_t* status;           // [n] MXP_RESOLVE_*
    uint32_t* err_rule;        // [n] first erroring rule (MXP_RESOLVE_PRED_ERROR)
    uint32_t* count;           // [n] selected rules
    const uint64_t* sel_off;   // [n + 1] exclusive scan of count (pass 2)
    uint32_t* sel_rules;       // selected rule ids, request by request, in resolution order
    // compact mode (resolver.cpp): no error bitmap -- err_in[q] is the request's first applicable
    // erroring rule in resolution order (~0: none), found from the error records; the count pass
    // also writes per-block sums for the device scan of the counts into sel_off
    const uint32_t* err_in;
    uint64_t* block_sum;       // [ceil(n / MXP_RES_SCAN_TILE)]
    uint64_t* sel_off_out;     // [n + 1] (scan pass)
    uint32_t ids16;            // pass 2 writes u16 rule ids (sel_rules as uint16_t*)
    uint32_t err_rank;         // err_in holds resolution ranks (mxp_resolve_first_err_kernel), not rules
    uint4* stash;              // [n] the count pass's first 4 selected rules of each request (pass 2
                               // copies them for requests with at most 4, instead of walking the
                               // bitmap again); nullptr: none
    // pair Resolve (resolver.cpp): the evaluation's deferred index pairs, filed per fill chunk and
    // lane quad by mxp_dtp_sort_kernel, read instead of the match bitmap, which the evaluation then
    // never wrote (kargs.dtp_lazy); every word of the rule set is a plain fill chunk's
    const uint16_t* pr_slots;  // [chunks][pr_row quads][8] g << 8 | plane << 7 | request % 4 << 5 | bit
    const uint8_t* pr_qn;      // [chunks][pr_row] entries in each quad's slots (<= 8)
    const uint32_t* pr_fills;  // [chunks][8] the fill chunks (vm.h mxp_fill: [2] first word, [3] words)
    uint64_t pr_row;           // quads per chunk row (MXP_DTP_ROW of the evaluation's tiles)
    uint32_t pr_nch;           // chunks, in ascending word order
    uint32_t pr_pad;
    // the write passes write nothing when the batch's ids exceed this many (sel_off[n] > sel_cap_dev;
    // 0: unchecked) -- the ids enqueued with the other outputs before the host knows their count
    uint64_t sel_cap_dev;
} mxp_resolve_args;
