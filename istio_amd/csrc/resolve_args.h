// resolve_args.h -- argument block of the batched-resolver kernels (resolve.hip).
#pragma once

#include <stdint.h>

#include "../../include/mxp.h"

#define MXP_NS_NONE 0x7FFFFFFDu      // namespace without rules (with the tcp bit it stays distinct from the two codes below)
#define MXP_NS_MISSING 0xFFFFFFFFu   // identity attribute absent
#define MXP_NS_NOTSTRING 0xFFFFFFFEu // identity attribute not a string

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
} mxp_resolve_args;
