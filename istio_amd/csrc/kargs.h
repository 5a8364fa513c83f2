// kargs.h -- argument block of the evaluation kernel (passed by value, lives in the kernarg segment).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

#include "vm.h"

#define MXP_QSTRIDE 32  // u32 stride between sub-queue counters (one 128-byte line each)

typedef struct mxp_kargs {
    // rule set (uploaded once per config snapshot)
    const mxp_vm_ins* prog;      // all rules' programs, concatenated
    const uint32_t* rule_off;    // [n_rules + 1]
    const mxp_guard* guards;     // [n_rules] leading-atom guards (vmopt.h)
    const mxp_group* groups;     // [n_words] per-group guard masks
    const mxp_seg* segs;         // column segments of the groups
    const uint64_t* gk;          // [n_words * 32] guard constants (0 for unguarded slots)
    const uint32_t* tqmask;      // per-group template masks (mxp_group.tq0 / ntq)
    const mxp_tmpl* tmpls;       // continuation templates
    const uint32_t* rule_tmpl;   // [n_rules] template of the rule's continuation (~0: none)
    const uint64_t* rconst;      // [n_rules][MXP_VM_MAXREG] per-rule template constants
    uint32_t n_rules;
    uint32_t n_words;            // ceil(n_rules / 32)
    uint32_t groups_per_wave;
    uint32_t n;                  // requests in the batch
    // columns: [n_cols][n] kinds / values (resolve columns, then virtual map[key] columns)
    const uint8_t* kinds;
    const uint64_t* vals;
    // interned strings: ids < n_gstr live in the rule set's pool, the rest in the batch pool
    uint64_t n_gstr;
    const uint64_t* gstr_off;
    const uint8_t* gstr;
    const uint64_t* bstr_off;
    const uint8_t* bstr;
    uint32_t empty_sid;
    uint32_t pad0;
    // per-request string maps (CSR over batch map ids)
    const uint32_t* map_off;
    const uint32_t* map_keys;
    const uint32_t* map_vals;
    // per-string pre-tables (ip(), timestamp()); ~0 = conversion error
    const uint64_t* ipof;
    const uint64_t* tsof;
    // outputs
    uint32_t* out_match;         // [n_words][n]
    uint32_t* out_err;           // [n_words][n]
    uint64_t* out_vals;          // optional [n][n_rules] result registers (Eval)
    mxp_err_rec* errlog;
    uint32_t* errcount;
    uint32_t errcap;
    uint32_t flags;              // debug / ablation: 1 = skip phase 2 (VM), 2 = no guards
    // pair queue (phase 1 -> mxp_queue_kernel); queue == nullptr disables the hand-off.  The queue
    // is split into qsub sub-queues (tile t appends to sub-queue t % qsub) so the append counters
    // do not serialise on one address.
    uint2* queue;                // [qsub][qsubcap] (request, rule)
    uint32_t* qcount;            // [qsub * MXP_QSTRIDE] appended pairs (may exceed qsubcap: the excess ran in-wave)
    uint32_t qsub;
    uint32_t qsubcap;
    uint32_t dense_min;          // survivors per tile from which a rule stays in-wave
    uint32_t pad1;
} mxp_kargs;
