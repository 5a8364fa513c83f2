// quota_args.h -- argument block of the batched memquota kernel (quota.hip / quota.cpp).
#pragma once

#include <stdint.h>

typedef struct mxp_quota_args {
    uint32_t n;                  // requests
    uint32_t n_keys;
    int64_t tick;                // currentTick of the batch (now / 100 ms)
    // requests
    const uint32_t* key;
    const int64_t* amount;       // QuotaArgs.QuotaAmount (> 0 alloc, < 0 free)
    const uint8_t* best_effort;
    const uint32_t* order;       // arrival indices sorted by key (stable)
    const uint32_t* seg_start;   // [n_keys + 1] key k's requests: order[seg_start[k] .. seg_start[k+1])
    const uint32_t* skeys;       // [n] the sorted (clamped) key ids
    int64_t* samt;               // [n] amounts in sorted order (mxp_quota_gather)
    uint8_t* sbe;                // [n] best-effort flags in sorted order
    int64_t* granted;            // QuotaResult.Amount per request
    int64_t* delta;              // optional [n_keys] += granted allocs - frees
    // per-key state (HBM, persistent across batches)
    const int64_t* max_amount;
    const uint32_t* ticks;       // window length in ticks; 0 = non-expiring cell
    int64_t* cells;              // in-use amount of non-expiring cells
    int64_t* avail;              // rolling windows: available units
    uint32_t* win_cur;           // current slot
    int64_t* win_tick;           // tick of the current slot
    const uint64_t* slot_off;    // first slot of each window
    int64_t* slots;
    // long keys cut into pieces (mxp_quota_kernel)
    uint32_t* big;               // [n_keys + 1] keys holding amounts past +-2^55 (set by mxp_quota_gather)
    int64_t* prec;               // [6 * (n_keys + 1 + mxp_quota_piece_waves(n))] piece records
    uint32_t* done;              // [n_keys + 1] pieces finished (0 between batches)
    int64_t* prof;               // optional [4 * waves] (debug, MXP_QUOTA_PROF): ticks, run steps, clocks
} mxp_quota_args;
