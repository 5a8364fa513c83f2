/*
 * mxp_group.h -- device groups: the engine over every GPU of a node behind one handle (C-ABI).
 *
 * A Go Mixer is one process (mixer/cmd/mixs), so the multi-GPU form of the engine lives in the
 * library, not in a launcher: one mxp_group owns one engine (include/mxp.h) per device, replicates
 * the compiled rule set, the resolver configuration, lists and memquota tables on each, evaluates
 * contiguous request shards (a Check request's predicates read only its own bag and
 * the immutable rule set, mixer/pkg/runtime/resolver.go:202-238), and sums the only cross-request
 * state -- the per-rule hit counters that stand for resolve_rules (resolver.go:125-138) and the
 * memquota deltas (mixer/adapter/memquota/memquota.go:43-52) -- with ONE all-reduce per step:
 * ncclAllReduce(ncclSum) over RCCL/xGMI on `hits[R] ++ quota_delta[K]` (int64), communicators from
 * ncclCommInitAll.  RCCL (librccl.so.1) is loaded on first use; when it cannot be loaded or
 * initialised, or a device appears twice in the group, the counters are summed on the host instead
 * (mxp_group_reduce_mode says which).  memquota keys have one owner member each: a key's requests
 * are routed to its owner in arrival order, so its sequence is replayed on one device exactly as
 * memquota.go:118-211 replays it in one process.
 *
 * Calls on one group are serialised by the caller (the Go shim's micro-batcher owns the group);
 * inside a call every member's work is enqueued by a thread of its own.  Member engines are ordinary
 * mxp_engine handles (mxp_group_engine): per-pair error texts, rule texts and values are read there
 * with the member-local request index (mxp_group_locate).
 */
#ifndef MXP_GROUP_H
#define MXP_GROUP_H

#include "mxp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxp_group mxp_group;

/* Flags of mxp_group_create. */
#define MXP_GROUP_HOST_REDUCE 1u  /* sum the counters on the host even when RCCL is available */
#define MXP_GROUP_RCCL_SINGLE 2u  /* a one-member group still runs its (one-rank) RCCL all-reduce */
/* mxp_group_reduce_mode */
#define MXP_REDUCE_NONE 0  /* one member: its counters are the totals, nothing to reduce */
#define MXP_REDUCE_RCCL 1  /* ncclAllReduce over the members' communicators (ncclCommInitAll) */
#define MXP_REDUCE_HOST 2  /* device -> host copies, host sum, host -> device copies */

/* A group over devices[0 .. n) (HIP ordinals; member k = devices[k]; a device may repeat, which
 * forces the host reduction).  mxp_last_error-style text of a failed create or of the group's last
 * failed call: mxp_group_last_error (also when *out is NULL after a failed create: pass NULL). */
int mxp_group_create(const int* devices, uint32_t n, uint32_t flags, mxp_group** out);
void mxp_group_destroy(mxp_group* g);
const char* mxp_group_last_error(const mxp_group* g);
uint32_t mxp_group_size(const mxp_group* g);
int mxp_group_reduce_mode(const mxp_group* g);
/* Member k's engine (owned by the group) and its HIP stream (the stream every group call enqueues
 * member k's work on). */
mxp_engine* mxp_group_engine(mxp_group* g, uint32_t member);
void* mxp_group_stream(mxp_group* g, uint32_t member);
/* Contiguous shard [lo, hi) of member k in a batch of n_total requests split over n members:
 * sizes differ by at most one (istio_amd/dist.py shard_bounds). */
void mxp_group_shard_bounds(uint64_t n_total, uint32_t member, uint32_t n_members, uint64_t* lo, uint64_t* hi);
/* Global request index -> (member, member-local index) of the group's last batch call (upload,
 * resolve, list check).  MXP_ERR_ARG when out of range. */
int mxp_group_locate(const mxp_group* g, uint64_t request, uint32_t* member, uint32_t* local);

/* Configuration, replicated on every member (each compiles on a thread of its own).  Semantics and
 * statuses as mxp_vocab_set / mxp_vocab_set_finder / mxp_ruleset_compile / mxp_resolver_set; a
 * finder is asked on the calling thread only (member 0 compiles first; the others take the
 * vocabulary it found).  A compile resets the group's counters. */
int mxp_group_vocab_set(mxp_group* g, const char* const* names, const int32_t* value_types, uint32_t n);
int mxp_group_vocab_set_finder(mxp_group* g, mxp_attr_finder find, void* ctx);
int mxp_group_ruleset_compile(mxp_group* g, const char* const* exprs, uint32_t n, int32_t* status);
int mxp_group_resolver_set(mxp_group* g, const char* identity_attr, const char* default_ns,
                           const char* const* rule_ns, const uint32_t* variety_mask, const uint8_t* is_tcp,
                           const uint8_t* empty_match, uint32_t n);

/*
 * Device-resident shards.  mxp_group_upload: shards[k] (member k's requests, packed by the caller --
 * e.g. one packing arena per device goroutine) uploaded to member k as mxp_batch_upload_ex does
 * (flags: MXP_UPLOAD_NO_WAIT), all members at once; n_shards = mxp_group_size.
 * mxp_group_upload_split: the same from ONE host batch, split into contiguous shards
 * (mxp_group_shard_bounds) whose columns point into the caller's arrays; every shard carries the
 * whole string / time / map tables, so each device receives all of them -- a binding that packs per
 * device sends less.
 */
typedef struct mxp_gbatch mxp_gbatch;
int mxp_group_upload(mxp_group* g, const mxp_bag_batch* const* shards, uint32_t n_shards, uint32_t flags,
                     mxp_gbatch** out);
/* ... of narrow shards (mxp_bag_batch2, mxp_batch_upload2 per member): a third fewer bytes over the
 * hosts' links.  mxp_group_resolve_uploaded then takes shards = NULL. */
int mxp_group_upload2(mxp_group* g, const mxp_bag_batch2* const* shards, uint32_t n_shards, uint32_t flags,
                      mxp_gbatch** out);
int mxp_group_upload_split(mxp_group* g, const mxp_bag_batch* batch, uint32_t flags, mxp_gbatch** out);
int mxp_group_batch_wait_copied(mxp_gbatch* gb);
void mxp_group_batch_free(mxp_group* g, mxp_gbatch* gb);
uint32_t mxp_group_batch_requests(const mxp_gbatch* gb, uint32_t member);

/*
 * One evaluation step of the group: every member evaluates its shard against the replicated rule set
 * (mxp_batch_eval_device_compact semantics; MXP_GROUP_EVAL_ERR_BITMAP: the full error bitmap as
 * mxp_batch_eval_device_hits writes it) into group-owned device buffers -- the match bitmap
 * (rule-word-major over the shard), per-request error flags or the error bitmap -- with the hit
 * counters fused into the step's hits[R].  Enqueued, nothing synchronised.  The results stay until
 * the next evaluation; mxp_group_download brings member k's back.
 */
#define MXP_GROUP_EVAL_ERR_BITMAP 1u
int mxp_group_eval(mxp_group* g, mxp_gbatch* gb, uint32_t flags);
/* match_bits: u32[ceil(R / 32)][n_k]; err_bits (error-bitmap evaluations) u32[ceil(R / 32)][n_k];
 * req_err (compact evaluations) u8[n_k]; any may be NULL.  Waits for member k's work. */
int mxp_group_download(mxp_group* g, uint32_t member, uint32_t* match_bits, uint32_t* err_bits, uint8_t* req_err);

/*
 * memquota across the group.  Every member holds the key table; owner[key] (NULL: key % members,
 * mxp_group_key_owners for load-balanced owners) is the member that replays the key's requests.
 * mxp_group_quota_upload routes n requests given in arrival order to their keys' owners (a stable
 * partition: each owner receives its keys' requests in arrival order) into device memory;
 * mxp_group_quota_eval enqueues each owner's batched HandleQuota (mxp_quota_alloc_device) at now_ns,
 * beside the evaluation on a second stream per member, with the per-key granted deltas accumulated
 * into the step's quota_delta[K]; mxp_group_quota_granted waits and writes QuotaResult.Amount per
 * request in the caller's order.  mxp_group_quota_alloc = upload + eval + granted.  The group's
 * counters carry the deltas of its most recently created quota table.
 */
typedef struct mxp_gquota mxp_gquota;
typedef struct mxp_gqbatch mxp_gqbatch;
int mxp_group_quota_create(mxp_group* g, uint32_t n_keys, const int64_t* max_amount, const int64_t* valid_duration_ns,
                           const uint32_t* owner, mxp_gquota** out);
void mxp_group_quota_destroy(mxp_group* g, mxp_gquota* q);
int mxp_group_quota_upload(mxp_group* g, mxp_gquota* q, uint32_t n, const uint32_t* key, const int64_t* amount,
                           const uint8_t* best_effort, mxp_gqbatch** out);
int mxp_group_quota_eval(mxp_group* g, mxp_gquota* q, mxp_gqbatch* qb, int64_t now_ns);
int mxp_group_quota_granted(mxp_group* g, mxp_gqbatch* qb, int64_t* granted);
void mxp_group_quota_batch_free(mxp_group* g, mxp_gqbatch* qb);
uint32_t mxp_group_quota_batch_requests(const mxp_gqbatch* qb, uint32_t member);
int mxp_group_quota_alloc(mxp_group* g, mxp_gquota* q, uint32_t n, const uint32_t* key, const int64_t* amount,
                          const uint8_t* best_effort, int64_t now_ns, int64_t* granted);
/* Owner of each of n_keys keys among n_members by expected load: longest-processing-time first over
 * weights (e.g. the last snapshot's per-key request counts), heaviest key first (ties by key id), each
 * to the least-loaded member (ties by member index).  Host only. */
int mxp_group_key_owners(const double* weights, uint32_t n_keys, uint32_t n_members, uint32_t* owner);

/*
 * Counters: step buffers hits[R] ++ quota_delta[K] (int64) per member, accumulated by
 * mxp_group_eval / mxp_group_quota_eval; mxp_group_reduce enqueues the step's one all-reduce and adds
 * the sums into the running totals (the step buffers are zeroed for the next step).
 * mxp_group_counters waits and reads the totals (hits: u64[R], quota_delta: i64[K]; either may be
 * NULL); mxp_group_counters_reset zeroes both.  mxp_group_sync waits for every member's work.
 */
int mxp_group_reduce(mxp_group* g);
int mxp_group_counters(mxp_group* g, uint64_t* hits, int64_t* quota_delta);
int mxp_group_counters_reset(mxp_group* g);
int mxp_group_sync(mxp_group* g);

/*
 * Batched Resolve over the group (mxp_resolve_batch_ex per member, all at once): request q of the
 * concatenated shards (shards[k] holds requests [lo_k, lo_k + n_k) in order) gets status[q],
 * err_rule[q] and its selected rules sel_rules[sel_off[q] .. sel_off[q + 1]) exactly as one engine
 * resolving the whole batch would return them; MXP_ERR_NOMEM when sel_cap is short, with status,
 * err_rule and sel_off complete.  Error texts: mxp_group_pair_error with the global request index.
 * mxp_group_resolve_split: from one host batch, split as mxp_group_upload_split.
 */
int mxp_group_resolve_batch(mxp_group* g, const mxp_bag_batch* const* shards, uint32_t n_shards, uint32_t variety,
                            uint32_t flags, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                            uint64_t sel_cap);
/* ... over shards uploaded before (mxp_group_upload, e.g. MXP_UPLOAD_NO_WAIT one call ahead: the next
 * batch's copies and packing overlap this one's Resolve on every member); shards = the host shards gb
 * was uploaded from, unchanged.  Takes gb over, whatever it returns (mxp_resolve_uploaded). */
int mxp_group_resolve_uploaded(mxp_group* g, mxp_gbatch* gb, const mxp_bag_batch* const* shards, uint32_t n_shards,
                               uint32_t variety, uint32_t flags, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                               void* sel_rules, uint64_t sel_cap);
/* mxp_group_resolve_uploaded in two calls (mxp_resolve_submit / mxp_resolve_finish on every member):
 * submit enqueues every member's evaluation and returns; between the two the caller may upload the
 * next batch (mxp_group_upload / _upload2, MXP_UPLOAD_NO_WAIT) and make no other group call; finish
 * resolves into the whole batch's arrays.  submit takes gb over; after a successful submit, finish
 * is called once. */
typedef struct mxp_gresolve mxp_gresolve;
int mxp_group_resolve_submit(mxp_group* g, mxp_gbatch* gb, const mxp_bag_batch* const* shards, uint32_t n_shards,
                             uint32_t variety, uint32_t flags, mxp_gresolve** out);
int mxp_group_resolve_finish(mxp_group* g, mxp_gresolve* r, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                             void* sel_rules, uint64_t sel_cap);
int mxp_group_resolve_split(mxp_group* g, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags, uint8_t* status,
                            uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap);
int mxp_group_pair_error(mxp_group* g, uint64_t request, uint32_t rule, char* buf, uint32_t cap);

/*
 * Lists replicated on every member; mxp_group_list_check splits n symbols (blob + offsets as
 * mxp_list_check) into contiguous shards checked on all members at once.  mxp_group_list_member:
 * member k's mxp_list, for mxp_list_check_device on device-resident symbols.
 */
typedef struct mxp_glist mxp_glist;
int mxp_group_list_create(mxp_group* g, int entry_type, const char* const* entries, const uint32_t* entry_lens,
                          uint32_t n_entries, const char* const* overrides, const uint32_t* override_lens,
                          uint32_t n_overrides, mxp_glist** out);
void mxp_group_list_destroy(mxp_group* g, mxp_glist* l);
mxp_list* mxp_group_list_member(mxp_glist* l, uint32_t member);
int mxp_group_list_check(mxp_group* g, const mxp_glist* l, int blacklist, const uint8_t* sym_bytes,
                         const uint64_t* sym_offsets, uint32_t n, int32_t* codes);
/* Device-resident lookups: member k checks its own n[k] symbols (d_sym_bytes[k] / d_sym_offsets[k] in
 * member k's device memory, as mxp_list_check_device) into d_codes[k], enqueued on member k's stream
 * (mxp_group_stream); nothing synchronised. */
int mxp_group_list_check_device(mxp_group* g, const mxp_glist* l, int blacklist, const uint8_t* const* d_sym_bytes,
                                const uint64_t* const* d_sym_offsets, const uint32_t* n, int32_t* const* d_codes);

#ifdef __cplusplus
}
#endif

#endif /* MXP_GROUP_H */
