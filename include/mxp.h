/*
 * mxp.h -- C-ABI of the MI355X-native batched policy engine for Istio Mixer's Check path.
 *
 * The engine replaces, for batches of requests, the per-request / per-rule Go call chain
 *
 *   runtime.Resolver.Resolve(bag, variety)            mixer/pkg/runtime/resolver.go:110
 *     filterActions -> expr.Evaluator.EvalPredicate    resolver.go:202-238, mixer/pkg/expr/evaluator.go:25-31
 *       evaluator.IL.EvalPredicate                     mixer/pkg/il/evaluator/evaluator.go:75
 *         compiler.Compile + interpreter.Interpreter   mixer/pkg/il/compiler/compiler.go:125,
 *                                                      mixer/pkg/il/interpreter/interpreterRun.go:18
 *
 * and is meant to be bound from the reference's Go code through cgo.  All
 * entry points take plain pointers and sizes, return an int status (0 = MXP_OK) and never throw.
 * Output arrays are caller-owned.  One engine = one GPU + one HIP stream; calls on one engine must
 * be serialised by the caller (the Go shim owns one goroutine per device stream).
 */
#ifndef MXP_H
#define MXP_H

#include <stddef.h>
#include <stdint.h>

#include "mxp_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MXP_OK 0
#define MXP_ERR_ARG 1       /* bad argument */
#define MXP_ERR_STATE 2     /* call out of order (e.g. eval before a rule set exists) */
#define MXP_ERR_DEVICE 3    /* HIP runtime error; mxp_last_error() has the text */
#define MXP_ERR_NOMEM 4

typedef struct mxp_engine mxp_engine;
typedef struct mxp_dbatch mxp_dbatch;  /* a device-resident batch (mxp_batch_upload) */

/* Engine lifetime.  device = HIP device ordinal; device = -1 creates a host-only engine that can
 * compile and inspect rule sets (IL text, VM listing) but not evaluate. */
int mxp_engine_create(int device, mxp_engine** out);
void mxp_engine_destroy(mxp_engine* eng);
const char* mxp_last_error(const mxp_engine* eng);

/*
 * Vocabulary (attribute manifest): names + ValueType enum values of istio.io/api
 * mixer/v1/config/descriptor (STRING=1, INT64=2, DOUBLE=3, BOOL=4, TIMESTAMP=5, IP_ADDRESS=6,
 * EMAIL_ADDRESS=7, URI=8, DNS_NAME=9, DURATION=10, STRING_MAP=11).
 * Replaces evaluator.IL.ChangeVocabulary (mixer/pkg/il/evaluator/evaluator.go:107); invalidates the
 * current rule set.
 */
int mxp_vocab_set(mxp_engine* eng, const char* const* names, const int32_t* value_types, uint32_t n);

/*
 * Vocabulary as a finder: the expr.AttributeDescriptorFinder of
 * runtime.VocabularyChangeListener.ChangeVocabulary(finder) (mixer/pkg/runtime/controller.go:100-102,
 * finder.go:45-47).  The engine calls find(ctx, name) for each attribute name its rules use, the
 * first time it meets the name after this call (at mxp_ruleset_compile / mxp_resolver_set);
 * find returns the name's ValueType, or -1 when GetAttribute returns nil.  Names get vocabulary
 * positions in the order they are found (mxp_vocab_name).  Invalidates the current rule set; find
 * must stay callable until the next mxp_vocab_set / mxp_vocab_set_finder.
 */
typedef int32_t (*mxp_attr_finder)(void* ctx, const char* name);
int mxp_vocab_set_finder(mxp_engine* eng, mxp_attr_finder find, void* ctx);

/* Name of vocabulary position `pos` (mxp_attr_ref.attr), NUL-terminated into buf. */
int mxp_vocab_name(mxp_engine* eng, uint32_t pos, char* buf, uint32_t cap);

/*
 * Compile a rule set: n predicate expressions (rule i = exprs[i]) compiled with the reference's
 * compiler (compiler.Compile, compiler.go:125) and lowered to the GPU bytecode; uploaded once.
 * status[i] (optional) receives one of MXP_RULE_*.
 */
#define MXP_RULE_OK 0
#define MXP_RULE_PARSE_ERROR 1     /* expr.Parse failed: the resolver drops such rules (controller.go:406-410) */
#define MXP_RULE_TYPE_ERROR 2      /* type check failed: every evaluation returns this error */
#define MXP_RULE_COMPILE_ERROR 3   /* code generation failed: every evaluation returns this error */
#define MXP_RULE_COMPILE_PANIC 4   /* the reference panics while compiling */
#define MXP_RULE_UNSUPPORTED 5     /* valid rule this build cannot lower yet (evaluations report it) */
int mxp_ruleset_compile(mxp_engine* eng, const char* const* exprs, uint32_t n, int32_t* status);
/* Text of rule i's compile error / IL (text.WriteText, mixer/pkg/il/text/write.go:26) / VM listing. */
int mxp_rule_error(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap);
int mxp_rule_il_text(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap);
int mxp_rule_vm_text(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap);
/* ValueType of rule i's expression (Expression.EvalType) and its il.Type return type. */
int mxp_rule_types(mxp_engine* eng, uint32_t rule, int32_t* value_type, int32_t* il_type);

/*
 * Evaluate every rule against every bag of the batch (EvalPredicate semantics for each pair).
 * Output bitmaps are rule-word-major: bit (r % 32) of word [(r / 32) * n_requests + q] describes
 * (request q, rule r).  match_bits: predicate true.  err_bits: evaluation error or Go panic.
 * Either pointer may be NULL.  Error details of the last batch: mxp_pair_error.
 */
int mxp_eval_batch(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t* match_bits, uint32_t* err_bits);

/*
 * Referenced attributes (the precondition cache key of a Check response): for every request, the
 * attribute reads EvalPredicate of every rule performs on its bag -- ProtoBag.Get / StringMap.Get
 * tracking (mixer/pkg/attribute/protoBag.go:78-159), the set grpcServer.Check returns as
 * ReferencedAttributes (mixer/pkg/api/grpcServer.go:177).  Short-circuiting makes it path
 * dependent; the engine records the reads its VM performs and adds the reads its guard and index
 * phases stand for.
 *   attr  position of the attribute in the mxp_vocab_set names (mxp_vocab_name);
 *   key   MXP_REF_NOKEY for an attribute reference, else the string id of the map key
 *         (StringMap.Get; text with mxp_string_text while this batch is the engine's last);
 *   cond  MXP_REF_ABSENCE / MXP_REF_EXACT (mixer/v1 ReferencedAttributes.Condition), or MXP_REF_MAP
 *         for a string map fetched whole: the test FakeBag lists its name (fakebag.go:54-60), a
 *         ProtoBag does not record it (protoBag.go:109-112) -- a cgo shim drops these entries.
 * Per request the entries are sorted by (attr, key) and distinct.  ref_off has n_requests + 1
 * entries; when cap is too small MXP_ERR_NOMEM is returned with ref_off complete (retry with
 * ref_off[n]).  match_bits / err_bits as mxp_eval_batch (may be NULL).  MXP_ERR_STATE when a rule is
 * MXP_RULE_UNSUPPORTED (its reads are unknown).  destination.* -> target.* fallbacks (compatBag,
 * grpcServer.go:93-107) happen while packing, in the caller, and are expanded there.
 */
#define MXP_REF_NOKEY 0xFFFFFFFFu
#define MXP_REF_ABSENCE 1u
#define MXP_REF_EXACT 2u
#define MXP_REF_MAP 16u
typedef struct mxp_attr_ref {
    uint32_t attr;
    uint32_t key;
    uint32_t cond;
    uint32_t pad;
} mxp_attr_ref;
int mxp_eval_refs(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t* match_bits, uint32_t* err_bits,
                  uint64_t* ref_off, mxp_attr_ref* refs, uint64_t cap);
/* Text of an engine string id of the last evaluated batch (map keys of mxp_eval_refs). */
int mxp_string_text(mxp_engine* eng, uint32_t sid, char* buf, uint32_t cap);

/*
 * Eval (expr.Evaluator.Eval) for small batches: raw result register per pair, [n_requests][n_rules],
 * plus per-pair code (0 false/ok, 1 true, 2 error, 3 panic).  Decode with mxp_value_text.
 */
int mxp_eval_values(mxp_engine* eng, const mxp_bag_batch* batch, uint64_t* values, uint8_t* codes);
/* Render a result register of rule `rule` as Go would print it with %v (strings raw). */
int mxp_value_text(mxp_engine* eng, uint32_t rule, uint64_t value, char* buf, uint32_t cap);
/* Result kind of a value register: MXP_STRING, MXP_INT64, ... (interface values report their kind). */
int mxp_value_kind(mxp_engine* eng, uint32_t rule, uint64_t value);
/*
 * A result register of the last batch as the Go value interpreter.Result.AsInterface returns
 * (mixer/pkg/il/interpreter/result.go): kind (MXP_*) and
 *   MXP_BOOL / MXP_INT64 / MXP_DURATION   i
 *   MXP_DOUBLE                            d
 *   MXP_TIMESTAMP                         i = Unix seconds, nsec
 *   MXP_STRING / MXP_BYTES                the bytes in buf[0 .. n)
 *   MXP_STRING_MAP                        i entries in buf[0 .. n): u32 key length, key, u32 value
 *                                         length, value (little endian) per entry
 * MXP_ERR_NOMEM when n > cap (n is set: call again with room).
 */
typedef struct mxp_value {
    uint32_t kind;
    uint32_t n;
    int64_t i;
    double d;
    int32_t nsec;
    uint32_t pad;
} mxp_value;
int mxp_value_decode(mxp_engine* eng, uint32_t rule, uint64_t value, mxp_value* out, uint8_t* buf, uint32_t cap);

/* Error text of pair (request, rule) from the last evaluated batch, as the reference would report it.
 * Returns MXP_OK with buf = "" if the pair did not fail, 1 if it failed with a panic. */
int mxp_pair_error(mxp_engine* eng, uint32_t request, uint32_t rule, char* buf, uint32_t cap);
/* Number of error pairs of the last batch (may exceed the log capacity). */
uint64_t mxp_error_count(mxp_engine* eng);

/*
 * Batched runtime.resolver (mixer/pkg/runtime/resolver.go:110-238).
 *
 * mxp_resolver_set configures resolution for the compiled rule set (call after mxp_ruleset_compile;
 * a new compile clears it).  Per rule: its config namespace, the varieties it has actions for (bit v
 * = adptTmpl.TemplateVariety v), whether it is a TCP rule (rule.rtype.IsTCP()), and whether its
 * match is empty (selected without evaluation).  Rules of one namespace must be contiguous and in
 * the reference's resolution order (the order of the namespace's rule slice); MXP_ERR_ARG otherwise.
 * identity_attr names the destination attribute (`destination.service`), default_ns the config
 * default namespace.
 *
 * mxp_resolve_batch evaluates every rule against every bag and resolves each request for `variety`:
 *   status[q]   MXP_RESOLVE_OK, or the reason Resolve returns an error:
 *               NO_IDENTITY / BAD_IDENTITY  (destAndNamespace, resolver.go:180-199),
 *               PRED_ERROR  (first predicate error in resolution order, resolver.go:226-228):
 *               err_rule[q] is that rule, mxp_pair_error(q, err_rule[q]) its error text;
 *   sel_off[q] .. sel_off[q+1]  the selected rules, in resolution order (sel_off has n+1 entries);
 *   sel_rules   capacity sel_cap entries; when too small, MXP_ERR_NOMEM is returned with status,
 *               err_rule and sel_off complete, so the caller can retry with sel_off[n].
 */
#define MXP_RESOLVE_OK 0
#define MXP_RESOLVE_NO_IDENTITY 1
#define MXP_RESOLVE_BAD_IDENTITY 2
#define MXP_RESOLVE_PRED_ERROR 3
int mxp_resolver_set(mxp_engine* eng, const char* identity_attr, const char* default_ns,
                     const char* const* rule_ns, const uint32_t* variety_mask, const uint8_t* is_tcp,
                     const uint8_t* empty_match, uint32_t n);
int mxp_resolve_batch(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                      uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap);
/* mxp_resolve_batch with options: flags MXP_RESOLVE_IDS_U16 writes the selected rule ids as uint16_t
 * (rule sets of at most 65536 rules; MXP_ERR_ARG otherwise): half the bytes of the action lists
 * brought back.  sel_rules has room for sel_cap ids of that width. */
#define MXP_RESOLVE_IDS_U16 1u
int mxp_resolve_batch_ex(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                         uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap);
/* mxp_resolve_batch_ex over a batch uploaded before (mxp_batch_upload / mxp_batch_upload_ex, e.g. with
 * MXP_UPLOAD_NO_WAIT one call ahead, so that batch k + 1's copies and device packing overlap batch
 * k's Resolve -- the Go micro-batcher's double buffering).  `batch` is the host batch db was
 * uploaded from, unchanged (error texts and host passes read it; NULL for a batch uploaded narrow,
 * mxp_batch_upload2).  The call takes db over, whatever
 * it returns: the engine keeps it as the last batch (mxp_pair_error) and recycles it with the next
 * one; the caller does not mxp_batch_free it. */
int mxp_resolve_uploaded(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                         uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap);
/* mxp_resolve_uploaded in two calls.  mxp_resolve_submit enqueues the batch's evaluation and request
 * namespaces and returns without waiting for the device; mxp_resolve_finish waits for them, resolves
 * and downloads (mxp_resolve_uploaded's outputs and errors).  Between the two the caller may upload
 * the next batch on the same engine (mxp_batch_upload_ex / mxp_batch_upload2, MXP_UPLOAD_NO_WAIT):
 * its host checks and packing then overlap this evaluation on the device -- the single-threaded
 * micro-batcher's pipeline -- and makes no other call on the engine.  submit takes db over whatever
 * it returns; after a successful submit, finish is called once (it frees the job, whatever it
 * returns). */
typedef struct mxp_resolve_job mxp_resolve_job;
int mxp_resolve_submit(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                       mxp_resolve_job** out);
int mxp_resolve_finish(mxp_resolve_job* job, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                       uint64_t sel_cap);
/* mxp_resolve_batch plus each Resolve's referenced attributes (mxp_attr_ref, as mxp_eval_refs): the
 * identity attribute; when it is a string, context.protocol (filterActions, resolver.go:208); and the
 * reads of the predicates filterActions evaluates, in order, up to and including the first that
 * fails.  ref_off / refs / ref_cap as mxp_eval_refs; MXP_ERR_NOMEM when either capacity is short,
 * with both offset arrays complete.  An identity or protocol attribute outside the vocabulary is
 * not listed (entries are vocabulary positions). */
int mxp_resolve_refs(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                     uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap, uint64_t* ref_off,
                     mxp_attr_ref* refs, uint64_t ref_cap);

/*
 * List adapter (mixer/adapter/list): membership checks of a batch of symbols against one list.
 *
 * mxp_list_create compiles a list the way the handler's parse*List functions build it
 * (list.go:182-204): entry_type is config.Params.ListEntryType (STRINGS 0,
 * CASE_INSENSITIVE_STRINGS 1, IP_ADDRESSES 2, REGEX 3).  `entries` are the provider payload's entries
 * -- the '\n'-split lines for STRINGS / CASE_INSENSITIVE / REGEX (stringList.go:29, regexList.go:44;
 * empty lines are skipped here), the YAML whitelist for IP_ADDRESSES (ipList.go:35) -- and
 * `overrides` are config.Params.Overrides.  Strings are (pointer, length) pairs.  An IP entry that
 * does not parse fails the whole list with MXP_ERR_ARG and mxp_last_error = the reference's text
 * ("could not parse list entry %s: invalid CIDR address: %s", ipList.go:62-75); override entries
 * that do not parse are ignored (ipList.go:47-51).
 *
 * mxp_list_check runs HandleListEntry (list.go:68-101) for n symbols (string blob + offsets,
 * mxp_bag_batch style) and writes the google.rpc code of each: OK 0, INVALID_ARGUMENT 3 (symbol is
 * not an IP address, IP lists), NOT_FOUND 5 (whitelist miss), PERMISSION_DENIED 7 (blacklist hit).
 * The status message follows from the code and the symbol ("%s is not whitelisted", "%s is
 * blacklisted", "%s is not a valid IP address").
 */
#define MXP_LIST_STRINGS 0
#define MXP_LIST_CASE_INSENSITIVE_STRINGS 1
#define MXP_LIST_IP_ADDRESSES 2
#define MXP_LIST_REGEX 3
#define MXP_RPC_OK 0
#define MXP_RPC_INVALID_ARGUMENT 3
#define MXP_RPC_NOT_FOUND 5
#define MXP_RPC_PERMISSION_DENIED 7
typedef struct mxp_list mxp_list;
int mxp_list_create(mxp_engine* eng, int entry_type, const char* const* entries, const uint32_t* entry_lens,
                    uint32_t n_entries, const char* const* overrides, const uint32_t* override_lens,
                    uint32_t n_overrides, mxp_list** out);
void mxp_list_destroy(mxp_engine* eng, mxp_list* list);
/* list.numEntries(): distinct strings for string lists, entries (duplicates included) otherwise */
uint64_t mxp_list_entries(const mxp_list* list);
/* REGEX lists: automata the patterns were packed into (union DFAs, and bit-parallel NFAs of patterns
 * whose own DFA is over budget); out[0] = parts, out[1] = of which NFAs.  (Engine introspection; no
 * reference counterpart.) */
void mxp_list_regex_parts(const mxp_list* list, uint32_t out[2]);
/* REGEX lists: out[0] = patterns dispatched by their literal prefix (tail automata, no union part),
 * out[1] = distinct prefixes.  (Engine introspection; no reference counterpart.) */
void mxp_list_regex_dispatch(const mxp_list* list, uint32_t out[2]);
int mxp_list_check(mxp_engine* eng, const mxp_list* list, int blacklist, const uint8_t* sym_bytes,
                   const uint64_t* sym_offsets, uint32_t n, int32_t* codes);
/* strings.ToUpper (Go 1.9: strings.Map(unicode.ToUpper, s), Unicode 9.0.0 simple uppercase) as the
 * case-insensitive lists apply it to entries and symbols (stringList.go:59,66,79): writes
 * min(cap, length) bytes of the result to out and its length to *out_len.  Host only, no engine. */
int mxp_go_to_upper(const uint8_t* s, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len);
/* Device-resident variant: symbols already in device memory (blob with >= 16 bytes of readable
 * slack after the last symbol), codes written to device memory, enqueued on `stream`. */
int mxp_list_check_device(mxp_engine* eng, const mxp_list* list, int blacklist, const uint8_t* d_sym_bytes,
                          const uint64_t* d_sym_offsets, uint32_t n, void* stream, int32_t* d_codes);
/* listentry ProcessCheck fused with HandleListEntry (mixer/template/template.gen.go
 * :2153-2202 -> mixer/adapter/list/list.go:68-101): per request, Value = Eval of rule `value_rule` of
 * the engine's compiled rule set (the instance's `value` expression, of type STRING), checked
 * against `list` in the same device pass -- no host round trip between the two.  codes[q] = the
 * google.rpc code, or MXP_LISTENTRY_EVAL_ERROR (-1) when Eval failed: the reference returns
 * "failed to evaluate field 'Value' for instance '<name>': " + mxp_pair_error(q, value_rule).
 * values (nullable): each request's Value as a result register of rule value_rule, for
 * mxp_value_text -- the symbol HandleListEntry's status messages print ("%s is not whitelisted",
 * "%s is blacklisted", "%s is not a valid IP address").
 * Every rule of the engine is evaluated (Eval mode), so instance expressions belong in an engine
 * of their own. */
#define MXP_LISTENTRY_EVAL_ERROR (-1)
/* an interface-typed Value that is not a string: the reference's `ValueInterface.(string)`
 * (template.gen.go:2177) panics */
#define MXP_LISTENTRY_NOT_STRING (-2)
int mxp_listentry_check(mxp_engine* eng, const mxp_list* list, int blacklist, const mxp_bag_batch* batch,
                        uint32_t value_rule, int32_t* codes, uint64_t* values);

/*
 * memquota (mixer/adapter/memquota): batched HandleQuota with the reference's sequential semantics.
 *
 * mxp_quota_create: n_keys quota keys with their limit (config.Params_Quota MaxAmount /
 * ValidDuration, or the matching override: limit(), memquota.go:88-105, is resolved by the caller,
 * as is the key itself, makeKey(instance.Name, instance.Dimensions)).  ValidDuration 0 = a
 * non-expiring cell, else a rolling window of ceil(ValidDuration / 1s) * 10 ticks (rollingWindow.go).
 *
 * mxp_quota_alloc: n requests in arrival order -- key id, QuotaArgs.QuotaAmount (> 0 alloc, < 0
 * free, 0 nothing), QuotaArgs.BestEffort -- all at time now_ns (currentTick = now_ns / 100 ms).
 * granted[i] = QuotaResult.Amount.  State persists across calls.  DeduplicationID handling
 * (dedup.go handleDedup) stays with the caller.  mxp_quota_alloc_device takes device arrays and can
 * accumulate per-key granted deltas (allocs - frees) into d_delta (i64[n_keys]) for the cross-GPU
 * all-reduce; a device key id >= n_keys is granted 0 and touches no key's state (the
 * host mxp_quota_alloc rejects it with MXP_ERR_ARG).  Multi-GPU: each key has one owner rank and its
 * requests are routed there (istio_amd/dist.py key_owner), so every key's sequence stays on one GPU.
 */
typedef struct mxp_quota mxp_quota;
int mxp_quota_create(mxp_engine* eng, uint32_t n_keys, const int64_t* max_amount, const int64_t* valid_duration_ns,
                     mxp_quota** out);
void mxp_quota_destroy(mxp_engine* eng, mxp_quota* quota);
int mxp_quota_alloc(mxp_engine* eng, mxp_quota* quota, uint32_t n, const uint32_t* key, const int64_t* amount,
                    const uint8_t* best_effort, int64_t now_ns, int64_t* granted);
int mxp_quota_alloc_device(mxp_engine* eng, mxp_quota* quota, uint32_t n, const uint32_t* d_key,
                           const int64_t* d_amount, const uint8_t* d_best_effort, int64_t now_ns, void* stream,
                           int64_t* d_granted, int64_t* d_delta);

/*
 * Regex compiler check (host only; test and tooling hook): compiles `pattern` with the engine's Go
 * regexp restatement and automaton builder under the rules' budget (a DFA of up to 65,536 states,
 * else the bit-parallel NFA), then matches `subject` on the host form of the automaton the device
 * would walk.  Returns 1 / 0 for match / no match, -1 for a syntax error (err = Go's "error parsing
 * regexp: ..." text), -2 for a program too large to compile, -3 when the DFA is over budget and the
 * program wider than the NFA (err says which).
 */
int mxp_regex_match_host(const char* pattern, uint32_t pattern_len, const char* subject, uint32_t subject_len,
                         char* err, uint32_t err_cap);

/*
 * Device-resident batches (benchmarking and pipelining): pack + upload once, evaluate many times.
 * mxp_batch_eval_device enqueues on `stream` (a hipStream_t; NULL = the engine's stream, which is
 * ordered with the device's legacy default stream: work the caller enqueued there first -- e.g.
 * zeroing the hit counters -- completes before the evaluation starts) and writes the bitmaps to
 * DEVICE pointers (rule-word-major, as above).  Nothing is synchronised.
 */
/*
 * Wire decoding: CompressedAttributes messages (mxp_batch.h mxp_wire_batch) ->
 * a columnar mxp_bag_batch holding one column per name, each value what ProtoBag.Get(name) returns
 * (mixer/pkg/attribute/protoBag.go:91-239): the name's index is its message-word slot when the
 * message lists it (last occurrence), else its global index (getIndex, :242-252); the value is
 * probed in Strings, StringMaps, Int64S, Doubles, Bools, Timestamps, Durations, Bytes order; a string
 * or map whose word index is defined in neither dictionary makes the attribute absent (:165-170,
 * :190-193).  names: the columns to decode; NULL = every attribute the compiled rule set reads plus,
 * when configured, the resolver's identity attribute and context.protocol.  The result owns its
 * memory and works with every call that takes an mxp_bag_batch; free with mxp_wire_free.  Host
 * threads as mxp_batch_pack_host.  No device is needed.
 */
typedef struct mxp_wire mxp_wire;
int mxp_wire_decode(mxp_engine* eng, const mxp_wire_batch* wire, const char* const* names, uint32_t n_names,
                    mxp_wire** out);
const mxp_bag_batch* mxp_wire_view(const mxp_wire* w);
void mxp_wire_free(mxp_wire* w);

/* Pinned (page-locked) host memory for the arrays of an mxp_bag_batch: a batch packed into such
 * memory is copied to the device by DMA at the link's rate, and the batch check (MXP_ERR_ARG on
 * malformed ids / offsets) runs on the host while the copies are in flight.  Pageable arrays work
 * too; the runtime stages them through its own buffers first.  A binding keeps a few such arenas
 * and reuses them batch after batch. */
int mxp_host_alloc(size_t bytes, void** out);
void mxp_host_free(void* p);

/* mxp_batch_upload returns once the batch's arrays are on the device (the caller may reuse them);
 * with the device packer, its kernels (interning, gather, pre-tables, value-class counts) run on,
 * and the batch's first evaluation waits for them and finishes the packing (value-class tables,
 * string heads, dictionary).  Uploading batch k + 1 before evaluating batch k overlaps one batch's
 * copies with the other's packing and evaluation. */
int mxp_batch_upload(mxp_engine* eng, const mxp_bag_batch* batch, mxp_dbatch** out);
/* mxp_batch_upload with flags.  MXP_UPLOAD_NO_WAIT: return once the copies are queued and the
 * batch checked, before the copies are in; the caller keeps the arrays unchanged until
 * mxp_batch_wait_copied(db) returns (or the batch's first evaluation has completed).  A worker then
 * overlaps batch k + 1's copies with its own host work for batch k (bench.py fresh_batch).  A call
 * that fails has finished reading the caller's arrays when it returns (its copy and packer streams
 * are synchronised on every error path). */
#define MXP_UPLOAD_NO_WAIT 1u
int mxp_batch_upload_ex(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t flags, mxp_dbatch** out);
int mxp_batch_wait_copied(mxp_dbatch* db);
/* mxp_batch_upload_ex of a narrow batch (mxp_batch.h mxp_bag_batch2): the u32 arrays are copied and
 * widened on the device, and checked on the host as u32.  The engine keeps a host view of the batch
 * with the device batch (mxp_resolve_uploaded takes batch = NULL for such a batch); the view's u32
 * columns are widened on the host only for a pass that reads the v1 layout (run-time regexp
 * patterns, rule sets wider than the device packer, a Resolve without device namespaces), from the
 * caller's arrays -- which such a call needs unchanged until it returns. */
int mxp_batch_upload2(mxp_engine* eng, const mxp_bag_batch2* batch, uint32_t flags, mxp_dbatch** out);
/* The host half of mxp_batch_upload alone (interning against the rule set's pools, column gather,
 * ip() / timestamp() / regexp pre-tables), for timing and tests; works on a host-only engine.
 * out[0] bytes of the packed device image, out[1] batch strings added to the overlay pool, out[2]
 * overlay byte strings.  Host threads: MXP_PACK_THREADS, else OMP_NUM_THREADS, else all cores. */
int mxp_batch_pack_host(mxp_engine* eng, const mxp_bag_batch* batch, uint64_t* out, uint32_t cap);
/* Frees a device batch without waiting for the device: its blocks are kept by the engine and
 * reused by later mxp_batch_upload calls once the work enqueued before the free -- on the engine's
 * stream and on every stream an evaluation of the batch was enqueued on -- is done.  Each
 * evaluation records the batch's completion event on its stream as it is enqueued, so the free
 * touches no caller stream: a caller may destroy its streams before freeing the batch.  The engine
 * keeps at most MXP_BIN_CAP_MB (environment, MiB) of such blocks, by default min(8 GiB, 1/16 of the
 * device's memory); a device allocation that fails first frees every engine's kept blocks and
 * retries once. */
void mxp_batch_free(mxp_engine* eng, mxp_dbatch* db);
/* Bytes of freed batch blocks the engine keeps for reuse (out[0]) and its cap (out[1]). */
int mxp_debug_bin(mxp_engine* eng, uint64_t* out);
int mxp_batch_eval_device(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match, uint32_t* d_err);
/* mxp_batch_eval_device plus fused per-rule hit counters: d_hits[rule] += the requests of this batch
 * whose predicate was true (device u64[n_rules], accumulated by the evaluation kernels as they set
 * the match bits -- the bitmap is not read back).  Same result as mxp_hits_device afterwards. */
int mxp_batch_eval_device_hits(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match, uint32_t* d_err,
                               unsigned long long* d_hits);
/* Compact error output: as mxp_batch_eval_device_hits without the error bitmap -- d_req_err[q]
 * (device u8[n_requests], cleared by the call) = 1 when some rule fails for request q, which is all a
 * Resolve needs to know that the request errs (resolver.go:225-227); the failing pairs and their texts
 * come from mxp_eval_batch / mxp_resolve_batch.  d_hits may be NULL (no counters). */
int mxp_batch_eval_device_compact(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match,
                                  uint8_t* d_req_err, unsigned long long* d_hits);
/* Per-rule hit counters: d_hits[rule] += number of requests whose predicate was true (device u64[n_rules]). */
int mxp_hits_device(mxp_engine* eng, const uint32_t* d_match, uint32_t n_requests, void* stream,
                    unsigned long long* d_hits);
uint32_t mxp_rule_count(const mxp_engine* eng);
/* Request pipelining of device evaluations: a batch of n >= 2 * min_requests requests runs as
 * min(max_chunks, n / min_requests) request chunks; the guard-index kernel of chunk c runs on a
 * second HIP stream of the engine, overlapped with the fill / guard / VM kernels of chunk c + 1, and
 * the evaluation stream waits for it before the call's work ends.  Results do not depend on it.
 * Defaults: min_requests 131072, max_chunks 1 (off: on C2 the two kernels slow each other down more
 * than the overlap saves); max_chunks <= 8. */
int mxp_set_pipeline(mxp_engine* eng, uint32_t min_requests, uint32_t max_chunks);
/* Per-kernel timing of device evaluations (off by default): with timing on, every evaluation
 * records HIP events around its launches on the evaluation stream; mxp_kernel_times waits for the
 * last one and returns its kernel durations in ms: [0] guard + VM kernels, [1] guard-index kernel
 * (0 when it did not run).  Pipelined evaluations: [0] the evaluation stream's kernels of every
 * chunk (index kernels of all but the last chunk overlapped), [1] the exposed index tail.
 * Evaluations that deferred their index pairs into the fills ([2] = 1.0 when cap
 * >= 3): [0] value-class kernels + guard-index kernel + pair sort, [1] the fills, guard / VM
 * kernels and the overflow pass.  The sum is the whole evaluation.  *n_out = values written. */
int mxp_set_timing(mxp_engine* eng, int on);
int mxp_kernel_times(mxp_engine* eng, float* ms, uint32_t cap, uint32_t* n_out);
/* Shape of the compiled rule set as the kernels see it: out[0] guarded rules (leading atom evaluated
 * group-wide), out[1] rules with a continuation template, out[2] distinct templates, out[3] column
 * segments, out[4] rules served by the guard index, out[5] device columns per request (attributes +
 * map[key] virtual columns), out[6] of the indexed rules those served by a composite (A == K1,
 * B startsWith K2) index, out[7] indexed rules that duplicate another rule's program (evaluated once,
 * results fanned out), out[8] of those canonical rules the "dense" ones whose true pairs are
 * injected once per bitmap word instead of per alias, out[9] value-class candidate columns (columns
 * whose rules depend on that column's value alone; a batch with few distinct values in such a column
 * evaluates its rules once per distinct value).  Returns the number of values written (<= cap). */
uint32_t mxp_ruleset_info(const mxp_engine* eng, uint32_t* out, uint32_t cap);
/* The attribute names the compiled rule set reads -- the columns a caller must pack into an
 * mxp_bag_batch (attribute.Bag.Get of each, protoBag.go:91-114) -- plus, once mxp_resolver_set has
 * run, the identity attribute and context.protocol (resolver.go:180-208).  Writes up to cap
 * pointers to engine-owned NUL-terminated names (valid until the next call on this engine) and
 * returns the total count; names may be NULL to count.  0 without a compiled rule set. */
uint32_t mxp_ruleset_columns(mxp_engine* eng, const char** names, uint32_t cap);
uint32_t mxp_dbatch_requests(const mxp_dbatch* db);
/* Profiling hook (engine created with MXP_WAVE_TIMES set): per wavefront of the last guard-index
 * kernel launch, {start, end, XCC} (wall_clock64 ticks, 100 MHz), 3 x u64 per wave; *n_out = values
 * written.  MXP_ERR_STATE when the hook is off. */
int mxp_debug_wave_times(mxp_engine* eng, uint64_t* out, uint64_t cap, uint64_t* n_out);

#ifdef __cplusplus
}
#endif

#endif /* MXP_H */
