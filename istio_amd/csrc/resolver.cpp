// resolver.cpp -- batched runtime.resolver on top of the predicate bitmaps (include/mxp.h,
// resolve.hip).
//
// Reference: resolver.Resolve (mixer/pkg/runtime/resolver.go:110-168), destAndNamespace
// (:180-199), filterActions (:202-238).  The host derives each request's namespace and TCP flag
// from its bag exactly as destAndNamespace / filterActions do; the GPU walks the namespace rule
// ranges over the bitmaps mxp_eval_kernel / mxp_index_kernel produced.
#include <cstring>
#include <numeric>
#include <string_view>

#include "engine_impl.h"
#include "pack_args.h"
#include "resolve_args.h"

extern "C" hipError_t mxp_launch_resolve(const mxp_resolve_args* a, int write, hipStream_t s);
extern "C" hipError_t mxp_launch_ns(const mxp_ns_args* a, hipStream_t s);
extern "C" hipError_t mxp_launch_resolve_scatter(const uint32_t* pairs, uint32_t m, uint32_t* err_in, hipStream_t s);
extern "C" hipError_t mxp_launch_resolve_first_err(const mxp_resolve_args* a, const void* recs, uint32_t m, hipStream_t s);

namespace {

const char* const kProtocolAttr = "context.protocol";  // ContextProtocolAttributeName (resolver.go:95)

// namespace info of every request: destAndNamespace + the tcp flag of filterActions (parallel over
// requests; namespace names looked up as string views)
int request_info(mxp_engine* eng, const mxp_bag_batch* b, std::vector<uint32_t>* info) {
    const auto& R = eng->resolver;
    const uint32_t n = b->n_requests;
    int idc = -1, pc = -1;
    for (uint32_t c = 0; c < b->n_columns; c++) {
        if (R.identity == b->column_names[c]) idc = (int)c;
        if (strcmp(kProtocolAttr, b->column_names[c]) == 0) pc = (int)c;
    }
    std::unordered_map<std::string_view, uint32_t> ns_ids;
    for (const auto& kv : R.ns_ids) ns_ids.emplace(std::string_view(kv.first), kv.second);
    auto str = [&](uint64_t sid) {
        return std::string_view((const char*)b->str_bytes + b->str_offsets[sid],
                                (size_t)(b->str_offsets[sid + 1] - b->str_offsets[sid]));
    };
    info->resize(n);
    uint32_t* out = info->data();
    mxp::par_for(n, 16384, [&](uint64_t q0, uint64_t q1, unsigned) {
        for (uint64_t q = q0; q < q1; q++) {
            // attrs.Get(idAttr): nil -> "identity not found"; not a string -> "identity must be string"
            if (idc < 0 || b->kinds[idc][q] == MXP_ABSENT) {
                out[q] = MXP_NS_MISSING;
                continue;
            }
            if (b->kinds[idc][q] != MXP_STRING) {
                out[q] = MXP_NS_NOTSTRING;
                continue;
            }
            const std::string_view d = str(b->values[idc][q]);
            // strings.SplitN(dest, ".", 3): ns = splits[1] when there is at least one '.'
            std::string_view ns;
            const size_t dot1 = d.find('.');
            if (dot1 != std::string_view::npos) {
                const std::string_view rest = d.substr(dot1 + 1);
                ns = rest.substr(0, rest.find('.'));
            }
            auto it = ns_ids.find(ns);
            const uint32_t v = it == ns_ids.end() ? MXP_NS_NONE : it->second;
            // tcp := attrs.Get("context.protocol") == "tcp": an interface compare, so only a string
            const bool tcp = pc >= 0 && b->kinds[pc][q] == MXP_STRING && str(b->values[pc][q]) == "tcp";
            out[q] = v | (tcp ? 0x80000000u : 0u);
        }
    });
    return MXP_OK;
}

}  // namespace

extern "C" {

int mxp_resolver_set(mxp_engine* eng, const char* identity_attr, const char* default_ns, const char* const* rule_ns,
                     const uint32_t* variety_mask, const uint8_t* is_tcp, const uint8_t* empty_match, uint32_t n) {
    if (!eng || !identity_attr || !default_ns || (n && (!rule_ns || !variety_mask || !is_tcp || !empty_match)))
        return MXP_ERR_ARG;
    if (!eng->have_rules) return eng->fail(MXP_ERR_STATE, "no rule set compiled");
    if (n != eng->rules.size()) return eng->fail(MXP_ERR_ARG, "resolver: rule count differs from the rule set");
    mxp_engine::ResolverConf R;
    R.identity = identity_attr;
    R.default_ns = default_ns;
    // the attributes every Resolve reads get their vocabulary positions now (the finder is asked
    // here, at snapshot time, never on the evaluation path: refs.cpp uses vocab_find)
    (void)eng->vocab_pos(R.identity);
    (void)eng->vocab_pos("context.protocol");
    R.vmask.assign(variety_mask, variety_mask + n);
    R.tcp.assign(is_tcp, is_tcp + n);
    R.empty.assign(empty_match, empty_match + n);
    for (uint32_t i = 0; i < n; i++) {
        const std::string ns = rule_ns[i] ? rule_ns[i] : "";
        auto it = R.ns_ids.find(ns);
        if (it == R.ns_ids.end()) {
            const uint32_t id = (uint32_t)R.ns_names.size();
            if (id >= MXP_NS_NONE) return eng->fail(MXP_ERR_ARG, "resolver: too many namespaces");
            R.ns_ids.emplace(ns, id);
            R.ns_names.push_back(ns);
            R.ns_lo.push_back(i);
            R.ns_hi.push_back(i + 1);
        } else if (R.ns_hi[it->second] != i) {
            return eng->fail(MXP_ERR_ARG, "resolver: rules of namespace '" + ns + "' are not contiguous");
        } else {
            R.ns_hi[it->second] = i + 1;
        }
    }
    auto d = R.ns_ids.find(R.default_ns);
    R.default_id = d == R.ns_ids.end() ? MXP_NS_NONE : d->second;
    R.set = true;
    eng->res_gen++;  // (the device tables of the previous configuration are stale)
    // the namespace names on the device (mxp_ns_kernel): content-hash table, descriptors, bytes
    if (eng->device >= 0) {
        hipError_t e;
        if ((e = hipSetDevice(eng->device)) != hipSuccess) return eng->hipfail(e, "hipSetDevice");
        uint32_t cap = 64;
        while (cap < 2 * R.ns_names.size()) cap <<= 1;
        std::vector<unsigned long long> tab(cap, 0ull);
        std::vector<uint64_t> desc;
        std::string blob;
        for (uint32_t id = 0; id < R.ns_names.size(); id++) {
            const std::string& nm = R.ns_names[id];
            desc.push_back(((uint64_t)blob.size() << 24) | nm.size());
            blob += nm;
            const uint64_t h = mxp_item_hash((const uint8_t*)nm.data(), (uint32_t)nm.size());
            uint32_t slot = (uint32_t)h & (cap - 1);
            while (tab[slot]) slot = (slot + 1) & (cap - 1);
            tab[slot] = ((h >> 32) << 32) | (id + 1ull);
        }
        blob.append(16, '\0');
        desc.push_back(0);
        auto put = [&](DevBuf& b, const void* src, size_t bytes) -> int {
            if ((e = b.alloc(bytes)) != hipSuccess || (e = hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess)
                return eng->hipfail(e, "resolver namespaces");
            return MXP_OK;
        };
        int rc;
        if ((rc = put(eng->res_ns_tab, tab.data(), tab.size() * 8)) || (rc = put(eng->res_ns_desc, desc.data(), desc.size() * 8)) ||
            (rc = put(eng->res_ns_blob, blob.data(), blob.size())))
            return rc;
        eng->res_ns_mask = cap - 1;
    }
    eng->resolver = std::move(R);
    return MXP_OK;
}

}  // extern "C"

namespace {

// MXP_DEBUG_FLAGS: resolve through the error bitmap (the pre-round-5 path), for A/B and tests
constexpr uint32_t kResolveBitmap = 1u << 28;
// ids enqueued with the other outputs only for capacities up to this many bytes (the device buffer
// is sized by the capacity, not the count)
constexpr uint64_t kEarlyIdsMax = 256ull << 20;

// Each request's first applicable erroring rule in resolution order (filterActions returns at the
// first EvalPredicate error, resolver.go:226-228) from the error records of a compact evaluation:
// (request, rule) pairs for the requests that fail.  hinfo: the requests' namespace info.
void first_errors(mxp_engine* eng, uint32_t n, uint32_t variety, const uint32_t* hinfo, std::vector<uint32_t>* pairs) {
    const auto& R = eng->resolver;
    std::vector<uint32_t>& best = eng->res_best;  // (kept all ~0 between calls)
    if (best.size() < n) best.assign(n, 0xFFFFFFFFu);
    const bool has_def = R.default_id != MXP_NS_NONE;
    const uint32_t dlo = has_def ? R.ns_lo[R.default_id] : 0u, dhi = has_def ? R.ns_hi[R.default_id] : 0u;
    const uint32_t dlen = dhi - dlo;
    std::vector<uint32_t> touched;
    (void)eng->ensure_recs();  // (class records make collect_errors download them at once; kept for safety)
    for (const mxp_err_rec& rec : eng->last_recs) {
        const uint32_t q = rec.req, r = rec.rule;
        if (q >= n || r >= R.vmask.size()) continue;
        const uint32_t info = hinfo[q];
        if (info == MXP_NS_MISSING || info == MXP_NS_NOTSTRING) continue;
        const uint32_t tcp = info >> 31, ns = info & 0x7FFFFFFFu;
        if (R.empty[r] || !((R.vmask[r] >> variety) & 1u) || R.tcp[r] != tcp) continue;
        uint32_t rank;
        if (has_def && r >= dlo && r < dhi) {
            rank = r - dlo;
        } else if (ns != MXP_NS_NONE && ns != R.default_id && r >= R.ns_lo[ns] && r < R.ns_hi[ns]) {
            rank = dlen + (r - R.ns_lo[ns]);
        } else {
            continue;
        }
        if (best[q] == 0xFFFFFFFFu) touched.push_back(q);
        if (rank < best[q]) best[q] = rank;
    }
    pairs->clear();
    pairs->reserve(2 * touched.size());
    for (uint32_t q : touched) {
        const uint32_t rank = best[q];
        const uint32_t ns = hinfo[q] & 0x7FFFFFFFu;
        pairs->push_back(q);
        pairs->push_back(rank < dlen ? dlo + rank : R.ns_lo[ns] + (rank - dlen));
        best[q] = 0xFFFFFFFFu;
    }
}

}  // namespace

// A Resolve in two phases (resolve_impl runs both; mxp_resolve_submit / _finish let a caller work
// between them): begin enqueues the evaluation and the request namespaces and returns without
// waiting for the device; end waits, finds the first errors, counts, places and downloads.
struct mxp_resolve_job {
    mxp_engine* eng = nullptr;
    const mxp_bag_batch* batch = nullptr;
    uint32_t variety = 0;
    bool ids16 = false;
    bool compact = false;
    uint32_t n = 0, W = 0;
    uint64_t* ref_off = nullptr;
    mxp_attr_ref* refs = nullptr;
    uint64_t ref_cap = 0;
    std::unique_ptr<mxp_dbatch> db;
    std::vector<mxp_ref_rec> recs;
    std::vector<uint32_t> info;  // host copy of the namespaces (host pass; referenced attributes)
    const uint32_t* hinfo = nullptr;
    mxp_engine::PairView pairs;  // the evaluation's filed pairs (pair Resolve; on = false: the bitmap)
    bool pairs_filed = false;    // (the evaluation filed them; pairs_ovf: how many overflowed)
    uint32_t pairs_ovf = 0;
    uint32_t recs_n = 0, class_recs_n = 0;  // (the evaluation's error records: diagnostics)
    // a group member whose ids go first in the batch's list (member 0): the group's capacity, so its
    // ids are enqueued with the other outputs, before the placement (0: after it)
    uint64_t first_cap = 0;
};

namespace {

int resolve_begin(mxp_resolve_job& J) {
    mxp_engine* eng = J.eng;
    const mxp_bag_batch* batch = J.batch;
    const uint32_t variety = J.variety;
    mxp_dbatch* pre = J.db.get();
    if (pre && (J.ref_off || pre->n != batch->n_requests))
        return eng->fail(MXP_ERR_ARG, "resolve: the uploaded batch is not this batch");
    if (pre && eng->device >= 0 && hipSetDevice(eng->device) != hipSuccess) return eng->fail(MXP_ERR_DEVICE, "hipSetDevice");
    if (!eng->resolver.set) return eng->fail(MXP_ERR_STATE, "resolver not configured (mxp_resolver_set)");
    const auto& R = eng->resolver;
    const uint32_t n = J.n = batch->n_requests;
    const uint32_t NR = (uint32_t)eng->rules.size();
    const uint32_t W = J.W = (NR + 31) / 32;
    if (J.ids16 && NR > 65536u) return eng->fail(MXP_ERR_ARG, "u16 rule ids: more than 65536 rules");
    DevBuf& dm = eng->res_dm;  // (engine-owned scratch: no allocation per call once large enough)
    DevBuf& de = eng->res_de;
    hipError_t e;
    int rc;
    // the resolver's tables first, before the evaluation is queued: a copy from pageable memory
    // returns only once the stream has reached it, so behind the evaluation it would hold the
    // caller until the kernels end (r6_s25: 0.79 ms)
    // (kept on the device while the configuration and variety stay: four pageable copies a call,
    // ~0.1 ms of the caller's time, before)
    DevBuf &d_info = eng->res_info, &d_lo = eng->res_lo, &d_hi = eng->res_hi, &d_amask = eng->res_amask,
           &d_empty = eng->res_empty;
    auto up = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.reserve(bytes)) != hipSuccess) return eng->hipfail(e, what);
        if (bytes && (e = hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
            return eng->hipfail(e, what);
        return MXP_OK;
    };
    const uint64_t tab_key = eng->res_gen << 6 | variety;
    if (eng->res_tab_key != tab_key) {
        std::vector<uint32_t> amask(2 * (size_t)W, 0), empty(W, 0);  // per-word masks: variety / tcp, empty matches
        bool any_empty = false;
        for (uint32_t r = 0; r < NR; r++) {
            const uint32_t bit = 1u << (r & 31);
            if ((R.vmask[r] >> variety) & 1u) amask[(size_t)R.tcp[r] * W + r / 32] |= bit;
            if (R.empty[r]) {
                empty[r / 32] |= bit;
                any_empty = true;
            }
        }
        eng->res_tab_key = ~0ull;  // (until every table is up)
        if ((rc = up(d_lo, R.ns_lo.data(), R.ns_lo.size() * 4, "upload ns_lo"))) return rc;
        if ((rc = up(d_hi, R.ns_hi.data(), R.ns_hi.size() * 4, "upload ns_hi"))) return rc;
        if ((rc = up(d_amask, amask.data(), amask.size() * 4, "upload amask"))) return rc;
        if ((rc = up(d_empty, empty.data(), empty.size() * 4, "upload empty"))) return rc;
        eng->res_tab_key = tab_key;
        eng->res_any_empty = any_empty;
    }
    const bool any_empty = eng->res_any_empty;
    J.compact = !J.ref_off && !(eng->debug_flags & kResolveBitmap);
    if (J.compact) {
        if (eng->device >= 0 && (e = eng->res_flags.reserve(n ? n : 1)) != hipSuccess) return eng->hipfail(e, "alloc flags");
        // pair Resolve: the selected rules from the evaluation's deferred pairs, the bitmap left
        // unwritten, where the plan allows it (the launch decides); rules with an empty match are
        // selected without a pair, so their sets keep the bitmap
        eng->pair_req = eng->resolve_pairs != 0 && !any_empty;
        if (pre) {
            rc = eng->evaluate_uploaded(J.db.get(), dm, de, nullptr, eng->res_flags.as<uint8_t>());
        } else {
            rc = eng->evaluate(batch, dm, de, nullptr, J.db, eng->res_flags.as<uint8_t>());
        }
        J.pairs = eng->pair_req && !rc ? eng->last_pairs : mxp_engine::PairView{};
        J.pairs_filed = J.pairs.on;
        eng->pair_req = false;
    } else {
        rc = J.ref_off ? eng->refs_evaluate(batch, dm, de, J.db, J.recs)
             : pre     ? eng->evaluate_uploaded(J.db.get(), dm, de, nullptr, nullptr)
                       : eng->evaluate(batch, dm, de, nullptr, J.db);
    }
    if (rc) return rc;
    // request namespaces: on the device from the batch as uploaded (pack_device), else on the host
    mxp_dbatch* db = J.db.get();
    if (db->res_raw && !J.ref_off) {
        if ((e = d_info.reserve((size_t)n * 4 + 4)) != hipSuccess) return eng->hipfail(e, "alloc nsinfo");
        mxp_ns_args N;
        memset(&N, 0, sizeof N);
        N.n = n;
        N.ns_mask = eng->res_ns_mask;
        N.id_kind = db->res_id_kind;
        N.id_val = db->res_id_val;
        N.pr_kind = db->res_pr_kind;
        N.pr_val = db->res_pr_val;
        N.soff = db->pk.pk_soff.as<uint64_t>();
        N.sbytes = db->pk.pk_sbytes.as<uint8_t>();
        N.ns_tab = eng->res_ns_tab.as<unsigned long long>();
        N.ns_desc = eng->res_ns_desc.as<uint64_t>();
        N.ns_blob = eng->res_ns_blob.as<uint8_t>();
        N.nsinfo = d_info.as<uint32_t>();
        if (n && (e = mxp_launch_ns(&N, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch namespaces");
        eng->trace_mark("request namespaces (device)");
    } else {
        if (db->wide && batch == &db->wide->view) db->wide->materialize();  // (a narrow upload)
        request_info(eng, batch, &J.info);
        J.hinfo = J.info.data();
        eng->trace_mark("request namespaces (host)");
        if ((rc = up(d_info, J.info.data(), J.info.size() * 4, "upload nsinfo"))) return rc;
    }
    return MXP_OK;
}

int resolve_end(mxp_resolve_job& J, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                uint64_t sel_cap, const mxp_resolve_place* place) {
    mxp_engine* eng = J.eng;
    const mxp_bag_batch* batch = J.batch;
    const uint32_t variety = J.variety, n = J.n, W = J.W;
    const bool ids16 = J.ids16, compact = J.compact;
    uint64_t* ref_off = J.ref_off;
    mxp_attr_ref* refs = J.refs;
    const uint64_t ref_cap = J.ref_cap;
    auto& db = J.db;
    auto& recs = J.recs;
    auto& info = J.info;
    const uint32_t* hinfo = J.hinfo;
    const auto& R = eng->resolver;
    DevBuf& dm = eng->res_dm;
    DevBuf& de = eng->res_de;
    DevBuf &d_info = eng->res_info, &d_lo = eng->res_lo, &d_hi = eng->res_hi, &d_amask = eng->res_amask,
           &d_empty = eng->res_empty, &d_status = eng->res_status, &d_err_rule = eng->res_err_rule,
           &d_count = eng->res_count, &d_off = eng->res_off, &d_sel = eng->res_sel;
    hipError_t e;
    int rc;
    auto up = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.reserve(bytes)) != hipSuccess) return eng->hipfail(e, what);
        if (bytes && (e = hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
            return eng->hipfail(e, what);
        return MXP_OK;
    };
    if ((e = d_status.reserve(n)) != hipSuccess) return eng->hipfail(e, "alloc status");
    if ((e = d_err_rule.reserve((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc err_rule");
    if ((e = d_count.reserve((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc count");
    const uint32_t grid = (n + 255u) / 256u;
    if ((e = eng->res_bsum.reserve((size_t)grid * 8 + 8)) != hipSuccess) return eng->hipfail(e, "alloc block sums");
    if ((e = d_off.reserve(((size_t)n + 1) * 8)) != hipSuccess) return eng->hipfail(e, "alloc sel_off");
    if ((e = eng->res_stash.reserve((size_t)n * 16 + 16)) != hipSuccess) return eng->hipfail(e, "alloc stash");
    mxp_resolve_args A;
    memset(&A, 0, sizeof A);
    A.n = n;
    A.n_words = W;
    A.nsinfo = d_info.as<uint32_t>();
    A.ns_lo = d_lo.as<uint32_t>();
    A.ns_hi = d_hi.as<uint32_t>();
    A.default_id = R.default_id;
    A.amask = d_amask.as<uint32_t>();
    A.empty = d_empty.as<uint32_t>();
    A.match = dm.as<uint32_t>();
    A.err = compact ? nullptr : de.as<uint32_t>();
    A.status = d_status.as<uint8_t>();
    A.err_rule = d_err_rule.as<uint32_t>();
    A.count = d_count.as<uint32_t>();
    A.block_sum = eng->res_bsum.as<uint64_t>();
    A.sel_off_out = d_off.as<uint64_t>();
    A.sel_off = d_off.as<uint64_t>();
    A.ids16 = ids16 ? 1u : 0u;
    A.stash = (uint4*)eng->res_stash.p;
    bool collected = false;  // (records collected after the resolve kernels unless a path needed them first)
    if (compact) {
        // the log's counts: [0] records, [2] class records (synchronises: the evaluation is done)
        // (into pinned memory: both copies queued, one synchronisation)
        if (!eng->res_small && (e = hipHostMalloc((void**)&eng->res_small, 64, hipHostMallocDefault)) != hipSuccess) {
            eng->res_small = nullptr;
            return eng->hipfail(e, "pinned counters");
        }
        uint32_t* const hs = eng->res_small;
        hs[4] = hs[5] = 0;
        if ((e = hipMemcpyAsync(hs, eng->d_errcount.p, 16, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess ||
            (J.pairs.on &&
             (e = hipMemcpyAsync(hs + 4, J.pairs.ovf_n, 8, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess) ||
            (e = hipStreamSynchronize(eng->stream)) != hipSuccess)
            return eng->hipfail(e, "download errcount");
        const uint32_t cnt[4] = {hs[0], hs[1], hs[2], hs[3]}, ovf[2] = {hs[4], hs[5]};
        // (pairs past their lists or slots: the fills stored the bitmap after all -- read it)
        J.pairs_ovf = ovf[0];
        J.recs_n = cnt[0];
        J.class_recs_n = cnt[2];
        if (ovf[0]) J.pairs.on = false;
        if ((e = eng->res_err_in.reserve((size_t)n * 4 + 4)) != hipSuccess) return eng->hipfail(e, "alloc err_in");
        if (n && (e = hipMemsetAsync(eng->res_err_in.p, 0xFF, (size_t)n * 4, eng->stream)) != hipSuccess)
            return eng->hipfail(e, "reset err_in");
        if (cnt[0] > eng->errcap) {
            // records past the log's capacity: the error bitmap after all (an evaluation without a log)
            if ((e = de.reserve((size_t)W * n * 4)) != hipSuccess) return eng->hipfail(e, "alloc err");
            if ((rc = eng->launch(db.get(), eng->stream, dm.as<uint32_t>(), de.as<uint32_t>(), nullptr, false))) return rc;
            A.err = de.as<uint32_t>();
            J.pairs.on = false;  // (this evaluation wrote both bitmaps)
            eng->trace_mark("error bitmap (log overflow)");
        } else if (!cnt[2]) {
            // each request's first error from the records, on the device
            A.err_in = eng->res_err_in.as<uint32_t>();
            A.err_rank = 1u;
            if ((e = mxp_launch_resolve_first_err(&A, eng->d_errlog.p, cnt[0], eng->stream)) != hipSuccess)
                return eng->hipfail(e, "launch first errors");
            eng->trace_mark("first errors (device)");
        } else {
            // value-class records stand for whole classes: expanded per request on the host
            // (collect_errors), then the first error of each failing request found there
            if ((rc = eng->collect_errors(batch, db))) return rc;
            collected = true;
            if (!eng->errors_complete) {
                if ((e = de.reserve((size_t)W * n * 4)) != hipSuccess) return eng->hipfail(e, "alloc err");
                if ((rc = eng->launch(eng->last_db.get(), eng->stream, dm.as<uint32_t>(), de.as<uint32_t>(), nullptr,
                                      false)))
                    return rc;
                A.err = de.as<uint32_t>();
                J.pairs.on = false;
            } else {
                if (n && hinfo == nullptr) {  // (the device namespaces, brought back for this pass)
                    info.resize(n);
                    if ((rc = eng->download(info.data(), d_info.p, (size_t)n * 4, "download nsinfo"))) return rc;
                    hinfo = info.data();
                }
                std::vector<uint32_t> pairs;
                first_errors(eng, n, variety, hinfo, &pairs);
                if ((rc = up(eng->res_pairs, pairs.data(), pairs.size() * 4, "upload first errors"))) return rc;
                if ((e = mxp_launch_resolve_scatter(eng->res_pairs.as<uint32_t>(), (uint32_t)(pairs.size() / 2),
                                                    eng->res_err_in.as<uint32_t>(), eng->stream)) != hipSuccess)
                    return eng->hipfail(e, "launch first errors");
                A.err_in = eng->res_err_in.as<uint32_t>();
            }
            eng->trace_mark("first errors (class records, host)");
        }
    }
    // (the default namespace's range tiled through LDS: resolve_tile; MXP_RESOLVE_TILE=0 the per-lane walk;
    // a pair Resolve reads the filed pairs instead)
    const bool tiled = eng->resolve_tile && R.default_id != MXP_NS_NONE;
    const bool pairs = J.pairs.on && !A.err;
    if (eng->resolve_pairs == 2 && n && !pairs) {
        char why[160];
        snprintf(why, sizeof why,
                 "pair Resolve not taken (MXP_RESOLVE_PAIRS=2): pairs filed %d, overflowed %u, error bitmap %d "
                 "(records %u of %u, class records %u)",
                 J.pairs_filed ? 1 : 0, J.pairs_ovf, A.err ? 1 : 0, J.recs_n, eng->errcap, J.class_recs_n);
        return eng->fail(MXP_ERR_STATE, why);
    }
    if (pairs) {
        A.pr_slots = J.pairs.slots;
        A.pr_qn = J.pairs.qn;
        A.pr_fills = J.pairs.fills;
        A.pr_row = J.pairs.row;
        A.pr_nch = J.pairs.nch;
    }
    const int count_mode = pairs ? 5 : tiled ? 3 : 0, write_mode = pairs ? 6 : tiled ? 4 : 1;
    if (n && (e = mxp_launch_resolve(&A, count_mode, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve");
    if (n && (e = mxp_launch_resolve(&A, 2, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve scan");
    eng->trace_mark("  resolve: count + scan kernels");
    // The ids enqueued now, with the other outputs, when they go to the start of pinned caller memory:
    // the write pass guarded by the capacity (it writes nothing past it) and a download sized on the
    // device by sel_off[n] -- one synchronisation for every output instead of two (the ids' count is
    // known on the host only after the first).  Otherwise, or when they do not fit, after it.
    const size_t isz = ids16 ? 2 : 4;
    const uint64_t early_cap = place ? J.first_cap : sel_cap;
    void* const sel_hd = n && early_cap && !ref_off && early_cap * isz <= kEarlyIdsMax ? eng->host_dev_ptr(sel_rules) : nullptr;
    if (sel_hd) {
        if ((e = d_sel.reserve(early_cap * isz)) != hipSuccess) return eng->hipfail(e, "alloc sel");
        A.sel_rules = d_sel.as<uint32_t>();
        A.sel_cap_dev = early_cap;
        if ((e = mxp_launch_resolve(&A, write_mode, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve write");
        if ((e = mxp_launch_d2h_copy_ids(sel_hd, d_sel.p, d_off.as<uint64_t>() + n, (uint32_t)isz, early_cap,
                                         eng->stream)) != hipSuccess)
            return eng->hipfail(e, "download sel");
        A.sel_cap_dev = 0;
    }
    if (!n) {
        if (!place) sel_off[0] = 0;
    } else {
        const std::vector<mxp_engine::Piece> outs = {{status, d_status.p, n},
                                                     {err_rule, d_err_rule.p, (size_t)n * 4},
                                                     // (a group member leaves sel_off[0] alone: that
                                                     // entry is the previous member's last one)
                                                     place ? mxp_engine::Piece{sel_off + 1, d_off.as<uint64_t>() + 1, (size_t)n * 8}
                                                           : mxp_engine::Piece{sel_off, d_off.p, ((size_t)n + 1) * 8}};
        if ((rc = eng->download_all(outs, "download resolve outputs"))) return rc;
    }
    eng->trace_mark("resolve kernels + downloads");
    if (!collected) {
        if ((rc = eng->collect_errors(batch, db))) return rc;  // synchronises the stream
        eng->trace_mark("error records");
    }
    int ref_rc = MXP_OK;
    if (ref_off) {
        const mxp_engine::RefScope scope{&info, status, err_rule, variety};
        ref_rc = eng->refs_assemble(batch, recs, &scope, ref_off, refs, ref_cap);
        if (ref_rc && ref_rc != MXP_ERR_NOMEM) return ref_rc;
    }
    const uint64_t total = n ? sel_off[n] : 0;
    // (a group member learns where its ids go in the whole batch's list once every member knows its
    // own count: place blocks until then, -1 = the whole list does not fit)
    int64_t at = 0;
    if (place) {
        at = (*place)(total);
        if (at < 0) return MXP_ERR_NOMEM;
    } else if (total > sel_cap) {
        return MXP_ERR_NOMEM;
    }
    if (total && sel_hd && total <= early_cap && at == 0) {
        eng->trace_mark("action lists (with the outputs)");
        return ref_rc;
    }
    if (total) {
        if ((e = d_sel.reserve(total * isz)) != hipSuccess) return eng->hipfail(e, "alloc sel");
        A.sel_rules = d_sel.as<uint32_t>();
        if ((e = mxp_launch_resolve(&A, write_mode, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve write");
        if ((rc = eng->download((uint8_t*)sel_rules + (size_t)at * isz, d_sel.p, total * isz, "download sel"))) return rc;
    }
    eng->trace_mark("action lists (gather + download)");
    return ref_rc;
}


// mxp_resolve_batch(_ex), and with ref_off its referenced attributes (mxp_resolve_refs).
//
// Compact path (round 5; not for referenced attributes): the evaluation writes the match bitmap and
// per-request error flags with error records instead of the error bitmap; namespaces come from the
// device (mxp_ns_kernel on the batch as uploaded); each failing request's first applicable error is
// found from the records on the host and scattered to the device; the counts are scanned on the
// device.  Records past the log's capacity fall back to the error bitmap.
int resolve_impl(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, bool ids16, uint8_t* status,
                 uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap, uint64_t* ref_off,
                 mxp_attr_ref* refs, uint64_t ref_cap, const mxp_resolve_place* place = nullptr,
                 mxp_dbatch* pre = nullptr, uint64_t first_cap = 0) {
    mxp_resolve_job J;
    J.first_cap = first_cap;
    J.db.reset(pre);  // (a batch uploaded before: taken over, whatever happens)
    if (!eng || !batch || !status || !err_rule || !sel_off || (sel_cap && !sel_rules) || variety >= 32)
        return MXP_ERR_ARG;
    J.eng = eng;
    J.batch = batch;
    J.variety = variety;
    J.ids16 = ids16;
    J.ref_off = ref_off;
    J.refs = refs;
    J.ref_cap = ref_cap;
    if (int rc = resolve_begin(J)) return rc;
    return resolve_end(J, status, err_rule, sel_off, sel_rules, sel_cap, place);
}

}  // namespace

int mxp_resolve_placed(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                       uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                       const mxp_resolve_place& place, uint64_t first_cap) {
    if (!batch && db && db->wide) batch = &db->wide->view;  // (a narrow upload: its host view)
    if (flags & ~(uint32_t)MXP_RESOLVE_IDS_U16) {
        if (eng && db) eng->recycle(db);
        return MXP_ERR_ARG;
    }
    return resolve_impl(eng, batch, variety, (flags & MXP_RESOLVE_IDS_U16) != 0, status, err_rule, sel_off, sel_rules,
                        0, nullptr, nullptr, 0, &place, db, first_cap);
}

// (group.cpp) a member's finish with its ids placed by the group, and dropping a submitted job
int mxp_resolve_finish_placed(mxp_resolve_job* job, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off,
                              void* sel_rules, const mxp_resolve_place& place, uint64_t first_cap) {
    std::unique_ptr<mxp_resolve_job> J(job);
    if (!J) return MXP_ERR_ARG;
    J->first_cap = first_cap;
    return resolve_end(*J, status, err_rule, sel_off, sel_rules, 0, &place);
}
void mxp_resolve_job_free(mxp_resolve_job* job) { delete job; }

extern "C" {

int mxp_resolve_batch(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                      uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap) {
    return resolve_impl(eng, batch, variety, false, status, err_rule, sel_off, sel_rules, sel_cap, nullptr, nullptr, 0);
}

int mxp_resolve_batch_ex(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                         uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap) {
    if (flags & ~(uint32_t)MXP_RESOLVE_IDS_U16) return MXP_ERR_ARG;
    return resolve_impl(eng, batch, variety, (flags & MXP_RESOLVE_IDS_U16) != 0, status, err_rule, sel_off, sel_rules,
                        sel_cap, nullptr, nullptr, 0);
}

int mxp_resolve_uploaded(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                         uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules, uint64_t sel_cap) {
    if (!db) return MXP_ERR_ARG;
    if (!batch && db->wide) batch = &db->wide->view;  // (a narrow upload: its host view)
    if (!eng || (flags & ~(uint32_t)MXP_RESOLVE_IDS_U16)) {
        if (eng) eng->recycle(db);
        return MXP_ERR_ARG;
    }
    return resolve_impl(eng, batch, variety, (flags & MXP_RESOLVE_IDS_U16) != 0, status, err_rule, sel_off, sel_rules,
                        sel_cap, nullptr, nullptr, 0, nullptr, db);
}

int mxp_resolve_submit(mxp_engine* eng, mxp_dbatch* db, const mxp_bag_batch* batch, uint32_t variety, uint32_t flags,
                       mxp_resolve_job** out) {
    std::unique_ptr<mxp_resolve_job> J(new mxp_resolve_job());
    J->db.reset(db);  // (taken over, whatever happens)
    if (!eng || !db || !out || (flags & ~(uint32_t)MXP_RESOLVE_IDS_U16) || variety >= 32) return MXP_ERR_ARG;
    if (!batch && db->wide) batch = &db->wide->view;  // (a narrow upload: its host view)
    if (!batch) return MXP_ERR_ARG;
    J->eng = eng;
    J->batch = batch;
    J->variety = variety;
    J->ids16 = (flags & MXP_RESOLVE_IDS_U16) != 0;
    if (int rc = resolve_begin(*J)) return rc;
    *out = J.release();
    return MXP_OK;
}

int mxp_resolve_finish(mxp_resolve_job* job, uint8_t* status, uint32_t* err_rule, uint64_t* sel_off, void* sel_rules,
                       uint64_t sel_cap) {
    std::unique_ptr<mxp_resolve_job> J(job);
    if (!J || !status || !err_rule || !sel_off || (sel_cap && !sel_rules)) return MXP_ERR_ARG;
    return resolve_end(*J, status, err_rule, sel_off, sel_rules, sel_cap, nullptr);
}

int mxp_resolve_refs(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                     uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap, uint64_t* ref_off,
                     mxp_attr_ref* refs, uint64_t ref_cap) {
    if (!ref_off) return MXP_ERR_ARG;
    return resolve_impl(eng, batch, variety, false, status, err_rule, sel_off, sel_rules, sel_cap, ref_off, refs,
                        ref_cap);
}

}  // extern "C"
