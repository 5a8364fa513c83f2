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
#include "resolve_args.h"

extern "C" hipError_t mxp_launch_resolve(const mxp_resolve_args* a, int write, hipStream_t s);

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
    eng->resolver = std::move(R);
    return MXP_OK;
}

}  // extern "C"

namespace {

// mxp_resolve_batch, and with ref_off its referenced attributes (mxp_resolve_refs)
int resolve_impl(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status, uint32_t* err_rule,
                 uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap, uint64_t* ref_off, mxp_attr_ref* refs,
                 uint64_t ref_cap) {
    if (!eng || !batch || !status || !err_rule || !sel_off || (sel_cap && !sel_rules) || variety >= 32)
        return MXP_ERR_ARG;
    if (!eng->resolver.set) return eng->fail(MXP_ERR_STATE, "resolver not configured (mxp_resolver_set)");
    const auto& R = eng->resolver;
    const uint32_t n = batch->n_requests;
    const uint32_t NR = (uint32_t)eng->rules.size();
    const uint32_t W = (NR + 31) / 32;
    std::unique_ptr<mxp_dbatch> db;
    DevBuf& dm = eng->res_dm;  // (engine-owned scratch: no allocation per call once large enough)
    DevBuf& de = eng->res_de;
    std::vector<mxp_ref_rec> recs;
    int rc = ref_off ? eng->refs_evaluate(batch, dm, de, db, recs) : eng->evaluate(batch, dm, de, nullptr, db);
    if (rc) return rc;
    // per-word masks: applicability for the variety (per request tcp flag), empty matches
    std::vector<uint32_t> amask(2 * (size_t)W, 0), empty(W, 0);
    for (uint32_t r = 0; r < NR; r++) {
        const uint32_t bit = 1u << (r & 31);
        if ((R.vmask[r] >> variety) & 1u) amask[(size_t)R.tcp[r] * W + r / 32] |= bit;
        if (R.empty[r]) empty[r / 32] |= bit;
    }
    std::vector<uint32_t> info;
    request_info(eng, batch, &info);
    eng->trace_mark("request namespaces (host)");
    hipError_t e;
    DevBuf &d_info = eng->res_info, &d_lo = eng->res_lo, &d_hi = eng->res_hi, &d_amask = eng->res_amask,
           &d_empty = eng->res_empty, &d_status = eng->res_status, &d_err_rule = eng->res_err_rule,
           &d_count = eng->res_count, &d_off = eng->res_off, &d_sel = eng->res_sel;
    auto up = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.reserve(bytes)) != hipSuccess) return eng->hipfail(e, what);
        if (bytes && (e = hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
            return eng->hipfail(e, what);
        return MXP_OK;
    };
    if ((rc = up(d_info, info.data(), info.size() * 4, "upload nsinfo"))) return rc;
    if ((rc = up(d_lo, R.ns_lo.data(), R.ns_lo.size() * 4, "upload ns_lo"))) return rc;
    if ((rc = up(d_hi, R.ns_hi.data(), R.ns_hi.size() * 4, "upload ns_hi"))) return rc;
    if ((rc = up(d_amask, amask.data(), amask.size() * 4, "upload amask"))) return rc;
    if ((rc = up(d_empty, empty.data(), empty.size() * 4, "upload empty"))) return rc;
    if ((e = d_status.reserve(n)) != hipSuccess) return eng->hipfail(e, "alloc status");
    if ((e = d_err_rule.reserve((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc err_rule");
    if ((e = d_count.reserve((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc count");
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
    A.err = de.as<uint32_t>();
    A.status = d_status.as<uint8_t>();
    A.err_rule = d_err_rule.as<uint32_t>();
    A.count = d_count.as<uint32_t>();
    if (n && (e = mxp_launch_resolve(&A, 0, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve");
    std::vector<uint32_t> count(n);
    if (n && (e = hipMemcpyAsync(count.data(), d_count.p, (size_t)n * 4, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "download count");
    if (n && (e = hipMemcpyAsync(status, d_status.p, n, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "download status");
    if (n && (e = hipMemcpyAsync(err_rule, d_err_rule.p, (size_t)n * 4, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "download err_rule");
    eng->trace_mark("resolve kernel + downloads");
    if ((rc = eng->collect_errors(batch, db))) return rc;  // synchronises the stream
    eng->trace_mark("error records");
    int ref_rc = MXP_OK;
    if (ref_off) {
        const mxp_engine::RefScope scope{&info, status, err_rule, variety};
        ref_rc = eng->refs_assemble(batch, recs, &scope, ref_off, refs, ref_cap);
        if (ref_rc && ref_rc != MXP_ERR_NOMEM) return ref_rc;
    }
    sel_off[0] = 0;
    for (uint32_t q = 0; q < n; q++) sel_off[q + 1] = sel_off[q] + count[q];
    const uint64_t total = sel_off[n];
    if (total > sel_cap) return MXP_ERR_NOMEM;
    if (total) {
        if ((rc = up(d_off, sel_off, ((size_t)n + 1) * 8, "upload sel_off"))) return rc;
        if ((e = d_sel.reserve(total * 4)) != hipSuccess) return eng->hipfail(e, "alloc sel");
        A.sel_off = d_off.as<uint64_t>();
        A.sel_rules = d_sel.as<uint32_t>();
        if ((e = mxp_launch_resolve(&A, 1, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch resolve write");
        if ((rc = eng->download(sel_rules, d_sel.p, total * 4, "download sel"))) return rc;
    }
    eng->trace_mark("action lists (gather + download)");
    return ref_rc;
}

}  // namespace

extern "C" {

int mxp_resolve_batch(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                      uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap) {
    return resolve_impl(eng, batch, variety, status, err_rule, sel_off, sel_rules, sel_cap, nullptr, nullptr, 0);
}

int mxp_resolve_refs(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t variety, uint8_t* status,
                     uint32_t* err_rule, uint64_t* sel_off, uint32_t* sel_rules, uint64_t sel_cap, uint64_t* ref_off,
                     mxp_attr_ref* refs, uint64_t ref_cap) {
    if (!ref_off) return MXP_ERR_ARG;
    return resolve_impl(eng, batch, variety, status, err_rule, sel_off, sel_rules, sel_cap, ref_off, refs, ref_cap);
}

}  // extern "C"
