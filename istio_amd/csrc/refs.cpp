// refs.cpp -- referenced attributes of a batch (mxp_eval_refs, mxp_resolve_refs; include/mxp.h).
//
// The reference tracks every attribute read an evaluation makes on the request's bag
// (ProtoBag.Get / StringMap.Get, mixer/pkg/attribute/protoBag.go:78-159; the tests' FakeBag,
// mixer/pkg/il/testing/fakebag.go:54-115).  For EvalPredicate of a rule over a request the reads are:
//   * the guard column of a guarded rule (its program starts by reading it: vmopt.h) -- the guard
//     and index phases decide such pairs without running the VM;
//   * for composite-indexed rules `A == K1 && B.startsWith(K2) && ...` (vmopt.h SecondAtom), B when
//     A holds the string K1 (the second atom runs exactly then);
//   * every read the VM performs for the pairs it runs (continuations, unguarded rules), recorded by
//     the *_refs kernels (kernels.hip ref_rec) as (request, rule, column | map lookup).
// Conditions follow from the bag: absent -> ABSENCE, present -> EXACT, a string map fetched whole ->
// MXP_REF_MAP (named by FakeBag, not by ProtoBag), map keys by their presence in the map.
//
// Two scopes: every rule (mxp_eval_refs, EvalPredicate of each rule), or one runtime.resolver
// Resolve per request (mxp_resolve_refs, resolver.go:110-238): the identity attribute, then
// context.protocol, then the rules filterActions evaluates -- the default namespace's and the
// destination namespace's rules with an action for the variety and the request's protocol and a
// non-empty match, in order, up to and including the first one that fails.
#include <cstring>
#include <string_view>
#include <unordered_set>

#include "engine_impl.h"
#include "resolve_args.h"

namespace {

int put_text(const std::string& s, char* buf, uint32_t cap) {
    if (!buf || cap == 0) return MXP_ERR_ARG;
    const size_t k = std::min<size_t>(s.size(), cap - 1);
    memcpy(buf, s.data(), k);
    buf[k] = 0;
    return s.size() < cap ? MXP_OK : MXP_ERR_NOMEM;
}

bool ref_less(const mxp_attr_ref& a, const mxp_attr_ref& b) { return a.attr != b.attr ? a.attr < b.attr : a.key < b.key; }

const char* const kProtocolAttr = "context.protocol";  // ContextProtocolAttributeName (resolver.go:95)

}  // namespace

int mxp_engine::refs_evaluate(const mxp_bag_batch* b, DevBuf& dm, DevBuf& de, std::unique_ptr<mxp_dbatch>& db,
                              std::vector<mxp_ref_rec>& recs) {
    if (!b) return MXP_ERR_ARG;
    if (!have_rules) return fail(MXP_ERR_STATE, "no rule set compiled");
    if (device < 0) return fail(MXP_ERR_STATE, "host-only engine");
    if (!refs_exact)
        return fail(MXP_ERR_STATE, "the rule set has rules the GPU lowering does not support: their reads are unknown");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hipfail(e, "hipSetDevice");
    if (!d_refcount.p && (e = d_refcount.alloc(16)) != hipSuccess) return hipfail(e, "refcount");
    if (d_refs.n < (size_t)refcap * sizeof(mxp_ref_rec) && (e = d_refs.alloc((size_t)refcap * sizeof(mxp_ref_rec))) != hipSuccess)
        return hipfail(e, "refs");
    uint32_t cnt = 0;
    refs_on = true;
    int rc = evaluate(b, dm, de, nullptr, db);
    for (int pass = 0; rc == MXP_OK && pass < 2; pass++) {
        if ((e = hipMemcpyAsync(&cnt, d_refcount.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess) {
            rc = hipfail(e, "download refcount");
            break;
        }
        if (cnt <= refcap) break;
        // more records than room: grow and evaluate again (results are deterministic)
        refcap = cnt + cnt / 4;
        if ((e = d_refs.alloc((size_t)refcap * sizeof(mxp_ref_rec))) != hipSuccess) {
            rc = hipfail(e, "refs");
            break;
        }
        rc = launch(db.get(), stream, dm.as<uint32_t>(), de.as<uint32_t>(), nullptr, true);
    }
    refs_on = false;
    if (rc) return rc;
    if (cnt > refcap) return fail(MXP_ERR_NOMEM, "referenced-attribute records");
    recs.resize(cnt);
    if (cnt && (e = hipMemcpyAsync(recs.data(), d_refs.p, (size_t)cnt * sizeof(mxp_ref_rec), hipMemcpyDeviceToHost,
                                   stream)) != hipSuccess)
        return hipfail(e, "download refs");
    return MXP_OK;
}

int mxp_engine::refs_assemble(const mxp_bag_batch* b, const std::vector<mxp_ref_rec>& recs, const RefScope* scope,
                              uint64_t* ref_off, mxp_attr_ref* out, uint64_t cap) {
    const uint32_t n = b->n_requests;
    const uint32_t NR = (uint32_t)rules.size();
    const uint32_t C = (uint32_t)cols.size(), V = (uint32_t)vcols.size();
    std::unordered_map<std::string, uint32_t> bcol;
    for (uint32_t c = 0; c < b->n_columns; c++) bcol.emplace(b->column_names[c], c);
    std::vector<int32_t> bc(C + V, -1);
    std::vector<uint32_t> attr_of(C + V, MXP_VM_DONE);
    for (uint32_t c = 0; c < C + V; c++) {
        const std::string& name = c < C ? cols[c] : vcols[c - C].first;
        auto it = bcol.find(name);
        if (it != bcol.end()) bc[c] = (int32_t)it->second;
        const int64_t vp = vocab_find(name);
        if (vp >= 0) attr_of[c] = (uint32_t)vp;
    }
    std::vector<uint32_t> battr(b->n_columns, MXP_VM_DONE);  // vocabulary position of each batch column
    for (uint32_t c = 0; c < b->n_columns; c++) {
        const int64_t vp = vocab_find(b->column_names[c]);
        if (vp >= 0) battr[c] = (uint32_t)vp;
    }
    // the rules of each composite (A, B) pair with their K1 strings (aliases included)
    struct CompRule {
        uint32_t rule;
        std::string_view k1;
    };
    struct CompGroup {
        uint32_t a, b;
        std::vector<CompRule> rules;
    };
    std::vector<CompGroup> comps;
    for (const RefComposite& x : ref_comp) {
        CompGroup* g = nullptr;
        for (auto& y : comps)
            if (y.a == x.a_col && y.b == x.b_col) g = &y;
        if (!g) {
            comps.push_back(CompGroup{x.a_col, x.b_col, {}});
            g = &comps.back();
        }
        g->rules.push_back(CompRule{x.rule, std::string_view(gstrs[x.k1])});
        for (uint32_t j = ref_alias_off[x.rule]; j < ref_alias_off[x.rule + 1]; j++)
            g->rules.push_back(CompRule{ref_aliases[j], std::string_view(gstrs[x.k1])});
    }
    // Rule lists a request evaluates, each with the set of rules of the list it may evaluate: all
    // rules (no scope), or per (namespace, tcp) the resolver-eligible ones.  Per list: the first rule
    // (lowest id = earliest in resolution order) reading each guard column, and per composite group
    // and K1 the first rule whose second atom runs.
    struct RuleList {
        uint32_t lo = 0, hi = 0;
        std::vector<std::pair<uint32_t, uint32_t>> guard_first;  // (column, first rule)
        std::vector<std::unordered_map<std::string_view, uint32_t, mxp::SvHash>> comp_first;  // [group]
    };
    const bool scoped = scope != nullptr;
    const auto& RC = resolver;
    auto eligible = [&](uint32_t r, uint32_t tcp) {
        return ((RC.vmask[r] >> scope->variety) & 1u) && RC.tcp[r] == tcp && !RC.empty[r];
    };
    auto build_list = [&](uint32_t lo, uint32_t hi, int tcp) {
        RuleList L;
        L.lo = lo;
        L.hi = hi;
        std::map<uint32_t, uint32_t> first;
        for (uint32_t r = lo; r < hi; r++) {
            if (ref_guard[r] == MXP_VM_DONE || (tcp >= 0 && !eligible(r, (uint32_t)tcp))) continue;
            first.emplace(ref_guard[r], r);  // keeps the first (lowest) rule
        }
        L.guard_first.assign(first.begin(), first.end());
        L.comp_first.resize(comps.size());
        for (size_t g = 0; g < comps.size(); g++)
            for (const CompRule& cr : comps[g].rules) {
                if (cr.rule < lo || cr.rule >= hi || (tcp >= 0 && !eligible(cr.rule, (uint32_t)tcp))) continue;
                auto ins = L.comp_first[g].emplace(cr.k1, cr.rule);
                if (!ins.second && cr.rule < ins.first->second) ins.first->second = cr.rule;
            }
        return L;
    };
    std::vector<RuleList> lists;  // unscoped: [0] = all rules; scoped: [2 * ns + tcp]
    if (!scoped) {
        lists.push_back(build_list(0, NR, -1));
    } else {
        for (size_t v = 0; v < RC.ns_lo.size(); v++)
            for (int t = 0; t < 2; t++) lists.push_back(build_list(RC.ns_lo[v], RC.ns_hi[v], t));
    }
    int32_t id_col = -1, proto_col = -1;
    uint32_t id_attr = MXP_VM_DONE, proto_attr = MXP_VM_DONE;
    if (scoped) {
        auto it = bcol.find(RC.identity);
        if (it != bcol.end()) id_col = (int32_t)it->second;
        auto pt = bcol.find(kProtocolAttr);
        if (pt != bcol.end()) proto_col = (int32_t)pt->second;
        const int64_t vi = vocab_find(RC.identity);
        if (vi >= 0) id_attr = (uint32_t)vi;
        const int64_t vp = vocab_find(kProtocolAttr);
        if (vp >= 0) proto_attr = (uint32_t)vp;
    }
    // records bucketed by request
    const uint64_t cnt = recs.size();
    std::vector<uint64_t> roff(n + 1, 0);
    for (const mxp_ref_rec& r : recs)
        if (r.req < n) roff[r.req + 1]++;
    for (uint32_t q = 0; q < n; q++) roff[q + 1] += roff[q];
    std::vector<uint32_t> rslot(cnt), rkey(cnt), rrule(cnt);
    {
        std::vector<uint64_t> at(roff.begin(), roff.end() - 1);
        for (const mxp_ref_rec& r : recs) {
            if (r.req >= n) continue;
            const uint64_t i = at[r.req]++;
            rslot[i] = r.slot;
            rkey[i] = r.key;
            rrule[i] = r.rule;
        }
    }
    auto bstr = [&](uint64_t sid) {
        return std::string_view((const char*)b->str_bytes + b->str_offsets[sid],
                                (size_t)(b->str_offsets[sid + 1] - b->str_offsets[sid]));
    };
    auto map_has = [&](uint64_t m, std::string_view key) {
        for (uint64_t x = b->map_offsets[m]; x < b->map_offsets[m + 1]; x++)
            if (bstr(b->map_keys[x]) == key) return true;
        return false;
    };
    std::vector<uint32_t> count(n, 0);
    const unsigned T = mxp::pack_threads();
    std::vector<std::vector<mxp_attr_ref>> part(T);
    std::vector<uint64_t> first_q(T, 0);
    mxp::par_for(n, 1024, [&](uint64_t q0, uint64_t q1, unsigned t) {
        std::vector<mxp_attr_ref>& o = part[t];
        first_q[t] = q0;
        std::vector<mxp_attr_ref> ents;
        for (uint64_t q = q0; q < q1; q++) {
            ents.clear();
            auto cond_of = [&](uint32_t k) {
                return k == MXP_ABSENT ? MXP_REF_ABSENCE : k == MXP_STRING_MAP ? MXP_REF_MAP : MXP_REF_EXACT;
            };
            auto kind_at = [&](int32_t col) -> uint32_t { return col < 0 ? (uint32_t)MXP_ABSENT : b->kinds[col][q]; };
            auto add_slot = [&](uint32_t c) {
                if (c >= C + V) return;
                const uint32_t a = attr_of[c];
                const uint32_t k = kind_at(bc[c]);
                if (c < C || k != MXP_STRING_MAP) {
                    ents.push_back(mxp_attr_ref{a, MXP_REF_NOKEY, cond_of(k), 0});
                    return;
                }
                // virtual column map[key] on a present map: Get(map) then StringMap.Get(key)
                ents.push_back(mxp_attr_ref{a, MXP_REF_NOKEY, MXP_REF_MAP, 0});
                const bool found = map_has(b->values[bc[c]][q], vcols[c - C].second);
                ents.push_back(mxp_attr_ref{a, vcol_key_sid[c - C], found ? MXP_REF_EXACT : MXP_REF_ABSENCE, 0});
            };
            // the rule lists of this request, each with the last rule it evaluates (cutoff)
            const RuleList* act[2] = {nullptr, nullptr};
            uint32_t cut[2] = {MXP_VM_DONE, MXP_VM_DONE};
            uint32_t tcp = 0;
            int nl = 0;
            if (!scoped) {
                act[nl++] = &lists[0];
            } else {
                ents.push_back(mxp_attr_ref{id_attr, MXP_REF_NOKEY, cond_of(kind_at(id_col)), 0});
                const uint32_t info = (*scope->info)[q];
                if (info != MXP_NS_MISSING && info != MXP_NS_NOTSTRING) {
                    ents.push_back(mxp_attr_ref{proto_attr, MXP_REF_NOKEY, cond_of(kind_at(proto_col)), 0});
                    const uint32_t v = info & 0x7FFFFFFFu;
                    tcp = info >> 31;
                    if (RC.default_id != MXP_NS_NONE) act[nl++] = &lists[2 * RC.default_id + tcp];
                    if (v != RC.default_id && v != MXP_NS_NONE) act[nl++] = &lists[2 * v + tcp];
                    if (scope->status[q] == MXP_RESOLVE_PRED_ERROR) {
                        // lists after the failing rule's are not reached
                        const uint32_t er = scope->err_rule[q];
                        for (int i = 0; i < nl; i++)
                            if (er >= act[i]->lo && er < act[i]->hi) {
                                cut[i] = er;
                                nl = i + 1;
                                break;
                            }
                    }
                }
            }
            for (int i = 0; i < nl; i++) {
                for (const auto& gf : act[i]->guard_first)
                    if (gf.second <= cut[i]) add_slot(gf.first);
                for (size_t g = 0; g < comps.size(); g++) {
                    const int32_t ca = bc[comps[g].a];
                    if (ca < 0 || b->kinds[ca][q] != MXP_STRING) continue;
                    auto it = act[i]->comp_first[g].find(bstr(b->values[ca][q]));
                    if (it != act[i]->comp_first[g].end() && it->second <= cut[i]) add_slot(comps[g].b);
                }
            }
            // does the request evaluate rule r (or one of its duplicates, whose reads are the same)?
            auto evaluated = [&](uint32_t r) {
                if (!scoped) return true;
                auto one = [&](uint32_t x) {
                    for (int i = 0; i < nl; i++)
                        if (x >= act[i]->lo && x < act[i]->hi && x <= cut[i] && eligible(x, tcp)) return true;
                    return false;
                };
                if (one(r)) return true;
                for (uint32_t j = ref_alias_off[r]; j < ref_alias_off[r + 1]; j++)
                    if (one(ref_aliases[j])) return true;
                return false;
            };
            for (uint64_t i = roff[q]; i < roff[q + 1]; i++) {
                if (scoped && !evaluated(rrule[i])) continue;
                const uint32_t s = rslot[i];
                if (!(s & MXP_REF_LOOKUP)) {
                    add_slot(s);
                    continue;
                }
                // StringMap.Get(key) on the request's map s & MXP_REF_MAPID: named by its attribute
                const uint64_t m = s & MXP_REF_MAPID;
                for (uint32_t c = 0; c < b->n_columns; c++) {
                    if (b->kinds[c][q] != MXP_STRING_MAP || b->values[c][q] != m) continue;
                    ents.push_back(mxp_attr_ref{battr[c], MXP_REF_NOKEY, MXP_REF_MAP, 0});
                    ents.push_back(mxp_attr_ref{battr[c], rkey[i], (s & MXP_REF_FOUND) ? MXP_REF_EXACT : MXP_REF_ABSENCE, 0});
                    break;
                }
            }
            std::sort(ents.begin(), ents.end(), ref_less);
            uint32_t k = 0;
            for (size_t i = 0; i < ents.size(); i++) {
                if (ents[i].attr == MXP_VM_DONE) continue;
                if (k && ents[i].attr == o.back().attr && ents[i].key == o.back().key) continue;
                o.push_back(ents[i]);
                k++;
            }
            count[q] = k;
        }
    });
    ref_off[0] = 0;
    for (uint32_t q = 0; q < n; q++) ref_off[q + 1] = ref_off[q] + count[q];
    if (ref_off[n] > cap || (!out && ref_off[n]))
        return fail(MXP_ERR_NOMEM, "referenced-attribute capacity " + std::to_string(cap) + " < " + std::to_string(ref_off[n]));
    for (unsigned t = 0; t < T; t++)
        if (!part[t].empty()) memcpy(out + ref_off[first_q[t]], part[t].data(), part[t].size() * sizeof(mxp_attr_ref));
    return MXP_OK;
}

int mxp_engine::eval_refs(const mxp_bag_batch* b, uint32_t* match, uint32_t* err, uint64_t* ref_off, mxp_attr_ref* out,
                          uint64_t cap) {
    if (!b || !ref_off) return MXP_ERR_ARG;
    std::unique_ptr<mxp_dbatch> db;
    DevBuf dm, de;
    std::vector<mxp_ref_rec> recs;
    int rc = refs_evaluate(b, dm, de, db, recs);
    if (rc) return rc;
    const uint32_t n = b->n_requests;
    const uint32_t W = ((uint32_t)rules.size() + 31) / 32;
    hipError_t e;
    if (match && (e = hipMemcpyAsync(match, dm.p, (size_t)W * n * 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hipfail(e, "download match");
    if (err && (e = hipMemcpyAsync(err, de.p, (size_t)W * n * 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hipfail(e, "download err");
    if ((rc = collect_errors(b, db))) return rc;  // synchronises; the batch becomes last_db
    return refs_assemble(b, recs, nullptr, ref_off, out, cap);
}

extern "C" {

int mxp_eval_refs(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t* match_bits, uint32_t* err_bits,
                  uint64_t* ref_off, mxp_attr_ref* refs, uint64_t cap) {
    if (!eng) return MXP_ERR_ARG;
    return eng->eval_refs(batch, match_bits, err_bits, ref_off, refs, cap);
}

int mxp_string_text(mxp_engine* eng, uint32_t sid, char* buf, uint32_t cap) {
    if (!eng) return MXP_ERR_ARG;
    if (sid >= eng->gstrs.size() + (eng->last_db ? eng->last_db->overlay_strings() : 0)) return MXP_ERR_ARG;
    return put_text(eng->string_of(nullptr, sid), buf, cap);
}

}  // extern "C"
