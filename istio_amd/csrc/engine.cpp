// engine.cpp -- host side of the MXP engine and the C-ABI of include/mxp.h.
//
// Responsibilities:
//   * vocabulary + rule-set compilation (compile_rule -> lower_rule), one upload per snapshot;
//   * batch packing: the caller's columnar bags (mxp_batch.h) become device SoA columns with every
//     string interned into one id space (rule-set constants first, then the batch's own strings),
//     IP byte strings and timestamps interned to canonical ids (so equality is id equality), and
//     `map[const key]` lookups pre-extracted into virtual columns;
//   * kernel launches on the engine's HIP stream and reporting of error pairs with the reference's
//     exact error texts.
#include <atomic>
#include <deque>

#include "engine_impl.h"

thread_local BlockBin* g_bin_take = nullptr;
thread_local const void* g_bin_db = nullptr;
thread_local size_t g_bin_db_size = 0;
thread_local std::vector<std::pair<void*, size_t>>* g_bin_give = nullptr;

namespace {
std::mutex g_bins_mu;
std::set<BlockBin*> g_bins;  // every live engine's bin
}  // namespace

BlockBin::BlockBin() {
    std::lock_guard<std::mutex> g(g_bins_mu);
    g_bins.insert(this);
}

BlockBin::~BlockBin() {
    {
        std::lock_guard<std::mutex> g(g_bins_mu);
        g_bins.erase(this);
    }
    release();
}

bool bins_release_all() {
    std::lock_guard<std::mutex> g(g_bins_mu);
    bool any = false;
    for (BlockBin* b : g_bins) {
        any |= b->held() > 0;
        b->release();
    }
    return any;
}

// A batch's device blocks go to the bin (no hipFree: it would wait for the whole device), with the
// completion events of its evaluations and one on the engine stream (the packer).
void mxp_engine::recycle(mxp_dbatch* db) {
    if (!db) return;
    BlockBin::Group g;
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, kOrderEvent) != hipSuccess || hipEventRecord(e, stream) != hipSuccess) {
        if (e) (void)hipEventDestroy(e);
        delete db;  // (no event: the plain frees)
        return;
    }
    g.evs.push_back(e);
    for (auto& se : db->done_ev) g.evs.push_back(se.second);  // (the group owns them now)
    db->done_ev.clear();
    for (hipEvent_t& pe : db->pk_ev)  // (the packer's kernels ran on a stream of their own)
        if (pe) {
            g.evs.push_back(pe);
            pe = nullptr;
        }
    g_bin_give = &g.blks;
    delete db;
    g_bin_give = nullptr;
    bin.put(std::move(g));
}

// the cap, set on first use (an upload or free: the engine's device is current)
size_t BlockBin::cap_locked() {
    if (!cap_set) {
        const char* e = getenv("MXP_BIN_CAP_MB");
        if (e && *e) {
            cap_bytes = (size_t)strtoull(e, nullptr, 10) << 20;
        } else {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot) cap_bytes = std::min(cap_bytes, tot / 16);
        }
        cap_set = true;
    }
    return cap_bytes;
}

size_t BlockBin::held() {
    std::lock_guard<std::mutex> g(mu);
    return bytes;
}

// the smallest block of at least `want` bytes and at most twice that (+ 1 MB), its group's work
// waited for once
bool BlockBin::take(size_t want, void** p, size_t* cap) {
    std::lock_guard<std::mutex> lk(mu);
    size_t bg = 0, bi = 0, best = SIZE_MAX;
    // groups whose work is done first (a query, no wait): a block released moments ago -- a packed
    // batch's scratch, its last kernels still running -- is taken only when nothing else fits
    for (int pass = 0; pass < 2 && best == SIZE_MAX; pass++)
        for (size_t g = 0; g < groups.size(); g++) {
            if (pass == 0 && !groups[g].done) {
                bool all = true;
                for (hipEvent_t e : groups[g].evs) all = all && hipEventQuery(e) == hipSuccess;
                (void)hipGetLastError();  // (hipErrorNotReady)
                if (!all) continue;
                groups[g].done = true;
            }
            for (size_t i = 0; i < groups[g].blks.size(); i++) {
                const size_t c = groups[g].blks[i].second;
                if (c >= want && c <= 2 * want + (1u << 20) && c < best) {
                    best = c;
                    bg = g;
                    bi = i;
                }
            }
        }
    if (best == SIZE_MAX) return false;
    Group& G = groups[bg];
    if (!G.done) {
        for (hipEvent_t e : G.evs) (void)hipEventSynchronize(e);
        G.done = true;
    }
    *p = G.blks[bi].first;
    *cap = G.blks[bi].second;
    bytes -= best;
    G.blks[bi] = G.blks.back();
    G.blks.pop_back();
    if (G.blks.empty()) {
        for (hipEvent_t e : G.evs) (void)hipEventDestroy(e);
        groups.erase(groups.begin() + (ptrdiff_t)bg);
    }
    return true;
}

void BlockBin::put(Group&& g) {
    std::lock_guard<std::mutex> lk(mu);
    const size_t cap = cap_locked();
    for (auto& b : g.blks) bytes += b.second;
    groups.push_back(std::move(g));
    while (bytes > cap && !groups.empty()) {
        Group& G = groups.front();
        for (hipEvent_t e : G.evs) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
        for (auto& b : G.blks) {
            (void)hipFree(b.first);
            bytes -= b.second;
        }
        groups.erase(groups.begin());
    }
}

void BlockBin::release() {
    std::lock_guard<std::mutex> lk(mu);
    for (Group& G : groups) {
        for (hipEvent_t e : G.evs) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
        for (auto& b : G.blks) (void)hipFree(b.first);
    }
    groups.clear();
    bytes = 0;
}


// ------------------------------------------------------------------------------------ compile
int mxp_engine::compile(const char* const* exprs, uint32_t n, int32_t* status) {
    reset_tables();
    res_gen++;  // (the resolver's device tables are sized by the rule count)
    ref_comp.clear();
    plans.clear();
    views_n[0] = ~(size_t)0;  // string-view indexes rebuilt at the next pack
    rules.resize(n);
    std::vector<mxp_vm_ins>& all = prog_h;
    std::vector<uint32_t>& off = off_h;
    all.clear();
    off.assign(n + 1, 0);
    if (finder) {  // vocabulary through the caller's finder: resolve every name the rules use
        std::vector<const mxp::Expr*> stack;
        for (uint32_t i = 0; i < n; i++) {
            std::string err;
            mxp::ExprP e = mxp::parse_expression(exprs[i] ? exprs[i] : "", &err);
            if (!e) continue;
            stack.assign(1, e.get());
            while (!stack.empty()) {
                const mxp::Expr* x = stack.back();
                stack.pop_back();
                if (x->kind == mxp::Expr::VAR) vocab_pos(x->var);
                if (x->target) stack.push_back(x->target.get());
                for (const auto& a : x->args) stack.push_back(a.get());
            }
        }
    }
    for (uint32_t i = 0; i < n; i++) {
        Rule& R = rules[i];
        mxp::CompiledRule cr;
        mxp::compile_rule(exprs[i] ? exprs[i] : "", vocab, fmap, &cr);
        R.status = (int32_t)cr.status;
        R.error = cr.error;
        R.value_type = cr.value_type;
        std::vector<mxp_vm_ins> code;
        if (cr.status == mxp::CompiledRule::OK) {
            const mxp::IlFunction* f = cr.program.get("eval");
            R.il_ret = f ? f->ret : 0;
            R.il_text = mxp::write_il_text(cr.program);
            R.low = mxp::lower_rule(cr.program, this);
            if (R.low.ok) {
                code = R.low.code;
                need_ipof |= R.low.uses_ipof;
                need_rxof |= R.low.uses_rxof;
                need_tsof |= R.low.uses_tsof;
                need_strings |= R.low.uses_strings;
                need_maps |= R.low.uses_maps;
            } else {
                R.status = MXP_RULE_UNSUPPORTED;
                R.error = "unsupported by the GPU lowering: " + R.low.why;
            }
        }
        if (code.empty()) {
            mxp_vm_ins e{};
            e.op = VM_ERR;
            e.y = R.status == MXP_RULE_COMPILE_PANIC ? PANIC_STATIC
                  : R.status == MXP_RULE_UNSUPPORTED ? ERR_UNSUPPORTED : ERR_STATIC;
            e.z = i;
            code.push_back(e);
        }
        off[i] = (uint32_t)all.size();
        all.insert(all.end(), code.begin(), code.end());
        if (status) status[i] = R.status;
    }
    off[n] = (uint32_t)all.size();
    // virtual columns follow the resolve columns
    const uint32_t C = (uint32_t)cols.size();
    for (auto& ins : all)
        if ((ins.op & 0x7F) == VM_VCOL) ins.x += C;
    for (auto& R : rules)
        for (auto& ins : R.low.code)
            if ((ins.op & 0x7F) == VM_VCOL) ins.x += C;
    // leading-atom guards (evaluated for a whole 32-rule group at once by the kernel)
    std::vector<mxp_guard>& guards = guards_h;
    guards.assign(n, mxp_guard{});
    struct RxPrefixed {
        uint32_t rule, dfa;
        std::string prefix;
    };
    std::vector<RxPrefixed> rx_prefixed;  // regexp rules guarded by their literal prefix
    rx_keys_h.assign(n, {});
    for (uint32_t i = 0; i < n; i++) {
        std::vector<mxp_vm_ins> code(all.begin() + off[i], all.begin() + off[i + 1]);
        guards[i] = mxp::extract_guard(code);
    }
    n_guarded = 0;
    for (auto& g : guards) n_guarded += (g.mode & 0xFF) != GM_NONE;

    // regexp rules `"^lit...".matches(col)` (program RES|VCOL x; REGEX y <- x; RET y): a subject can
    // only match when it starts with the pattern's literal prefix -- a necessary-condition guard
    // (GM_AND, continuation = the whole program) that the prefix index can serve
    {
        std::vector<std::string> pattern_of(rx_set.hdr.size());
        for (auto& kv : rx_ids)
            if (kv.second.first >= 0) pattern_of[kv.second.first] = kv.first;
        for (uint32_t i = 0; i < n; i++) {
            if ((guards[i].mode & 0xFF) != GM_NONE || off[i + 1] - off[i] != 3) continue;
            const mxp_vm_ins& r = all[off[i]];
            const mxp_vm_ins& x = all[off[i] + 1];
            const mxp_vm_ins& t = all[off[i] + 2];
            const uint32_t rop = r.op & 0x7F;
            const bool col_ok = (rop == VM_RES && r.y == W_S) || rop == VM_VCOL;
            if (!col_ok || (x.op & 0x7F) != VM_REGEX || x.a != r.d || (t.op & 0x7F) != VM_RET || t.a != x.d ||
                t.y != 1 || ((x.op | t.op) & MXP_VM_WAKE))
                continue;
            std::string prefix;
            if (!mxp::regex_required_prefix(pattern_of[x.x], &prefix)) continue;
            mxp_guard g{};
            g.col = r.x | ((rop == VM_VCOL ? (uint32_t)GK_VCOL : (uint32_t)W_S) << 24);
            g.mode = GM_AND | GT_PREFIX;  // continuation pc 0: the whole program
            g.klo = intern_string(prefix);
            guards[i] = g;
            rx_prefixed.push_back({i, x.x, prefix});
        }
    }

    // continuation templates (vmopt.h hoist_continuation): rules whose continuations are identical
    // up to constants share one program; template code is appended after the rules' programs
    std::map<std::string, uint32_t> tmpl_ids;
    std::vector<mxp_tmpl>& tmpls = tmpls_h;
    tmpls.clear();
    std::vector<mxp_vm_ins> tcode;
    std::vector<uint32_t>& rule_tmpl = rule_tmpl_h;
    rule_tmpl.assign(n, MXP_VM_DONE);
    std::vector<uint64_t> rconst((size_t)n * MXP_VM_MAXREG, 0);
    const uint32_t prog_end = (uint32_t)all.size();
    n_templated = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t mode = guards[i].mode & 0xFF, pc0 = guards[i].mode >> 16;
        if (mode != GM_AND && mode != GM_OR) continue;
        if (rules[i].low.nregs > MXP_VM_MAXREG) continue;  // deep rule: the index kernels' registers are too few
        std::vector<mxp_vm_ins> code(all.begin() + off[i], all.begin() + off[i + 1]);
        mxp::HoistedCont h;
        if (!mxp::hoist_continuation(code, pc0, &h)) continue;
        uint32_t hdr[4] = {pc0, (uint32_t)code.size(), h.creg0, (uint32_t)h.consts.size()};
        std::string key((const char*)hdr, sizeof hdr);
        key.append((const char*)h.code.data(), h.code.size() * sizeof(mxp_vm_ins));
        auto it = tmpl_ids.find(key);
        uint32_t id;
        if (it != tmpl_ids.end()) {
            id = it->second;
        } else {
            id = (uint32_t)tmpls.size();
            tmpl_ids.emplace(key, id);
            mxp_tmpl t{};
            t.off = prog_end + (uint32_t)tcode.size();
            t.pc0 = pc0;
            t.len = (uint32_t)code.size();
            t.nconst = (uint32_t)h.consts.size();
            t.creg0 = h.creg0;
            tmpls.push_back(t);
            tcode.insert(tcode.end(), h.code.begin(), h.code.end());
        }
        rule_tmpl[i] = id;
        for (size_t j = 0; j < h.consts.size(); j++) rconst[(size_t)i * MXP_VM_MAXREG + j] = h.consts[j];
        n_templated++;
    }
    all.insert(all.end(), tcode.begin(), tcode.end());

    // A prefix-guarded regexp rule runs (through its template, from the guard index) only for
    // subjects that start with its literal prefix: its template constant names a derived DFA that
    // starts in the state the prefix leads to, `skip` bytes in -- or that is decided by the prefix
    // alone (`^/api[a-z]*`: the empty star already matches).  The rule's own program keeps the full
    // DFA (Eval mode, referenced-attribute scopes, plans without the index).
    for (const RxPrefixed& rp : rx_prefixed) {
        if (rule_tmpl[rp.rule] == MXP_VM_DONE) continue;
        const mxp_tmpl& t = tmpls[rule_tmpl[rp.rule]];
        uint32_t creg = MXP_VM_DONE;
        for (uint32_t pc = t.pc0; pc < t.len; pc++) {
            const mxp_vm_ins& ti = all[t.off - t.pc0 + pc];
            if ((ti.op & 0x7F) == VM_REGEXR) creg = ti.b;
        }
        if (creg == MXP_VM_DONE || creg < t.creg0 || creg >= t.creg0 + t.nconst) continue;
        const mxp::Dfa& d = rx_dfas[rp.dfa];
        if (d.is_nfa()) continue;  // the NFA walks the whole subject
        uint32_t st = d.start;
        for (size_t b = 0; b < rp.prefix.size() && st < mxp::kDfaReject;) {
            const uint8_t c = (uint8_t)rp.prefix[b];
            uint32_t cls, w = 1;
            if (c < 0x80) {
                cls = d.ascii[c];
            } else {  // a literal rune's UTF-8 bytes
                uint32_t r = 0;
                w = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
                r = c & (0xFFu >> (w + 1));
                for (uint32_t k = 1; k < w; k++) r = (r << 6) | ((uint8_t)rp.prefix[b + k] & 0x3Fu);
                const size_t at = std::upper_bound(d.hi_lo.begin(), d.hi_lo.end(), r) - d.hi_lo.begin() - 1;
                cls = d.hi_cls[at];
            }
            st = d.trans[(size_t)st * d.ncls + cls];
            b += w;
        }
        if (st == mxp::kDfaReject) continue;
        // a few literal continuations decide the match (`^/p(/.*)?$`: the subject is /p, or starts
        // with /p/): direct postings on the full keys, exact-length ones where the subject must end
        // (MXP_DEBUG_FLAGS 67108864: keep the DFA template -- A/B)
        std::vector<mxp::LiteralKey> keys;
        if (!(debug_flags & 67108864u) && n < (1u << 23) && mxp::dfa_literal_keys(d, st, 8, 8, &keys)) {
            auto& rk = rx_keys_h[rp.rule];
            for (const auto& k : keys) rk.push_back({intern_string(rp.prefix + k.bytes), k.tail ? 2u : k.exact ? 1u : 0u});
            guards[rp.rule].mode = GM_ONLY | GT_PREFIX;
            continue;
        }
        mxp_dfa_hdr h = rx_set.hdr[rp.dfa];
        h.start = st == mxp::kDfaAccept ? 0u : st;
        h.skip = st == mxp::kDfaAccept ? MXP_DFA_DECIDED : (uint32_t)rp.prefix.size();
        rx_set.hdr.push_back(h);
        rx_dfas.emplace_back();  // (keeps rx_dfas aligned with the device headers; never walked)
        rconst[(size_t)rp.rule * MXP_VM_MAXREG + (creg - t.creg0)] = rx_set.hdr.size() - 1;
    }

    // value-class candidates: rules whose result is a function of ONE column's (kind, string value)
    // alone, so a batch with few distinct values in that column evaluates them once per value
    // (mxp_vt_eval_kernel) and broadcasts the words by class (vt_merge)
    {
        std::vector<uint32_t> vcol(n, MXP_VM_DONE);
        std::map<uint32_t, uint32_t> count;
        for (uint32_t i = 0; i < n; i++) {
            // (mxp_vt_eval_kernel has the MXP_VM_MAXREG register file)
            if (rules[i].status != MXP_RULE_OK || rules[i].low.nregs > MXP_VM_MAXREG) continue;
            uint32_t col = MXP_VM_DONE;
            bool ok = true;
            for (uint32_t p = off[i]; p < off[i + 1] && ok; p++) {
                const mxp_vm_ins& ins = all[p];
                uint32_t c = MXP_VM_DONE;
                switch (ins.op & 0x7F) {
                case VM_RES: case VM_TRES: ok = ins.y == W_S; c = ins.x; break;
                case VM_VCOL: c = ins.x; break;
                case VM_LOOKUP: case VM_LOOKUPK: case VM_REGEXD: ok = false; break;
                default: break;
                }
                if (c != MXP_VM_DONE) {
                    if (col == MXP_VM_DONE) col = c;
                    else if (col != c) ok = false;
                }
            }
            if (ok && col != MXP_VM_DONE) {
                vcol[i] = col;
                count[col]++;
            }
        }
        std::vector<std::pair<uint32_t, uint32_t>> cand;  // (rules, column)
        for (auto& kv : count)
            if (kv.second >= kVtMinRules) cand.push_back({kv.second, kv.first});
        std::sort(cand.begin(), cand.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
        if (cand.size() > kVtCandMax) cand.resize(kVtCandMax);
        vt_cand_col.clear();
        vt_slot_of_rule.assign(n, 0xFF);
        std::map<uint32_t, uint32_t> slot_of;
        for (auto& c : cand) {
            slot_of[c.second] = (uint32_t)vt_cand_col.size();
            vt_cand_col.push_back(c.second);
        }
        for (uint32_t i = 0; i < n; i++)
            if (vcol[i] != MXP_VM_DONE && slot_of.count(vcol[i])) vt_slot_of_rule[i] = (uint8_t)slot_of[vcol[i]];
    }

    vcol_key_sid.resize(vcols.size());
    for (size_t j = 0; j < vcols.size(); j++) vcol_key_sid[j] = intern_string(vcols[j].second);
    refs_exact = true;
    for (auto& R : rules) refs_exact &= R.status != MXP_RULE_UNSUPPORTED;
    // referenced attributes (mxp_eval_refs): the guard of every guarded rule reads its column for
    // every request
    ref_guard.assign(n, MXP_VM_DONE);
    for (uint32_t i = 0; i < n; i++)
        if ((guards[i].mode & 0xFF) != GM_NONE) ref_guard[i] = guards[i].col & 0xFFFFFFu;

    have_rules = false;
    if (device >= 0) {
        // upload the rule-level tables: programs (+ template code), constants, regexp DFAs, strings
        hipError_t e;
        if ((e = hipSetDevice(device)) != hipSuccess) return hipfail(e, "hipSetDevice");
        auto put = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
            if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return hipfail(e, what);
            if (bytes && (e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess) return hipfail(e, what);
            return MXP_OK;
        };
        int rc;
        if ((rc = put(d_prog, all.data(), all.size() * sizeof(mxp_vm_ins), "upload prog"))) return rc;
        if ((rc = put(d_rule_off, off.data(), off.size() * 4, "upload rule_off"))) return rc;
        if ((rc = put(d_rconst, rconst.data(), rconst.size() * 8, "upload rconst"))) return rc;
        rx_nfa = rx_set.has_nfa();
        rx_wmax = rx_set.nfa_wmax();
        if ((rc = put(d_rx_hdr, rx_set.hdr.data(), rx_set.hdr.size() * sizeof(mxp_dfa_hdr), "upload rx hdr"))) return rc;
        if ((rc = put(d_rx_trans, rx_set.trans.data(), rx_set.trans.size() * 4, "upload rx trans"))) return rc;
        if ((rc = put(d_rx_ascii, rx_set.ascii.data(), rx_set.ascii.size() * 2, "upload rx ascii"))) return rc;
        if ((rc = put(d_rx_hilo, rx_set.hilo.data(), rx_set.hilo.size() * 4, "upload rx hilo"))) return rc;
        if ((rc = put(d_rx_hicls, rx_set.hicls.data(), rx_set.hicls.size() * 2, "upload rx hicls"))) return rc;
    }
    // plan 0 (no value classes) interns nothing new, so the string pool can go up after it
    Plan* p0 = nullptr;
    int rc = get_plan(0, &p0);
    if (rc) return rc;
    if (device >= 0) {
        hipError_t e;
        std::vector<uint64_t> soff;
        std::string blob;
        if (!string_pool(gstrs, &soff, &blob)) return fail(MXP_ERR_ARG, "rule-set string longer than 16 MiB");
        if ((e = d_gstr_off.alloc(soff.size() * 8)) != hipSuccess) return hipfail(e, "hipMalloc gstr_off");
        if ((e = d_gstr.alloc(blob.size())) != hipSuccess) return hipfail(e, "hipMalloc gstr");
        if ((e = hipMemcpy(d_gstr_off.p, soff.data(), soff.size() * 8, hipMemcpyHostToDevice)) != hipSuccess)
            return hipfail(e, "upload gstr_off");
        if (!blob.empty() && (e = hipMemcpy(d_gstr.p, blob.data(), blob.size(), hipMemcpyHostToDevice)) != hipSuccess)
            return hipfail(e, "upload gstr");
    }
    have_rules = true;
    return MXP_OK;
}

int mxp_engine::get_plan(uint32_t mask, Plan** out) {
    auto it = plans.find(mask);
    if (it != plans.end()) {
        *out = it->second.get();
        return MXP_OK;
    }
    std::unique_ptr<Plan> P(new Plan());
    P->mask = mask;
    int rc = build_plan(*P);
    if (rc) return rc;
    *out = P.get();
    plans.emplace(mask, std::move(P));
    return MXP_OK;
}

// The kernels' view of the rule set for one set of value-class columns (Plan::mask): the rules the
// value classes serve are left out of every table below -- groups, segments, guard indexes, fills,
// aliases -- and come back as per-group merge entries (gvt) instead.
int mxp_engine::build_plan(Plan& P) {
    const uint32_t n = (uint32_t)rules.size();
    const std::vector<mxp_vm_ins>& all = prog_h;
    const std::vector<uint32_t>& off = off_h;
    std::vector<mxp_guard> guards = guards_h;
    std::vector<uint32_t> rule_tmpl = rule_tmpl_h;
    std::vector<mxp_tmpl> tmpls = tmpls_h;
    std::vector<uint8_t> excluded(n, 0);
    for (uint32_t i = 0; i < n; i++)
        excluded[i] = vt_slot_of_rule[i] != 0xFF && ((P.mask >> vt_slot_of_rule[i]) & 1u);
    const bool base = P.mask == 0;  // plan 0 also fills the referenced-attribute tables

    // guard index.  Equality: GM_AND, non-negated, templated rules -- their continuing pairs are the
    // requests whose column value equals K.  Prefix: `col.startsWith(K)` alone (GM_ONLY: a posting IS
    // a true pair) or followed by `&& ...` (GM_AND, templated), and the regexp prefix guards above.
    // Per (column, want class, kind) a hash table K -> postings.  A prefix guard the index cannot
    // serve falls back to a guard-less rule (phase 1 only compares equality atoms).
    std::vector<uint8_t> indexed(n, 0);
    std::map<std::pair<uint32_t, bool>, std::map<uint64_t, std::vector<uint32_t>>> index_of;
    // composite: (A column, B column) -> (K1, K2 string id) -> rules
    std::map<std::pair<uint32_t, uint32_t>, std::map<std::pair<uint64_t, uint32_t>, std::vector<uint32_t>>> comp_of;
    std::vector<uint32_t> rule_tmpl2(n, MXP_VM_DONE);
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> tmpl2_ids;  // (template, resume pc) -> template
    P.n_indexed = 0;
    P.n_composite = 0;
    // duplicate predicates: indexed rules whose programs are identical (same code, same constants)
    // compute identical results, so only the first one (the canonical rule) enters the index; each
    // result the index kernel produces for it is fanned out to its aliases (kargs.alias_off / aliases)
    std::unordered_map<std::string, uint32_t> canon_of;
    std::vector<std::vector<uint32_t>> aliases_of(n);
    P.n_alias = 0;
    if (base) ref_comp.clear();
    for (uint32_t i = 0; i < n; i++) {
        if (excluded[i]) continue;
        mxp_guard& gd = guards[i];
        const uint32_t mode = gd.mode & 0xFF;
        const bool prefix = (gd.mode & GT_PREFIX) != 0, neg = (gd.mode >> 8) & 1;
        // GM_ONLY prefix atoms (`attr.startsWith(K)` alone): a posting IS a true pair.  Equality
        // atoms alone stay with phase 1's group compares -- indexing them too (MXP_DEBUG_FLAGS 512)
        // measured slower on C4 (header equality: 0.35 ms compared, 0.92 ms indexed)
        bool ok = !(debug_flags & 8u) && !neg &&
                  ((mode == GM_AND && rule_tmpl[i] != MXP_VM_DONE) || (mode == GM_ONLY && (debug_flags & 512u)) ||
                   (prefix && mode == GM_ONLY));
        if (!ok) {
            if (prefix) {
                gd = mxp_guard{0, GM_NONE, 0, 0};
                rule_tmpl[i] = MXP_VM_DONE;
            }
            continue;
        }
        if (mode == GM_ONLY) rule_tmpl[i] = MXP_TMPL_DIRECT;
        indexed[i] = 1;
        P.n_indexed++;
        if (!(debug_flags & 64u)) {
            std::string key((const char*)&gd, sizeof gd);
            key.append((const char*)(all.data() + off[i]), (size_t)(off[i + 1] - off[i]) * sizeof(mxp_vm_ins));
            auto ins = canon_of.emplace(std::move(key), i);
            if (!ins.second) {
                aliases_of[ins.first->second].push_back(i);
                P.n_alias++;
                continue;
            }
        }
        const uint64_t k1 = (uint64_t)gd.klo | ((uint64_t)gd.khi << 32);
        mxp::SecondAtom sa;
        std::vector<mxp_vm_ins> code(all.begin() + off[i], all.begin() + off[i + 1]);
        if (!prefix && mode == GM_AND && !(debug_flags & 16u) && mxp::extract_second_prefix(code, gd.mode >> 16, &sa)) {
            if (sa.direct) {
                rule_tmpl2[i] = MXP_TMPL_DIRECT;
            } else {
                const uint32_t t1 = rule_tmpl[i];
                auto it = tmpl2_ids.find({t1, sa.cont});
                if (it == tmpl2_ids.end()) {
                    mxp_tmpl t = tmpls[t1];
                    t.off += sa.cont - t.pc0;
                    t.pc0 = sa.cont;
                    it = tmpl2_ids.emplace(std::make_pair(t1, sa.cont), (uint32_t)tmpls.size()).first;
                    tmpls.push_back(t);
                }
                rule_tmpl2[i] = it->second;
            }
            comp_of[{gd.col, sa.col}][{k1, sa.k2}].push_back(i);
            if (base) ref_comp.push_back(RefComposite{gd.col & 0xFFFFFFu, sa.col, (uint32_t)k1, i});
            P.n_composite++;
            continue;
        }
        if (!rx_keys_h[i].empty()) {  // a literal-key regexp rule: one posting per key
            for (const auto& k : rx_keys_h[i])
                index_of[{gd.col, true}][k.first].push_back(i | (k.second == 1 ? 1u << 31 : k.second == 2 ? 1u << 30 : 0u));
            continue;
        }
        index_of[{gd.col, prefix}][k1].push_back(i);
    }
    P.n_tmpls = (uint32_t)tmpls.size();
    std::vector<mxp_index> idx;
    std::vector<mxp_hent> hents;
    std::vector<uint32_t> postings, plens;
    // postings carry their rule's continuation template (rule | code << 23; code 511 direct, 510
    // look it up): the index kernel then loads no template id per posting or per pair
    P.post_tmpl = n < (1u << 23);
    // (literal-key regexp rules, n < 2^23: code 509, an exact key -- true only when the subject ends at
    // the key -- for a rule id with bit 31 set in `rs`; code 508, a `.*$` tail key -- true only when
    // no '\n' follows the key in the subject -- for bit 30)
    auto rid = [&](uint32_t r) { return r & (P.post_tmpl ? 0x3FFFFFFFu : 0x7FFFFFFFu); };
    auto post = [&](const std::vector<uint32_t>& rs, const std::vector<uint32_t>& tmpl_of) -> uint32_t {  // postings emitted
        const size_t p0 = postings.size();
        for (uint32_t r : rs) {
            const uint32_t rr = rid(r), t = tmpl_of[rr];
            const uint32_t code = (r >> 31) ? 509u : ((r >> 30) & 1u) ? 508u : t == MXP_TMPL_DIRECT ? 511u : t < 508u ? t : 510u;
            postings.push_back(!P.post_tmpl ? rr : rr | code << 23);
        }
        return (uint32_t)std::min<size_t>(postings.size() - p0, 0xFFFFFFFFu);
    };
    // slots of a table of n keys: >= 2^(1 + index_sparsity) per key (mxp_engine.index_sparsity), the
    // growth past 2 per key stopping at 2^20 slots per table and 2^24 entries (256 MB) over all tables
    auto table_cap = [&](size_t n) -> uint32_t {
        uint32_t cap = 1;
        while (cap < 2 * n ||
               (cap < (2ull << index_sparsity) * n && cap < (1u << 20) && hents.size() + 4ull * cap <= (1ull << 24)))
            cap <<= 1;
        return cap;
    };
    // open-addressing table of `groups` (key -> rules) at hents[hoff ..): returns hmask
    auto add_eq_table = [&](const std::map<uint64_t, std::vector<uint32_t>>& groups, const std::vector<uint32_t>& tmpl_of,
                            uint32_t* hoff) -> uint32_t {
        const uint32_t cap = table_cap(groups.size());
        *hoff = (uint32_t)hents.size();
        hents.resize(hents.size() + cap, mxp_hent{0, 0, 0, 0});
        for (auto& kv : groups) {
            std::vector<uint32_t> rs = kv.second;
            std::stable_sort(rs.begin(), rs.end(), [&](uint32_t a, uint32_t b) { return tmpl_of[a] < tmpl_of[b]; });
            uint32_t h = mxp_hash64(kv.first) & (cap - 1);
            while (hents[*hoff + h].len) h = (h + 1) & (cap - 1);
            const uint32_t start = (uint32_t)postings.size();
            hents[*hoff + h] = mxp_hent{(uint32_t)kv.first, (uint32_t)(kv.first >> 32), start, post(rs, tmpl_of)};
        }
        return cap - 1;
    };
    for (auto& ci : index_of) {
        const bool prefix = ci.first.second;
        mxp_index x{};
        x.col = ci.first.first & 0xFFFFFFu;
        x.okset = okset_of(ci.first.first >> 24);
        x.prefix = prefix ? MXP_IX_PREFIX : MXP_IX_EQ;
        if (!prefix) {
            x.hmask = add_eq_table(ci.second, rule_tmpl, &x.hoff);
            idx.push_back(x);
            continue;
        }
        const uint32_t cap = table_cap(ci.second.size());
        x.hmask = cap - 1;
        x.hoff = (uint32_t)hents.size();
        hents.resize(hents.size() + 2 * (size_t)cap, mxp_hent{0, 0, 0, 0});
        std::set<uint32_t> lens;
        for (auto& kv : ci.second) {
            std::vector<uint32_t> rs = kv.second;
            std::stable_sort(rs.begin(), rs.end(), [&](uint32_t a, uint32_t b) {
                return rule_tmpl[rid(a)] < rule_tmpl[rid(b)];
            });
            for (uint32_t r : rs) x.tailk |= P.post_tmpl && ((r >> 30) & 3u) == 1u;
            // hash of the key bytes, as the kernel hashes the request's leading bytes
            const std::string& key = gstrs[(uint32_t)kv.first];
            lens.insert((uint32_t)key.size());
            const uint64_t hh = mxp_str_hash((const uint8_t*)key.data(), key.size());
            uint32_t h = (uint32_t)hh & x.hmask;
            while (hents[x.hoff + 2 * h].len) h = (h + 1) & x.hmask;
            // (vm.h mxp_index: entry pairs; a key of <= 20 bytes rides inline -- bytes 0..3 in the first
            // entry's klo, 4..19 in the second entry -- so a probe verifies it with no key-string loads;
            // longer keys keep their string id; the key length sits in the top byte of the count)
            uint32_t kw[5] = {0, 0, 0, 0, 0};
            const bool inl = key.size() <= 20;
            if (inl) memcpy(kw, key.data(), key.size());
            const uint32_t start = (uint32_t)postings.size(), cnt = post(rs, rule_tmpl);
            if (cnt >= (1u << 24)) return fail(MXP_ERR_NOMEM, "prefix posting list too long");
            hents[x.hoff + 2 * h] = mxp_hent{inl ? kw[0] : (uint32_t)kv.first, (uint32_t)(hh >> 32), start,
                                             cnt | ((uint32_t)std::min<size_t>(key.size(), 255) << 24)};
            hents[x.hoff + 2 * h + 1] = mxp_hent{kw[1], kw[2], kw[3], kw[4]};
        }
        x.plen0 = (uint32_t)plens.size();
        x.nplen = (uint32_t)lens.size();
        plens.insert(plens.end(), lens.begin(), lens.end());
        idx.push_back(x);
    }
    for (auto& ci : comp_of) {
        mxp_index x{};
        x.col = ci.first.first & 0xFFFFFFu;
        x.okset = okset_of(ci.first.first >> 24);
        x.prefix = MXP_IX_COMPOSITE;
        x.col2 = ci.first.second;
        x.okset2 = okset_of(W_S);
        // fallback equality table over K1 (B not a string): every rule of the key, continuation after A
        std::map<uint64_t, std::vector<uint32_t>> by_k1;
        for (auto& kv : ci.second) {
            auto& v = by_k1[kv.first.first];
            v.insert(v.end(), kv.second.begin(), kv.second.end());
        }
        for (auto& kv : by_k1) std::sort(kv.second.begin(), kv.second.end());
        x.hmask = add_eq_table(by_k1, rule_tmpl, &x.hoff);
        // composite table: entry pairs
        const uint32_t cap = table_cap(ci.second.size());
        x.hmask2 = cap - 1;
        x.hoff2 = (uint32_t)hents.size();
        hents.resize(hents.size() + 2 * (size_t)cap, mxp_hent{0, 0, 0, 0});
        std::set<uint32_t> lens;
        for (auto& kv : ci.second) {
            std::vector<uint32_t> rs = kv.second;
            std::stable_sort(rs.begin(), rs.end(), [&](uint32_t a, uint32_t b) { return rule_tmpl2[a] < rule_tmpl2[b]; });
            const uint64_t k1 = kv.first.first;
            const std::string& key = gstrs[kv.first.second];
            lens.insert((uint32_t)key.size());
            const uint64_t hh = mxp_str_hash_seeded(mxp_composite_seed(k1), (const uint8_t*)key.data(), key.size());
            uint32_t h = (uint32_t)hh & x.hmask2;
            while (hents[x.hoff2 + 2 * h].len) h = (h + 1) & x.hmask2;
            // (vm.h MXP_COMP_*: a key of <= 12 bytes rides inline in the pair -- bytes 0..3 in the
            // first entry's klo, 4..11 in the second's start / len -- so a probe verifies it with
            // no key-string loads; longer keys keep their string id; the key length sits in the top
            // byte of the posting count, 255 for 255 bytes and more)
            if (rs.size() >= (1u << 24)) return fail(MXP_ERR_NOMEM, "composite posting list too long");
            uint32_t kw[3] = {0, 0, 0};
            if (key.size() <= 12) memcpy(kw, key.data(), key.size());
            const uint32_t start = (uint32_t)postings.size();
            post(rs, rule_tmpl2);  // (no expansion: the composite table's own templates)
            hents[x.hoff2 + 2 * h] = mxp_hent{key.size() <= 12 ? kw[0] : kv.first.second, (uint32_t)(hh >> 32),
                                              start, (uint32_t)rs.size() | ((uint32_t)std::min<size_t>(key.size(), 255) << 24)};
            hents[x.hoff2 + 2 * h + 1] = mxp_hent{(uint32_t)k1, (uint32_t)(k1 >> 32), kw[1], kw[2]};
        }
        x.plen0 = (uint32_t)plens.size();
        x.nplen = (uint32_t)lens.size();
        plens.insert(plens.end(), lens.begin(), lens.end());
        idx.push_back(x);
    }
    // lite index kernel: no template the postings can run (code from its start to its end) holds a
    // heavy opcode -- templates of rules this plan serves otherwise (value classes) or that became
    // direct postings (literal-key regexps) do not count
    {
        std::vector<uint8_t> used(tmpls.size(), P.post_tmpl ? 0 : 1);
        auto use = [&](uint32_t t) {
            if (t < used.size()) used[t] = 1;
        };
        if (P.post_tmpl)
            for (uint32_t pe : postings) {
                const uint32_t code = pe >> 23, r = pe & 0x7FFFFFu;
                if (code < 508u) use(code);
                if (code == 510u) {  // (either table's template: the posting does not say which)
                    use(rule_tmpl[r]);
                    use(rule_tmpl2[r]);
                }
            }
        P.tmpl_lite = !(debug_flags & 8388608u);
        for (uint32_t i = 0; i < tmpls.size() && P.tmpl_lite; i++) {
            if (!used[i]) continue;
            const mxp_tmpl& t = tmpls[i];
            for (uint32_t pc = t.pc0; pc < t.len && P.tmpl_lite; pc++) {
                const uint32_t op = prog_h[t.off - t.pc0 + pc].op & 0x7Fu;
                if (op == VM_VCOL || op == VM_LOOKUP || op == VM_LOOKUPK || op == VM_REGEX || op == VM_REGEXR || op == VM_REGEXD)
                    P.tmpl_lite = false;
            }
        }
    }
    // string heads: plan 0 assigns a row to every column its prefix / composite indexes probe (the
    // other plans leave value-class rules out, so their indexes probe a subset of those columns)
    if (base) {
        head_cols.clear();
        head_slot_of.assign(cols.size() + vcols.size(), MXP_VM_DONE);
    }
    for (mxp_index& x : idx) {
        x.hslot = MXP_VM_DONE;
        if (x.prefix == MXP_IX_EQ || x.tailk) continue;  // (`.*$` tail keys look at the whole subject)
        const uint32_t c = x.prefix == MXP_IX_COMPOSITE ? x.col2 : x.col;
        if (c >= head_slot_of.size()) continue;
        if (base && head_slot_of[c] == MXP_VM_DONE) {
            head_slot_of[c] = (uint32_t)head_cols.size();
            head_cols.push_back(c);
        }
        x.hslot = head_slot_of[c];
    }
    P.n_idx = (uint32_t)idx.size();
    std::vector<uint32_t> alias_off(P.n_alias ? n + 1 : 0, 0), alias_list;
    if (P.n_alias) {
        for (uint32_t i = 0; i < n; i++) {
            alias_off[i] = (uint32_t)alias_list.size();
            alias_list.insert(alias_list.end(), aliases_of[i].begin(), aliases_of[i].end());
        }
        alias_off[n] = (uint32_t)alias_list.size();
    }

    // value-class merge entries: per group the (active slot, word position) pairs of the rules the
    // value classes serve; per active slot its words (group, rule mask) for mxp_vt_eval_kernel
    const uint32_t W = (n + 31) / 32;
    P.vt_cols.clear();
    std::vector<uint32_t> act_of(vt_cand_col.size(), MXP_VM_DONE);
    for (uint32_t s = 0; s < vt_cand_col.size(); s++)
        if ((P.mask >> s) & 1u) {
            act_of[s] = (uint32_t)P.vt_cols.size();
            P.vt_cols.push_back(vt_cand_col[s]);
        }
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> words_of(P.vt_cols.size());  // (group, mask)
    std::vector<uint32_t> gvt_off(W + 1, 0), gvt, gvt_mask(W, 0);
    for (uint32_t g = 0; g < W; g++) {
        gvt_off[g] = (uint32_t)gvt.size();
        std::vector<uint32_t> mk(P.vt_cols.size(), 0);
        for (uint32_t k = 0; k < 32 && g * 32 + k < n; k++)
            if (excluded[g * 32 + k]) mk[act_of[vt_slot_of_rule[g * 32 + k]]] |= 1u << k;
        for (uint32_t a = 0; a < P.vt_cols.size(); a++)
            if (mk[a]) {
                gvt_mask[g] |= 1u << a;
                gvt.push_back((a << 24) | (uint32_t)words_of[a].size());
                words_of[a].push_back({g, mk[a]});
            }
    }
    gvt_off[W] = (uint32_t)gvt.size();
    std::vector<uint32_t> vt_woff(P.vt_cols.size() + 1, 0), vt_words;  // pairs (group, mask)
    P.vt_nw.clear();
    for (uint32_t a = 0; a < P.vt_cols.size(); a++) {
        vt_woff[a] = (uint32_t)vt_words.size() / 2;
        P.vt_nw.push_back((uint32_t)words_of[a].size());
        for (auto& w : words_of[a]) {
            vt_words.push_back(w.first);
            vt_words.push_back(w.second);
        }
    }
    vt_woff[P.vt_cols.size()] = (uint32_t)vt_words.size() / 2;
    P.vt_max_nw = 0;
    for (uint32_t x : P.vt_nw) P.vt_max_nw = std::max(P.vt_max_nw, x);

    // phase-1 group tables: mode masks, column segments, guard constants
    std::vector<mxp_rgroup> groups(W);
    std::vector<mxp_seg> segs;
    std::vector<uint64_t> gk((size_t)W * 32, 0);
    for (uint32_t g = 0; g < W; g++) {
        mxp_rgroup& G = groups[g];
        memset(&G, 0, sizeof G);
        std::vector<mxp_seg> seg_of;
        for (uint32_t k = 0; k < 32 && g * 32 + k < n; k++) {
            const uint32_t r = g * 32 + k, bit = 1u << k;
            if (excluded[r]) continue;  // served by value classes (gvt)
            const mxp_guard& gd = guards[r];
            const uint32_t mode = gd.mode & 0xFF;
            G.all |= bit;
            if (mode == GM_NONE) continue;
            G.guarded |= bit;
            if (mode == GM_ONLY) G.only |= bit;
            if (mode == GM_OR) G.orm |= bit;
            if ((gd.mode >> 8) & 1) G.neg |= bit;
            if (indexed[r]) G.indexed |= bit;
            gk[r] = (uint64_t)gd.klo | ((uint64_t)gd.khi << 32);
            const uint32_t col = gd.col & 0xFFFFFFu, kind = gd.col >> 24;
            auto sit = std::find_if(seg_of.begin(), seg_of.end(),
                                    [&](const mxp_seg& q) { return q.col == col && (q.okset >> 24) == kind; });
            if (sit == seg_of.end()) {
                seg_of.push_back(mxp_seg{col, okset_of(kind) | (kind << 24), 0, 0});
                sit = seg_of.end() - 1;
            }
            sit->rules |= bit;
            if (!indexed[r]) sit->cmp |= bit;
        }
        G.id = g;
        G.nseg = (uint32_t)seg_of.size();
        G.seg0 = (uint32_t)segs.size();
        if (!seg_of.empty()) {
            G.s_col = seg_of[0].col;
            G.s_okset = seg_of[0].okset;
            G.s_rules = seg_of[0].rules;
            G.s_cmp = seg_of[0].cmp;
            segs.insert(segs.end(), seg_of.begin() + 1, seg_of.end());
        }
        // continuing lanes after phase 1 need the VM: rules without a guard, OR guards, AND guards
        // that are not indexed (ONLY guards and indexed AND guards never continue in-wave)
        const uint32_t andm = G.guarded & ~(G.only | G.orm);
        G.vm = ((G.all & ~G.guarded) | G.orm | (andm & ~G.indexed)) != 0;
    }
    std::vector<uint32_t> glean, gvm, gall, gdeep, fill_masks;
    std::vector<mxp_fill> fills;
    P.n_gfill = 0;
    // groups holding a rule with more live values than MXP_VM_MAXREG (lower.cpp colouring): their
    // VM runs in the kernels with the MXP_VM_DEEPREG register file, in every mode
    std::vector<uint8_t> deep(W, 0);
    for (uint32_t i = 0; i < n; i++)
        if (!excluded[i] && rules[i].low.ok && rules[i].low.nregs > MXP_VM_MAXREG) deep[i / 32] = 1;
    for (uint32_t g = 0; g < W; g++) {
        // (a deep group is never a fill group: the deep kernel's plain stores would erase the fill's
        // merged deferred pairs; deep rules are never templated, hence never indexed, so this only
        // states what hoist_continuation already guarantees)
        (deep[g] ? gdeep : gall).push_back(g);
        const mxp_rgroup& G = groups[g];
        const bool has_vt = gvt_off[g + 1] > gvt_off[g];
        // uniform indexed group: every rule indexed, one guard column, nothing compared in-wave --
        // its words depend only on that column's kind (and the value classes' merge entries); a
        // group the value classes serve entirely joins whatever chunk is open (its mask is 0)
        const bool only_vt = G.all == 0 && has_vt;
        const bool uniform = !G.vm && (only_vt || (G.all && G.indexed == G.all && G.guarded == G.all && G.nseg == 1 &&
                                                   G.s_cmp == 0 && G.s_rules == G.all)) &&
                             !deep[g] && !(debug_flags & 32u);
        if (uniform) {
            mxp_fill* F = fills.empty() ? nullptr : &fills.back();
            const bool joins = F && F->g0 + F->n == g && F->n < fill_chunk &&
                               (only_vt || (F->col == G.s_col && F->okset == G.s_okset) || F->okset == 0xFFFFu);
            if (joins) {
                if (!only_vt && F->okset == 0xFFFFu) {  // a chunk of value-class-only groups adopts a column
                    F->col = G.s_col;
                    F->okset = G.s_okset;
                }
                F->n++;
            } else {
                mxp_fill f{};
                f.col = only_vt ? 0u : G.s_col;
                f.okset = only_vt ? 0xFFFFu : G.s_okset;  // (every kind passes: no guard to type-check)
                f.g0 = g;
                f.n = 1;
                f.moff = (uint32_t)fill_masks.size();
                fills.push_back(f);
                F = &fills.back();
            }
            fill_masks.push_back(G.all);
            F->vt |= has_vt ? 1u : 0u;
            P.n_gfill++;
            continue;
        }
        // the lean kernels carry no value-class merge: such groups go to the VM kernel
        if (deep[g]) continue;
        (G.vm || has_vt ? gvm : glean).push_back(g);
    }
    // chunks with value-class merge entries go to mxp_vtfill_kernel
    std::vector<mxp_fill> vtfills;
    {
        std::vector<mxp_fill> plain;
        for (auto& f : fills) (f.vt ? vtfills : plain).push_back(f);
        fills.swap(plain);
    }
    P.n_fills = (uint32_t)fills.size();
    P.n_vtfills = (uint32_t)vtfills.size();
    P.n_glean = (uint32_t)glean.size();
    // columns < MXP_CC the lean groups read: mxp_guard2_kernel loads them into LDS up front
    P.lean_cc = 0;
    for (uint32_t g : glean) {
        const mxp_rgroup& G = groups[g];
        if (G.nseg && G.s_col < MXP_CC) P.lean_cc |= 1u << G.s_col;
        for (uint32_t k = 0; k + 1 < G.nseg; k++)
            if (segs[G.seg0 + k].col < MXP_CC) P.lean_cc |= 1u << segs[G.seg0 + k].col;
    }
    P.n_gvm = (uint32_t)gvm.size();
    P.n_gall = (uint32_t)gall.size();
    P.n_gdeep = (uint32_t)gdeep.size();
    P.n_segs = (uint32_t)segs.size();

    // dense canonical rules: indexed rules with many duplicates, true pairs injected per bitmap word
    // at the end of the index kernel instead of one atomic per alias (kernels.hip inject_dense)
    std::vector<uint8_t> dense_of;
    std::vector<uint32_t> inj;
    {
        std::vector<uint32_t> cand;
        // (direct postings -- `attr.startsWith(K)` alone -- stay with per-alias atomics: their true
        // pairs are sparse, and C4 measured them slower injected)
        for (uint32_t i = 0; i < n; i++)
            if (aliases_of[i].size() + 1 >= kDenseMin && rule_tmpl[i] != MXP_TMPL_DIRECT) cand.push_back(i);
        std::stable_sort(cand.begin(), cand.end(),
                         [&](uint32_t a, uint32_t b) { return aliases_of[a].size() > aliases_of[b].size(); });
        if (cand.size() > 64) cand.resize(64);
        if (debug_flags & 256u) cand.clear();  // ablation: fan out with atomics
        dense_of.assign(n, 0xFF);
        std::map<uint32_t, std::vector<uint32_t>> by_word;
        for (uint32_t d = 0; d < cand.size(); d++) {
            dense_of[cand[d]] = (uint8_t)d;
            by_word[cand[d] >> 5].push_back((cand[d] & 31u) | (d << 5));
            for (uint32_t a : aliases_of[cand[d]]) by_word[a >> 5].push_back((a & 31u) | (d << 5));
        }
        for (auto& kv : by_word)
            for (size_t e0 = 0; e0 < kv.second.size(); e0 += MXP_INJ_SLOT - 4) {
                const size_t e1 = std::min(kv.second.size(), e0 + MXP_INJ_SLOT - 4);
                uint32_t slot[MXP_INJ_SLOT] = {};
                uint64_t dm = 0;
                for (size_t e = e0; e < e1; e++) {
                    dm |= 1ull << (kv.second[e] >> 5);
                    slot[4 + e - e0] = kv.second[e];
                }
                slot[0] = (uint32_t)dm;
                slot[1] = (uint32_t)(dm >> 32);
                slot[2] = kv.first;
                slot[3] = (uint32_t)(e1 - e0);
                inj.insert(inj.end(), slot, slot + MXP_INJ_SLOT);
            }
        P.n_dense = (uint32_t)cand.size();
        P.n_inj = P.n_dense ? (uint32_t)(inj.size() / MXP_INJ_SLOT) : 0u;
    }
    // deferred index pairs: every group holding an indexed rule (or an alias of one) must be a
    // fill or value-class fill group -- the writers that merge them
    // (chunk ids: the plain fill chunks, then the value-class ones)
    std::vector<uint32_t> dtp_chunk(W, 0xFFFFFFFFu);
    {
        bool ok = (!fills.empty() || !vtfills.empty()) && P.n_dense == 0 && n < (1u << 23);
        const uint32_t nf = (uint32_t)fills.size();
        for (uint32_t c = 0; ok && c < nf + vtfills.size(); c++) {
            const mxp_fill& F = c < nf ? fills[c] : vtfills[c - nf];
            if (F.n > 255u || c >= (1u << 24)) ok = false;  // (group 255: the queue's pad)
            for (uint32_t k = 0; ok && k < F.n; k++) dtp_chunk[F.g0 + k] = c << 8 | k;
        }
        for (uint32_t g = 0; ok && g < W; g++)
            if (groups[g].indexed && dtp_chunk[g] == 0xFFFFFFFFu) ok = false;
        P.dtp_ok = ok && P.n_indexed > 0;
    }
    if (base) {
        ref_alias_off.assign(n + 1, 0);
        ref_aliases.clear();
        for (uint32_t i = 0; i < n; i++) {
            ref_aliases.insert(ref_aliases.end(), aliases_of[i].begin(), aliases_of[i].end());
            ref_alias_off[i + 1] = (uint32_t)ref_aliases.size();
        }
    }
    if (device < 0) return MXP_OK;  // host-only engine: compile / inspect, no device tables

    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return hipfail(e, "hipSetDevice");
    auto put = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return hipfail(e, what);
        if (bytes && (e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess) return hipfail(e, what);
        return MXP_OK;
    };
    int rc;
    if ((rc = put(P.d_guards, guards.data(), guards.size() * sizeof(mxp_guard), "upload guards"))) return rc;
    if ((rc = put(P.d_groups, groups.data(), groups.size() * sizeof(mxp_rgroup), "upload groups"))) return rc;
    if ((rc = put(P.d_segs, segs.data(), segs.size() * sizeof(mxp_seg), "upload segs"))) return rc;
    if ((rc = put(P.d_glean, glean.data(), glean.size() * 4, "upload glean"))) return rc;
    if ((rc = put(P.d_fills, fills.data(), fills.size() * sizeof(mxp_fill), "upload fills"))) return rc;
    if ((rc = put(P.d_vtfills, vtfills.data(), vtfills.size() * sizeof(mxp_fill), "upload vtfills"))) return rc;
    if ((rc = put(P.d_dtp_chunk, dtp_chunk.data(), dtp_chunk.size() * 4, "upload dtp chunks"))) return rc;
    if ((rc = put(P.d_fill_masks, fill_masks.data(), fill_masks.size() * 4, "upload fill masks"))) return rc;
    if ((rc = put(P.d_gvm, gvm.data(), gvm.size() * 4, "upload gvm"))) return rc;
    if ((rc = put(P.d_gall, gall.data(), gall.size() * 4, "upload gall"))) return rc;
    if ((rc = put(P.d_gdeep, gdeep.data(), gdeep.size() * 4, "upload gdeep"))) return rc;
    if ((rc = put(P.d_gk, gk.data(), gk.size() * 8, "upload gk"))) return rc;
    // occupancy bitmaps of the pair tables: most probes of a key length end at an empty slot, which
    // one bit of a small, L1-resident array tells without the entry pair's L2 request
    std::vector<uint32_t> hbits;
    for (mxp_index& x : idx) {
        if (x.prefix == MXP_IX_EQ) continue;
        const uint32_t off = x.prefix == MXP_IX_COMPOSITE ? x.hoff2 : x.hoff;
        const uint32_t cap = (x.prefix == MXP_IX_COMPOSITE ? x.hmask2 : x.hmask) + 1u;
        x.boff = (uint32_t)hbits.size();
        hbits.resize(hbits.size() + (cap + 31u) / 32u, 0u);
        for (uint32_t sl = 0; sl < cap; sl++)
            if (hents[off + 2ull * sl].len) hbits[x.boff + sl / 32u] |= 1u << (sl % 32u);
    }
    if ((rc = put(P.d_idx, idx.data(), idx.size() * sizeof(mxp_index), "upload idx"))) return rc;
    if ((rc = put(P.d_hbits, hbits.data(), hbits.size() * 4, "upload hbits"))) return rc;
    if ((rc = put(P.d_hents, hents.data(), hents.size() * sizeof(mxp_hent), "upload hents"))) return rc;
    if ((rc = put(P.d_postings, postings.data(), postings.size() * 4, "upload postings"))) return rc;
    if ((rc = put(P.d_plens, plens.data(), plens.size() * 4, "upload plens"))) return rc;
    if ((rc = put(P.d_tmpls, tmpls.data(), tmpls.size() * sizeof(mxp_tmpl), "upload tmpls"))) return rc;
    if ((rc = put(P.d_rule_tmpl, rule_tmpl.data(), rule_tmpl.size() * 4, "upload rule_tmpl"))) return rc;
    if ((rc = put(P.d_rule_tmpl2, rule_tmpl2.data(), rule_tmpl2.size() * 4, "upload rule_tmpl2"))) return rc;
    if ((rc = put(P.d_alias_off, alias_off.data(), alias_off.size() * 4, "upload alias_off"))) return rc;
    if ((rc = put(P.d_aliases, alias_list.data(), alias_list.size() * 4, "upload aliases"))) return rc;
    if ((rc = put(P.d_dense_of, dense_of.data(), dense_of.size(), "upload dense_of"))) return rc;
    if ((rc = put(P.d_inj, inj.data(), inj.size() * 4, "upload inj"))) return rc;
    if ((rc = put(P.d_gvt_off, gvt_off.data(), gvt_off.size() * 4, "upload gvt_off"))) return rc;
    if ((rc = put(P.d_gvt, gvt.data(), gvt.size() * 4, "upload gvt"))) return rc;
    if ((rc = put(P.d_gvt_mask, gvt_mask.data(), gvt_mask.size() * 4, "upload gvt mask"))) return rc;
    if ((rc = put(P.d_vt_woff, vt_woff.data(), vt_woff.size() * 4, "upload vt_woff"))) return rc;
    if ((rc = put(P.d_vt_words, vt_words.data(), vt_words.size() * 4, "upload vt_words"))) return rc;
    return MXP_OK;
}

// ---------------------------------------------------------------------------------------- pack
void mxp_engine::build_views() {
    // string-view indexes of the rule set's interning tables (rebuilt when a compile grew them:
    // the vectors may have moved their strings)
    if (views_n[0] == gstrs.size() && views_n[1] == gbytes.size() && views_n[2] == gcanon.size()) return;
    auto build = [](const std::vector<std::string>& v, mxp::SvMap& m) {
        m.clear();
        m.reserve(v.size() * 2);
        for (size_t i = 0; i < v.size(); i++) m.emplace(std::string_view(v[i]), (uint32_t)i);
    };
    build(gstrs, gstr_view);
    build(gbytes, gbytes_view);
    build(gcanon, gcanon_view);
    views_n[0] = gstrs.size();
    views_n[1] = gbytes.size();
    views_n[2] = gcanon.size();
}

// Host half of packing (mxp_batch_upload): the caller's columnar batch -> the engine's device
// columns.  Batch strings are interned against the rule set's pool (ids < G) or a per-batch overlay
// in four passes: (1) mark the batch strings the rule set's columns reach, (2) look them up in the
// rule set's tables in parallel, (3) assign overlay ids to the misses in batch-string order
// (sequential, deterministic), (4) gather the columns in parallel.
int mxp_engine::pack_host(const mxp_bag_batch* b, mxp_dbatch* db, PackedHost& H) {
    const uint32_t n = b->n_requests;
    const uint32_t C = (uint32_t)cols.size(), V = (uint32_t)vcols.size();
    const uint32_t ncol = C + V;
    db->n = n;
    build_views();
    std::unordered_map<std::string, uint32_t> bcol;
    for (uint32_t c = 0; c < b->n_columns; c++) bcol.emplace(b->column_names[c], c);
    std::vector<int32_t> src(ncol, -1);  // batch column of each engine column
    for (uint32_t c = 0; c < ncol; c++) {
        auto it = bcol.find(c < C ? cols[c] : vcols[c - C].first);
        if (it != bcol.end()) src[c] = (int32_t)it->second;
    }
    const uint32_t NS = b->n_strings;
    auto view = [&](uint64_t sid) {
        return std::string_view((const char*)b->str_bytes + b->str_offsets[sid],
                                (size_t)(b->str_offsets[sid + 1] - b->str_offsets[sid]));
    };
    // ---- (1) usage marks: 1 = string value, 2 = bytes value
    std::vector<uint8_t> use(NS, 0);
    auto mark = [&](uint64_t sid, uint8_t bit) {
        if (sid < NS) __atomic_fetch_or(&use[sid], bit, __ATOMIC_RELAXED);
    };
    // virtual map[key] columns: the matching entry's value string (per request, ~0 = key absent)
    std::vector<uint32_t> vhit((size_t)V * n, MXP_VM_DONE);
    mxp::par_for(n, 4096, [&](uint64_t r0, uint64_t r1, unsigned) {
        for (uint32_t c = 0; c < C; c++) {
            if (src[c] < 0) continue;
            const uint8_t* bk = b->kinds[src[c]];
            const uint64_t* bv = b->values[src[c]];
            for (uint64_t r = r0; r < r1; r++) {
                // (OTHER values are interned too: their text is the value of a conversion error)
                if (bk[r] == MXP_STRING || bk[r] == MXP_OTHER) mark(bv[r], 1);
                else if (bk[r] == MXP_BYTES) mark(bv[r], 2);
            }
        }
        for (uint32_t j = 0; j < V; j++) {
            if (src[C + j] < 0) continue;
            const std::string& key = vcols[j].second;
            const uint8_t* bk = b->kinds[src[C + j]];
            const uint64_t* bv = b->values[src[C + j]];
            for (uint64_t r = r0; r < r1; r++) {
                if (bk[r] != MXP_STRING_MAP) continue;
                const uint64_t m = bv[r];
                for (uint64_t e = b->map_offsets[m]; e < b->map_offsets[m + 1]; e++) {
                    if (view(b->map_keys[e]) == key) {
                        vhit[(size_t)j * n + r] = b->map_values[e];
                        mark(b->map_values[e], 1);
                        break;
                    }
                }
            }
        }
    });
    if (need_maps) {
        const uint64_t E = b->n_maps ? b->map_offsets[b->n_maps] : 0;
        mxp::par_for(E, 1 << 14, [&](uint64_t e0, uint64_t e1, unsigned) {
            for (uint64_t e = e0; e < e1; e++) {
                mark(b->map_keys[e], 1);
                mark(b->map_values[e], 1);
            }
        });
    }
    // ---- (2) rule-set pool lookups (+ content hashes of the misses)
    const uint32_t G = (uint32_t)gstrs.size();
    constexpr uint32_t NONE = MXP_VM_DONE;
    std::vector<uint32_t> sid(NS, NONE), braw(NS, NONE), bcan(NS, NONE);
    std::vector<uint64_t> hs(NS, 0), hc;
    bool any_bytes = false;
    for (uint32_t s = 0; s < NS && !any_bytes; s++) any_bytes = use[s] & 2;
    if (any_bytes) hc.assign(NS, 0);
    // net.IP.Equal class of a byte string: 4-byte addresses in their 16-byte v4-mapped form
    auto canon_of = [&](uint64_t s, char* buf) -> std::string_view {
        const std::string_view v = view(s);
        if (v.size() != 4) return v;
        memset(buf, 0, 10);
        buf[10] = buf[11] = (char)0xff;
        memcpy(buf + 12, v.data(), 4);
        return std::string_view(buf, 16);
    };
    mxp::par_for(NS, 2048, [&](uint64_t s0, uint64_t s1, unsigned) {
        char buf[16];
        for (uint64_t s = s0; s < s1; s++) {
            if (!use[s]) continue;
            const std::string_view v = view(s);
            if (use[s] & 1) {
                auto it = gstr_view.find(v);
                if (it != gstr_view.end()) sid[s] = it->second;
            }
            if (use[s] & 2) {
                auto it = gbytes_view.find(v);
                if (it != gbytes_view.end()) braw[s] = it->second;
                const std::string_view c = canon_of(s, buf);
                auto ct = gcanon_view.find(c);
                if (ct != gcanon_view.end()) bcan[s] = ct->second;
                else hc[s] = mxp::hash_bytes(c.data(), c.size());
            }
            if (sid[s] == NONE || braw[s] == NONE) hs[s] = mxp::hash_bytes(v.data(), v.size());
        }
    });
    // ---- (3) overlay ids for the misses: equal strings found in parallel (hash shards), ids
    // assigned in batch-string order of first appearance
    auto assign = [&](std::vector<uint32_t>& out, uint8_t bit, const std::vector<uint64_t>& hash, auto&& eq,
                      auto&& add) {
        std::vector<uint32_t> cand;
        for (uint32_t s = 0; s < NS; s++)
            if ((use[s] & bit) && out[s] == NONE) cand.push_back(s);
        std::vector<uint32_t> rep(cand.size());
        mxp::dedupe_first((uint32_t)cand.size(), [&](uint32_t i) { return hash[cand[i]]; },
                          [&](uint32_t i, uint32_t j) { return eq(cand[i], cand[j]); }, rep);
        for (uint32_t i = 0; i < cand.size(); i++)
            out[cand[i]] = rep[i] == i ? add(cand[i]) : out[cand[rep[i]]];
        return cand.size();
    };
    auto same = [&](uint32_t a, uint32_t b2) { return view(a) == view(b2); };
    bool too_long = false;
    assign(sid, 1, hs, same, [&](uint32_t s) {
        too_long |= !db->overlay.push(view(s));
        return G + (uint32_t)db->overlay.size() - 1;
    });
    if (too_long) return fail(MXP_ERR_ARG, "batch string longer than 16 MiB");
    std::vector<uint32_t> canon_rep;  // overlay canonical classes: a batch string of each
    if (any_bytes) {
        assign(braw, 2, hs, same, [&](uint32_t s) {
            db->overlay_bytes.push(view(s));
            return (uint32_t)(gbytes.size() + db->overlay_bytes.size() - 1);
        });
        assign(bcan, 2, hc, [&](uint32_t a, uint32_t b2) {
            char x[16], y[16];
            return canon_of(a, x) == canon_of(b2, y);
        }, [&](uint32_t s) {
            canon_rep.push_back(s);
            return (uint32_t)(gcanon.size() + canon_rep.size() - 1);
        });
    }
    // bytes ids of strings outside the batch table (parsed ip() values), after the batch's own
    // (maps built on first use; keys view `keep`, a deque: stable addresses)
    std::deque<std::string> keep;
    mxp::SvMap obytes, ocanon;
    bool omaps = false;
    uint32_t n_canon = (uint32_t)canon_rep.size();
    auto bytes_id = [&](const std::string& raw) -> uint64_t {
        if (!omaps) {
            omaps = true;
            for (size_t i = 0; i < db->overlay_bytes.size(); i++)
                obytes.emplace(db->overlay_bytes[i], (uint32_t)(gbytes.size() + i));
            for (size_t i = 0; i < canon_rep.size(); i++) {
                char buf[16];
                keep.emplace_back(canon_of(canon_rep[i], buf));
                ocanon.emplace(std::string_view(keep.back()), (uint32_t)(gcanon.size() + i));
            }
        }
        uint32_t rid, cid;
        auto it = gbytes_view.find(std::string_view(raw));
        if (it != gbytes_view.end()) {
            rid = it->second;
        } else {
            auto jt = obytes.find(std::string_view(raw));
            if (jt != obytes.end()) {
                rid = jt->second;
            } else {
                rid = (uint32_t)(gbytes.size() + db->overlay_bytes.size());
                db->overlay_bytes.push(raw);
                keep.push_back(raw);
                obytes.emplace(std::string_view(keep.back()), rid);
            }
        }
        std::string c = mxp::ip_canonical((const uint8_t*)raw.data(), raw.size());
        auto ct = gcanon_view.find(std::string_view(c));
        if (ct != gcanon_view.end()) {
            cid = ct->second;
        } else {
            auto dt = ocanon.find(std::string_view(c));
            if (dt != ocanon.end()) {
                cid = dt->second;
            } else {
                cid = (uint32_t)gcanon.size() + n_canon++;
                keep.push_back(c);
                ocanon.emplace(std::string_view(keep.back()), cid);
            }
        }
        return MXP_BYTES_ID(cid, rid);
    };
    std::map<TimeKey, uint32_t> otimes;
    auto time_id = [&](int64_t s, int32_t ns) -> uint32_t {
        TimeKey k{s, ns};
        auto it = gtime_ids.find(k);
        if (it != gtime_ids.end()) return it->second;
        auto jt = otimes.find(k);
        if (jt != otimes.end()) return jt->second;
        uint32_t id = (uint32_t)(gtimes.size() + db->overlay_times.size());
        otimes.emplace(k, id);
        db->overlay_times.push_back(k);
        return id;
    };
    // timestamps (sequential: ordered map, rare)
    std::vector<uint32_t> tid(b->n_times, MXP_VM_DONE);
    for (uint32_t c = 0; c < C; c++) {
        if (src[c] < 0) continue;
        const uint8_t* bk = b->kinds[src[c]];
        const uint64_t* bv = b->values[src[c]];
        for (uint32_t r = 0; r < n; r++)
            if (bk[r] == MXP_TIMESTAMP && tid[bv[r]] == MXP_VM_DONE)
                tid[bv[r]] = time_id(b->time_sec[bv[r]], b->time_nsec[bv[r]]);
    }
    // ---- (4) columns
    H.kinds.assign((size_t)ncol * n, 0);
    H.vals.assign((size_t)ncol * n, 0);
    mxp::par_for(n, 4096, [&](uint64_t r0, uint64_t r1, unsigned) {
        for (uint32_t c = 0; c < C; c++) {
            if (src[c] < 0) continue;
            const uint8_t* bk = b->kinds[src[c]];
            const uint64_t* bv = b->values[src[c]];
            uint8_t* ok = H.kinds.data() + (size_t)c * n;
            uint64_t* ov = H.vals.data() + (size_t)c * n;
            for (uint64_t r = r0; r < r1; r++) {
                const uint8_t k = bk[r];
                uint64_t v = bv[r];
                switch (k) {
                case MXP_STRING: case MXP_OTHER: v = sid[v]; break;
                case MXP_BYTES: v = MXP_BYTES_ID(bcan[v], braw[v]); break;
                case MXP_TIMESTAMP: v = tid[v]; break;
                default: break;
                }
                ok[r] = k;
                ov[r] = v;
            }
        }
        for (uint32_t j = 0; j < V; j++) {
            uint8_t* ok = H.kinds.data() + (size_t)(C + j) * n;
            uint64_t* ov = H.vals.data() + (size_t)(C + j) * n;
            if (src[C + j] < 0) continue;  // VC_ABSENT (0)
            const uint8_t* bk = b->kinds[src[C + j]];
            for (uint64_t r = r0; r < r1; r++) {
                const uint8_t k = bk[r];
                if (k == MXP_ABSENT) {
                    ok[r] = VC_ABSENT;
                } else if (k != MXP_STRING_MAP) {
                    ok[r] = VC_NOTMAP;
                } else {
                    ok[r] = VC_VALUE;
                    const uint32_t h = vhit[(size_t)j * n + r];
                    ov[r] = h == MXP_VM_DONE ? empty_sid : sid[h];
                }
            }
        }
    });
    // value classes: the candidate columns with few distinct class keys (mxp_vt_key) in this batch
    // -- distinct string ids by a bitmap over the id space, plus one class per other kind
    db->vt_mask = 0;
    db->vt_capc.assign(vt_cand_col.size(), 0);
    if (!(debug_flags & 131072u) && n) {
        const uint64_t S = G + db->overlay.size();
        uint32_t active = 0;
        std::vector<uint64_t> bits;
        for (uint32_t s = 0; s < vt_cand_col.size() && active < MXP_VT_MAX; s++) {
            const uint32_t c = vt_cand_col[s];
            const uint8_t* kk = H.kinds.data() + (size_t)c * n;
            const uint64_t* vv = H.vals.data() + (size_t)c * n;
            bits.assign(S / 64 + 1, 0);
            uint32_t kmask = 0;
            mxp::par_for(n, 1 << 15, [&](uint64_t r0, uint64_t r1, unsigned) {
                uint32_t km = 0;
                for (uint64_t r = r0; r < r1; r++) {
                    if (kk[r] == 1u) {
                        const uint64_t x = vv[r] < S ? vv[r] : S;
                        if (!(bits[x >> 6] >> (x & 63) & 1u)) __atomic_fetch_or(&bits[x >> 6], 1ull << (x & 63), __ATOMIC_RELAXED);
                    } else {
                        km |= 1u << (kk[r] & 31u);
                    }
                }
                __atomic_fetch_or(&kmask, km, __ATOMIC_RELAXED);
            });
            uint64_t D = (uint64_t)__builtin_popcount(kmask);
            for (uint64_t w : bits) D += (uint64_t)__builtin_popcountll(w);
            const bool force = (debug_flags & 262144u) != 0;  // tests: value classes at any batch size
            if (D > kVtMaxClasses || (!force && D * 16 > n)) continue;
            uint32_t cap = 64;
            while (cap < 2 * D) cap <<= 1;
            db->vt_capc[s] = cap;
            db->vt_mask |= 1u << s;
            active++;
        }
    }
    if (need_maps) {
        H.moff.assign(b->n_maps + 1, 0);
        for (uint32_t m = 0; m < b->n_maps; m++) H.moff[m + 1] = (uint32_t)b->map_offsets[m + 1];
        const uint64_t E = b->n_maps ? b->map_offsets[b->n_maps] : 0;
        H.mk.resize(E);
        H.mv.resize(E);
        mxp::par_for(E, 1 << 14, [&](uint64_t e0, uint64_t e1, unsigned) {
            for (uint64_t e = e0; e < e1; e++) {
                H.mk[e] = sid[b->map_keys[e]];
                H.mv[e] = sid[b->map_values[e]];
            }
        });
    }
    // per-string pre-tables for dynamic ip() / timestamp(): parsed in parallel, interned in order
    const uint64_t S = G + db->overlay.size();
    auto str_at = [&](uint64_t s) -> std::string_view {
        return s < G ? std::string_view(gstrs[s]) : db->overlay[s - G];
    };
    if (need_ipof) {
        H.ipof.assign(S, kNoValue);
        std::vector<std::string> parsed(S);
        mxp::par_for(S, 2048, [&](uint64_t s0, uint64_t s1, unsigned) {
            for (uint64_t s = s0; s < s1; s++) {
                const std::string_view v = str_at(s);
                uint8_t out[16];
                if (mxp::go_parse_ip((const uint8_t*)v.data(), v.size(), out)) parsed[s].assign((const char*)out, 16);
            }
        });
        for (uint64_t s = 0; s < S; s++)
            if (!parsed[s].empty()) H.ipof[s] = MXP_FH(MXP_BYTES, bytes_id(parsed[s]));
    }
    if (need_tsof) {
        H.tsof.assign(S, kNoValue);
        std::vector<std::pair<int64_t, int32_t>> ts(S);
        std::vector<uint8_t> ok(S, 0);
        mxp::par_for(S, 2048, [&](uint64_t s0, uint64_t s1, unsigned) {
            for (uint64_t s = s0; s < s1; s++) {
                const std::string_view v = str_at(s);
                ok[s] = mxp::go_parse_rfc3339((const uint8_t*)v.data(), v.size(), &ts[s].first, &ts[s].second);
            }
        });
        for (uint64_t s = 0; s < S; s++)
            if (ok[s]) H.tsof[s] = MXP_FH(MXP_TIMESTAMP, time_id(ts[s].first, ts[s].second));
    }
    // run-time regexp patterns: every distinct string a pattern can take in this batch (pattern
    // columns, map values, constants; lower.cpp provenance), compiled once per batch
    if (need_rxof) {
        H.rxof.assign(S, MXP_RXOF_SYNTAX);
        std::vector<uint8_t> done(S, 0);
        auto add = [&](uint64_t id) {
            if (id >= S || done[id]) return;
            done[id] = 1;
            mxp::Dfa d;
            std::string e;
            const int rc = mxp::regex_compile({std::string(str_at(id))}, kRegexStates, &d, &e);
            H.rxof[id] = rc == mxp::RX_OK ? H.rxb.add(d) : rc == mxp::RX_SYNTAX ? MXP_RXOF_SYNTAX : MXP_RXOF_UNSUPPORTED;
        };
        for (uint32_t c : rx_pattern_cols()) {
            const uint8_t* k = H.kinds.data() + (size_t)c * n;
            const uint64_t* v = H.vals.data() + (size_t)c * n;
            for (uint32_t q = 0; q < n; q++)
                if (k[q] == MXP_STRING) add(v[q]);  // (VC_VALUE == MXP_STRING for virtual columns)
        }
        for (uint32_t c : rx_mapcols) {
            const uint8_t* k = H.kinds.data() + (size_t)c * n;
            const uint64_t* v = H.vals.data() + (size_t)c * n;
            for (uint32_t q = 0; q < n; q++)
                if (k[q] == MXP_STRING_MAP)
                    for (uint32_t e = H.moff[v[q]]; e < H.moff[v[q] + 1]; e++) add(H.mv[e]);
        }
        for (uint32_t sid_c : rx_consts) add(sid_c);
    }
    db->overlay.finish();
    return MXP_OK;
}

int mxp_engine::pack_on_host(const mxp_bag_batch* b, mxp_dbatch* db) {
    PackedHost H;
    int rc = pack_host(b, db, H);
    if (rc) return rc;
    auto& kinds = H.kinds;
    auto& vals = H.vals;
    auto& moff = H.moff;
    auto& mk = H.mk;
    auto& mv = H.mv;
    auto& ipof = H.ipof;
    auto& tsof = H.tsof;
    const std::vector<uint64_t> no_off;
    const std::string no_blob;
    const auto& ooff = need_strings ? db->overlay.desc : no_off;
    const auto& oblob = need_strings ? db->overlay.blob : no_blob;
    auto& rxof = H.rxof;
    auto& rxb = H.rxb;
    hipError_t e;
    auto up = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes)) != hipSuccess) return hipfail(e, what);
        if (bytes && (e = hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, stream)) != hipSuccess)
            return hipfail(e, what);
        return MXP_OK;
    };
    if ((rc = up(db->kinds, kinds.data(), kinds.size(), "upload kinds"))) return rc;
    if ((rc = up(db->vals, vals.data(), vals.size() * 8, "upload vals"))) return rc;
    if ((rc = up(db->map_off, moff.data(), moff.size() * 4, "upload map_off"))) return rc;
    if ((rc = up(db->map_keys, mk.data(), mk.size() * 4, "upload map_keys"))) return rc;
    if ((rc = up(db->map_vals, mv.data(), mv.size() * 4, "upload map_vals"))) return rc;
    if ((rc = up(db->ipof, ipof.data(), ipof.size() * 8, "upload ipof"))) return rc;
    if ((rc = up(db->tsof, tsof.data(), tsof.size() * 8, "upload tsof"))) return rc;
    if ((rc = up(db->bstr_off, ooff.data(), ooff.size() * 8, "upload bstr_off"))) return rc;
    if ((rc = up(db->bstr, oblob.data(), oblob.size(), "upload bstr"))) return rc;
    if ((rc = up(db->rxof, rxof.data(), rxof.size() * 4, "upload rxof"))) return rc;
    db->rx_nfa = rxb.has_nfa();
    db->rx_wmax = rxb.nfa_wmax();
    if ((rc = up(db->rx_hdr, rxb.hdr.data(), rxb.hdr.size() * sizeof(mxp_dfa_hdr), "upload rx hdr"))) return rc;
    if ((rc = up(db->rx_trans, rxb.trans.data(), rxb.trans.size() * 4, "upload rx trans"))) return rc;
    if ((rc = up(db->rx_ascii, rxb.ascii.data(), rxb.ascii.size() * 2, "upload rx ascii"))) return rc;
    if ((rc = up(db->rx_hilo, rxb.hilo.data(), rxb.hilo.size() * 4, "upload rx hilo"))) return rc;
    if ((rc = up(db->rx_hicls, rxb.hicls.data(), rxb.hicls.size() * 2, "upload rx hicls"))) return rc;
    if ((rc = pack_vt_tables(db))) return rc;
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, "pack sync");
    return MXP_OK;
}

int mxp_engine::pack_vt_tables(mxp_dbatch* db) {
    if (!db->vt_mask) return MXP_OK;  // value-class tables of the batch's active columns
    hipError_t e;
    uint64_t keys = 0;
    for (uint32_t c : db->vt_capc) keys += c;
    db->vt_keys_n = keys;
    const uint32_t act = (uint32_t)__builtin_popcount(db->vt_mask);
    if ((e = db->vt_cls.alloc((size_t)act * MXP_VT_PITCH(db->n) * 2)) != hipSuccess) return hipfail(e, "vt classes");
    if ((e = db->vt_keys.alloc(keys * 8)) != hipSuccess) return hipfail(e, "vt keys");
    if ((e = db->vt_rep.alloc(keys * 4)) != hipSuccess) return hipfail(e, "vt reps");
    if ((e = db->vt_cnt.alloc(keys * 4)) != hipSuccess) return hipfail(e, "vt counts");
    return MXP_OK;
}

// texts of a device-packed batch's local ids, read back from the device
bool mxp_dbatch::overlay_string(uint64_t j, std::string* out) const {
    wait_packed();
    if (!dev_packed) {
        if (j >= overlay.size()) return false;
        *out = std::string(overlay[j]);
        return true;
    }
    if (j >= ns) return false;
    uint64_t d = 0;
    if (hipMemcpy(&d, bstr_off.as<uint64_t>() + j, 8, hipMemcpyDeviceToHost) != hipSuccess) return false;
    out->assign((size_t)(d & 0xFFFFFFu), '\0');
    return out->empty() || hipMemcpy(&(*out)[0], bstr.as<uint8_t>() + (d >> 24), out->size(), hipMemcpyDeviceToHost) == hipSuccess;
}

bool mxp_dbatch::overlay_bytes_at(uint64_t j, std::string* out) const {
    wait_packed();
    if (!dev_packed) {
        if (j >= overlay_bytes.size()) return false;
        *out = std::string(overlay_bytes[j]);
        return true;
    }
    if (j < ns) return overlay_string(j, out);  // a batch string used as bytes
    const uint64_t q = j - ns;                  // a parsed ip() value
    if (q >= (uint64_t)G + ns) return false;
    out->assign(16, '\0');
    return hipMemcpy(&(*out)[0], pip.as<uint8_t>() + 16 * q, 16, hipMemcpyDeviceToHost) == hipSuccess;
}

bool mxp_dbatch::overlay_time(uint64_t j, TimeKey* out) const {
    wait_packed();
    if (!dev_packed) {
        if (j >= overlay_times.size()) return false;
        *out = overlay_times[j];
        return true;
    }
    const int64_t* sec = btsec.as<int64_t>();
    const int32_t* nsec = btnsec.as<int32_t>();
    uint64_t k = j;
    if (j >= nt) {  // a parsed timestamp() value
        k = j - nt;
        if (k >= (uint64_t)G + ns) return false;
        sec = pts_sec.as<int64_t>();
        nsec = pts_nsec.as<int32_t>();
    }
    int64_t s = 0;
    int32_t x = 0;
    if (hipMemcpy(&s, sec + k, 8, hipMemcpyDeviceToHost) != hipSuccess) return false;
    if (hipMemcpy(&x, nsec + k, 4, hipMemcpyDeviceToHost) != hipSuccess) return false;
    *out = TimeKey{s, x};
    return true;
}

void mxp_engine::fill_args(mxp_kargs* A, const mxp_dbatch* db, const Plan& P) const {
    memset(A, 0, sizeof *A);
    A->prog = d_prog.as<mxp_vm_ins>();
    A->rule_off = d_rule_off.as<uint32_t>();
    A->guards = P.d_guards.as<mxp_guard>();
    A->groups = P.d_groups.as<mxp_rgroup>();
    A->segs = P.d_segs.as<mxp_seg>();
    A->gk = P.d_gk.as<uint64_t>();
    A->idx = P.d_idx.as<mxp_index>();
    A->hents = P.d_hents.as<mxp_hent>();
    A->hbits = (debug_flags & 4u) || !P.d_hbits.p ? nullptr : P.d_hbits.as<uint32_t>();
    A->postings = P.d_postings.as<uint32_t>();
    A->post_tmpl = P.post_tmpl ? 1u : 0u;
    A->tmpl_lite = P.tmpl_lite ? 1u : 0u;
    A->plens = P.d_plens.as<uint32_t>();
    A->n_idx = P.n_idx;
    A->tmpls = P.d_tmpls.as<mxp_tmpl>();
    A->rule_tmpl = P.d_rule_tmpl.as<uint32_t>();
    A->rule_tmpl2 = P.d_rule_tmpl2.as<uint32_t>();
    A->alias_off = P.n_alias ? P.d_alias_off.as<uint32_t>() : nullptr;
    A->aliases = P.d_aliases.as<uint32_t>();
    A->dense_of = P.n_dense ? P.d_dense_of.as<uint8_t>() : nullptr;
    A->inj = P.d_inj.as<uint32_t>();
    A->n_inj = P.n_inj;
    A->fill_masks = P.d_fill_masks.as<uint32_t>();
    A->rconst = d_rconst.as<uint64_t>();
    A->flags = debug_flags;
    A->fill_span = fill_span;
    A->lean_cols = P.lean_cc;
    A->n_rules = (uint32_t)rules.size();
    A->n_words = (A->n_rules + 31) / 32;
    A->groups_per_wave = groups_per_wave;
    A->n = db->n;
    A->kinds = db->kinds.as<uint8_t>();
    A->vals = db->vals.as<uint64_t>();
    A->heads = db->heads.p && db->heads_ncol == (uint32_t)head_cols.size() ? db->heads.as<uint4>() : nullptr;
    A->n_gstr = gstrs.size();
    A->gstr_off = d_gstr_off.as<uint64_t>();
    A->gstr = d_gstr.as<uint8_t>();
    A->bstr_off = db->bstr_off.as<uint64_t>();
    A->bstr = db->bstr.as<uint8_t>();
    A->empty_sid = empty_sid;
    A->map_off = db->map_off.as<uint32_t>();
    A->map_keys = db->map_keys.as<uint32_t>();
    A->map_vals = db->map_vals.as<uint32_t>();
    A->ipof = db->ipof.as<uint64_t>();
    A->tsof = db->tsof.as<uint64_t>();
    A->rx = mxp_dfa_set{d_rx_hdr.as<mxp_dfa_hdr>(), d_rx_trans.as<uint32_t>(), d_rx_ascii.as<uint16_t>(),
                        d_rx_hilo.as<uint32_t>(), d_rx_hicls.as<uint16_t>()};
    A->rx_batch = mxp_dfa_set{db->rx_hdr.as<mxp_dfa_hdr>(), db->rx_trans.as<uint32_t>(), db->rx_ascii.as<uint16_t>(),
                              db->rx_hilo.as<uint32_t>(), db->rx_hicls.as<uint16_t>()};
    A->rxof = db->rxof.as<uint32_t>();
    A->nfa = rx_nfa || db->rx_nfa ? 1u : 0u;
    if (!P.vt_cols.empty()) {
        A->gvt_off = P.d_gvt_off.as<uint32_t>();
        A->gvt = P.d_gvt.as<uint32_t>();
        A->gvt_mask = P.d_gvt_mask.as<uint32_t>();
        A->vt_words = P.d_vt_words.as<uint32_t>();
        A->vt_meta = db->vt_meta.as<uint32_t>();
        A->vt_cls = db->vt_cls.as<uint16_t>();
        A->vt_tm = db->vt_t.as<uint32_t>();
        A->vt_keys = db->vt_keys.as<unsigned long long>();
        A->vt_rep = db->vt_rep.as<uint32_t>();
        A->vt_cnt = db->vt_cnt.as<uint32_t>();
        A->n_vt = (uint32_t)P.vt_cols.size();
        A->vt_imm = db->vt_meta_h.size() >= (size_t)A->n_vt * 8 ? 1u : 0u;
        for (uint32_t a = 0; a < A->n_vt && A->vt_imm; a++)
            if (db->vt_meta_h[a * 8 + MXP_VTM_CAP] != 64u) A->vt_imm = 0u;
        // (marks sized at the batch's first plan: a plan with more value-class chunks takes the
        // LDS-row fill)
        A->vtf_slow = db->vtf_slow.p && db->vtf_slow.n >= MXP_VTF_MARKS(db->n, P.n_vtfills) ? db->vtf_slow.as<uint8_t>() : nullptr;
    }
}

// String heads of a packed batch (kargs.heads): one gather over every column, on the engine stream,
// as the last step of packing -- part of the batch layout, like the columns themselves.
int mxp_engine::pack_heads(mxp_dbatch* db) {
    const uint32_t nrow = (uint32_t)head_cols.size();
    db->heads_ncol = 0;
    if (!heads_on || !db->n || !nrow) return MXP_OK;
    hipError_t e;
    // heads are an accelerator, not part of the batch's meaning: without the memory the index
    // kernel reads the strings themselves (A.heads = null)
    if (db->heads.alloc((size_t)nrow * db->n * 16) != hipSuccess) {
        (void)hipGetLastError();
        db->heads.p = nullptr;
        db->heads.reset();
        return MXP_OK;
    }
    if ((e = d_head_cols.reserve(nrow * 4u)) != hipSuccess) return hipfail(e, "hipMalloc head columns");
    // (async on the engine stream from the engine's own vector: a synchronous hipMemcpy on the legacy
    // stream would wait for every blocking stream's queued work -- a group's evaluations among them)
    if ((e = hipMemcpyAsync(d_head_cols.p, head_cols.data(), nrow * 4u, hipMemcpyHostToDevice, stream)) != hipSuccess)
        return hipfail(e, "upload head columns");
    mxp_kargs A;
    memset(&A, 0, sizeof A);
    A.n = db->n;
    A.kinds = db->kinds.as<uint8_t>();
    A.vals = db->vals.as<uint64_t>();
    A.n_gstr = gstrs.size();
    A.gstr_off = d_gstr_off.as<uint64_t>();
    A.gstr = d_gstr.as<uint8_t>();
    A.bstr_off = db->bstr_off.as<uint64_t>();
    A.bstr = db->bstr.as<uint8_t>();
    if ((e = mxp_launch_heads(&A, d_head_cols.as<uint32_t>(), nrow, db->heads.as<uint4>(), stream)) != hipSuccess)
        return hipfail(e, "launch heads");
    db->heads_ncol = nrow;  // (pack() synchronises once, after the dictionary)
    return MXP_OK;
}

// The value-class dictionary of a packed batch, part of its layout like the interned columns: per
// active column the distinct class keys (a hash table at most half full), the first request that
// claimed each (its representative, on which mxp_vt_eval_kernel evaluates the column's rules) and
// the class sizes (the value-class rules' hit counters).  Every evaluation then only looks its
// requests' classes up (mxp_vt_lookup_kernel).
int mxp_engine::pack_dict(mxp_dbatch* db) {
    if (!db->vt_mask || !db->n) return MXP_OK;
    Plan* P = nullptr;
    int rc = get_plan(db->vt_mask, &P);
    if (rc) return rc;
    if ((rc = vt_prepare(db, *P))) return rc;
    hipError_t e;
    if ((e = hipMemsetAsync(db->vt_keys.p, 0xFF, db->vt_keys_n * 8, stream)) != hipSuccess) return hipfail(e, "vt reset");
    if ((e = hipMemsetAsync(db->vt_cnt.p, 0, db->vt_keys_n * 4, stream)) != hipSuccess) return hipfail(e, "vt count reset");
    mxp_kargs A;
    fill_args(&A, db, *P);
    A.q0 = 0;
    A.q1 = db->n;
    if (db->vtd_ready && !(debug_flags & 134217728u)) {
        // the device packer's two-level dictionary (pack.hip mxp_pack_vtd_*): its provisional tables
        // into the final ones (MXP_DEBUG_FLAGS 134217728: the one-level classify kernel -- A/B)
        mxp_vtd_final_args F;
        memset(&F, 0, sizeof F);
        F.tkey = db->pk.pk_vtd_tkey.as<unsigned long long>();
        F.tcr = db->pk.pk_vtd_tcr.as<uint2>();
        uint32_t a = 0;
        for (uint32_t s = 0; s < vt_cand_col.size() && a < MXP_VT_MAX; s++)
            if ((db->vt_mask >> s) & 1u) F.cand[a++] = s;
        if ((e = mxp_launch_vtd_final(&A, &F, stream)) != hipSuccess) return hipfail(e, "launch vt final");
    } else if ((e = mxp_launch_vt_classify(&A, stream)) != hipSuccess) {
        return hipfail(e, "launch vt classify");
    }
    return MXP_OK;
}

// The batch's value-class layout under plan P (first launch of the batch): per active slot its
// column, class table capacity, offsets into the key / representative tables and the class words.
int mxp_engine::vt_prepare(mxp_dbatch* db, const Plan& P) {
    if (!db->vt_meta_h.empty()) return MXP_OK;
    const uint32_t act = (uint32_t)P.vt_cols.size();
    std::vector<uint32_t> meta((size_t)act * 8, 0);
    uint64_t kbase = 0, tbase = 0, woff = 0;
    uint32_t a = 0;
    for (uint32_t s = 0; s < vt_cand_col.size(); s++) {
        if (!((P.mask >> s) & 1u)) continue;
        const uint32_t cap = db->vt_capc[s];
        meta[a * 8 + MXP_VTM_COL] = P.vt_cols[a];
        meta[a * 8 + MXP_VTM_CAP] = cap;
        meta[a * 8 + MXP_VTM_KBASE] = (uint32_t)kbase;
        meta[a * 8 + MXP_VTM_TBASE] = (uint32_t)tbase;
        meta[a * 8 + MXP_VTM_NW] = P.vt_nw[a];
        meta[a * 8 + MXP_VTM_WOFF] = (uint32_t)woff;
        kbase += cap;
        tbase += (uint64_t)cap * P.vt_nw[a];
        woff += P.vt_nw[a];
        a++;
    }
    if (tbase >= (1ull << 31)) return fail(MXP_ERR_NOMEM, "value-class tables too large");
    hipError_t e;
    if ((e = db->vt_meta.alloc(meta.size() * 4)) != hipSuccess) return hipfail(e, "vt meta");
    db->vt_meta_h.swap(meta);  // (the async copy's source: kept with the batch)
    // (async on the engine stream: see pack_heads; the batch's first launch is ordered after it --
    // pk_ev[3], or the wait below when the launch itself prepared the batch)
    if ((e = hipMemcpyAsync(db->vt_meta.p, db->vt_meta_h.data(), db->vt_meta_h.size() * 4, hipMemcpyHostToDevice,
                            stream)) != hipSuccess)
        return hipfail(e, "upload vt meta");
    db->vt_t_words = tbase;
    if ((e = db->vt_t.alloc(2 * tbase * 4)) != hipSuccess) return hipfail(e, "vt class words");
    if (P.n_vtfills && (e = db->vtf_slow.alloc(MXP_VTF_MARKS(db->n, P.n_vtfills))) != hipSuccess)
        return hipfail(e, "vt fill marks");
    // (zeroed: the fast fill marks only the tiles it ran, so a slow-kernel block never reads a stale
    // mark of a recycled block and stages for nothing -- ADVICE r5)
    if (P.n_vtfills && (e = hipMemsetAsync(db->vtf_slow.p, 0, MXP_VTF_MARKS(db->n, P.n_vtfills), stream)) != hipSuccess)
        return hipfail(e, "vt fill marks");
    vt_fresh = true;
    return MXP_OK;
}

int mxp_dbatch::note_done(hipStream_t s) {
    hipEvent_t ev = nullptr;
    for (auto& se : done_ev)
        if (se.first == s) ev = se.second;
    if (!ev) {
        if (hipEventCreateWithFlags(&ev, kOrderEvent) != hipSuccess) return MXP_ERR_DEVICE;
        done_ev.push_back({s, ev});
    }
    return hipEventRecord(ev, s) == hipSuccess ? MXP_OK : MXP_ERR_DEVICE;
}

// An evaluation of `db` on stream s, then the batch's completion event on s (whatever the body
// enqueued before an early return also reads the batch).
int mxp_engine::launch(mxp_dbatch* db, hipStream_t s, uint32_t* d_match, uint32_t* d_err, uint64_t* d_vals,
                       bool log, unsigned long long* d_hits, uint64_t* stats, uint32_t q_lo, uint32_t q_hi) {
    if (db && db->pack_pending)
        if (int rc0 = finish_pack(db)) return rc0;
    // (a device-packed batch's packer, dictionary and heads ran on the engine stream)
    hipError_t e;
    if (db && db->pk_ev[3] && s != stream && (e = hipStreamWaitEvent(s, db->pk_ev[3], 0)) != hipSuccess)
        return hipfail(e, "wait for the packed batch");
    const int rc = launch_body(db, s, d_match, d_err, d_vals, log, d_hits, stats, q_lo, q_hi);
    if (db && db->note_done(s) != MXP_OK && !rc) return fail(MXP_ERR_DEVICE, "batch completion event");
    return rc;
}

int mxp_engine::launch_body(mxp_dbatch* db, hipStream_t s, uint32_t* d_match, uint32_t* d_err, uint64_t* d_vals,
                            bool log, unsigned long long* d_hits, uint64_t* stats, uint32_t q_lo, uint32_t q_hi) {
    // (no stale flags from the previous evaluation survive an early return below)
    last_dtp = false;
    last_dtp_counted = false;
    last_pairs.on = false;
    // guards on: guard-only groups through the lean kernel, the rest through the VM kernel;
    // guards off (Eval, ablation): every group through the VM kernel
    const bool guards_on = !d_vals && !(debug_flags & 2u);
    // value classes only for plain predicate evaluations: Eval mode, referenced attributes and
    // recomputed error windows (which need every record) run plan 0
    const uint32_t mask = (guards_on && !refs_on && !win_log_cap) ? db->vt_mask : 0u;
    Plan* P = nullptr;
    int rc = get_plan(mask, &P);
    if (rc) return rc;
    vt_fresh = false;
    if (mask && (rc = vt_prepare(db, *P))) return rc;
    if (vt_fresh && s != stream) {  // (this launch prepared the batch's tables on the engine stream)
        hipEvent_t ev = nullptr;
        hipError_t e2;
        if ((e2 = hipEventCreateWithFlags(&ev, kOrderEvent)) != hipSuccess || (e2 = hipEventRecord(ev, stream)) != hipSuccess ||
            (e2 = hipStreamWaitEvent(s, ev, 0)) != hipSuccess) {
            if (ev) (void)hipEventDestroy(ev);
            return hipfail(e2, "vt prepare wait");
        }
        (void)hipEventDestroy(ev);
    }
    mxp_kargs A;
    fill_args(&A, db, *P);
    // NFAs wider than the private-memory walk: the global thread-set scratch (dfa_dev.h)
    const uint32_t wmax = std::max(rx_wmax, db ? db->rx_wmax : 0u);
    if (wmax > MXP_NFA_WIDE_WORDS) {
        if ((rc = nfa_scratch.ensure(wmax))) return fail(rc, "NFA thread-set scratch");
        for (mxp_dfa_set* S : {&A.rx, &A.rx_batch}) nfa_scratch.set(S);
    }
    A.req_err = req_err_out;
    A.hits_gate = hits_gate_out;
    A.hits = d_vals ? nullptr : d_hits;
    A.stats = d_vals ? nullptr : stats;
    A.out_match = d_match;
    A.out_err = d_err;
    A.out_vals = d_vals;
    hipError_t e;
    if (log && win_log_cap) {  // a recomputed window (recompute_errors): its own log, room for every pair
        if (d_winlog.n < (size_t)win_log_cap * sizeof(mxp_err_rec) &&
            (e = d_winlog.alloc((size_t)win_log_cap * sizeof(mxp_err_rec))) != hipSuccess)
            return hipfail(e, "window errlog");
        if (!d_wincount.p && (e = d_wincount.alloc(16)) != hipSuccess) return hipfail(e, "window errcount");
        if ((e = hipMemsetAsync(d_wincount.p, 0, 16, s)) != hipSuccess) return hipfail(e, "memset errcount");
        A.errlog = d_winlog.as<mxp_err_rec>();
        A.errcount = d_wincount.as<uint32_t>();
        A.errcap = win_log_cap;
    } else if (log) {
        if (!d_errlog.p) {
            if ((e = d_errlog.alloc((size_t)errcap * sizeof(mxp_err_rec))) != hipSuccess) return hipfail(e, "errlog");
            if ((e = d_errcount.alloc(16)) != hipSuccess) return hipfail(e, "errcount");
        }
        // errcount[0]: records; [1]: value-class error pairs (not logged per pair); [2]: class records
        if ((e = hipMemsetAsync(d_errcount.p, 0, 16, s)) != hipSuccess) return hipfail(e, "memset errcount");
        A.errlog = d_errlog.as<mxp_err_rec>();
        A.errcount = d_errcount.as<uint32_t>();
        A.errcap = errcap;
    }
    if (refs_on) {
        if ((e = hipMemsetAsync(d_refcount.p, 0, 4, s)) != hipSuccess) return hipfail(e, "memset refcount");
        A.refs = d_refs.as<mxp_ref_rec>();
        A.refcount = d_refcount.as<uint32_t>();
        A.refcap = refcap;
    }
    if (A.n == 0 || A.n_rules == 0) return MXP_OK;
    // guard-index phase: predicate mode only (Eval runs whole programs in mxp_eval_kernel)
    const bool use_index = !d_vals && !(debug_flags & 2u) && P->n_idx > 0;
    if (!use_index) A.n_idx = 0;
    auto gy_of = [&](uint32_t ng) { return (ng + 4 * A.groups_per_wave - 1) / (4 * A.groups_per_wave); };
    if (timing && (e = hipEventRecord(ev[0], s)) != hipSuccess) return hipfail(e, "event");
    struct Part {
        const DevBuf* list;
        uint32_t n;
        int vm;
    } parts[3] = {{guards_on ? &P->d_glean : &P->d_gall, guards_on ? P->n_glean : 0u, 0},
                  {guards_on ? &P->d_gvm : &P->d_gall, guards_on ? P->n_gvm : P->n_gall, 1},
                  {&P->d_gdeep, P->n_gdeep, 2}};  // groups with deep rules (MXP_VM_DEEPREG registers)
    // a request window (error recomputation) or the whole batch, possibly in pipelined chunks:
    // the index kernel of chunk c (which ORs its true / error bits into the words the fill, guard
    // and VM kernels wrote) runs on the side stream while chunk c + 1's fill streams its stores
    const bool window = q_lo != 0 || q_hi < A.n;
    const uint32_t lo = window ? q_lo : 0u, hi = window ? std::min(q_hi, A.n) : A.n;
    if (lo >= hi) return MXP_OK;
    const uint32_t span = hi - lo;
    uint32_t nchunk = 1;
    if (!window && use_index && chunks_max > 1 && span >= 2 * chunk_min)
        nchunk = std::min<uint32_t>(chunks_max, span / chunk_min);
    // chunks start at multiples of 1024 requests (the fill kernel's 16-byte rows)
    const uint32_t step = nchunk > 1 ? (span / nchunk + 1023u) / 1024u * 1024u : span;
    nchunk = (span + step - 1) / step;
    if (nchunk > 1) {
        if (!side && (e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking)) != hipSuccess) {
            side = nullptr;
            return hipfail(e, "side stream");
        }
        for (auto& x : chunk_ev)
            if (!x && (e = hipEventCreateWithFlags(&x, kOrderEvent)) != hipSuccess) {
                x = nullptr;
                return hipfail(e, "chunk event");
            }
    }
    if (guards_on && P->n_fills) A.fills = P->d_fills.as<mxp_fill>();
    if (!use_index) A.dense_of = nullptr;
    if (A.dense_of) {
        if (d_dense_cm.n < (size_t)A.n * 8 && (e = d_dense_cm.alloc((size_t)A.n * 8)) != hipSuccess)
            return hipfail(e, "dense masks");
        A.dense_cm = d_dense_cm.as<uint64_t>();
    }
    if (wave_times) {  // profiling hook (MXP_WAVE_TIMES): per index-kernel wave start / end / phase marks
        const size_t need = ((size_t)A.n + 63) / 64 * 64;
        if (d_wave_t.n < need && (e = d_wave_t.alloc(need)) != hipSuccess) return hipfail(e, "wave times");
        A.wave_t = d_wave_t.as<unsigned long long>();
        wave_t_n = (A.n + 63) / 64;
    }
    // deferred index pairs (kargs.dtp_*): index kernel first, its pairs filed per fill chunk and
    // lane quad and OR-ed in by the value-class fill as it writes the words -- instead of one read-modify-write
    // atomic per true pair on rows the fill wrote before (C4: ~14 per request, 0.6 ms of atomics)
    const bool dtp_on = dtp && P->dtp_ok && use_index && guards_on && nchunk == 1 && !window && lo == 0 &&
                        !A.dense_of && !refs_on && !A.nfa && A.out_match;
    last_dtp = dtp_on;
    // ... whose true pairs are counted where they are filed (mxp_dtp_sort_kernel's per-tile
    // histograms, summed by mxp_dtp_hits_kernel): the hit counters are fused into every kernel of
    // the evaluation, whatever the device gate says, and the bitmap is not streamed again
    // (eval_device_hits; MXP_DEBUG_FLAGS 1048576 keeps the streaming counters)
    const bool dtp_count = dtp_on && A.hits && !(debug_flags & 1048576u) && A.n_rules <= kDtpHist;
    last_dtp_counted = dtp_count;
    // (and the true-pair count that steers the fused / streamed choice is not kept: one atomic per
    // index wave on one address congests its L2 channel -- C2 0.517 -> 0.409 ms same-box, profiles/r3_v6_ab_nostats_c2.log)
    if (dtp_count) {
        A.hits_gate = nullptr;
        A.stats = nullptr;
    }
    if (A.n_vt) {
        // value classes: classify every request of [lo, hi) per active column, then evaluate the
        // columns' rules once per class (class records -> errcount[2], the host expands them)
        // (the batch's dictionary -- keys, representatives, class sizes -- was built at upload)
        A.q0 = lo;
        A.q1 = hi;
        if ((e = mxp_launch_vt_lookup(&A, s)) != hipSuccess) return hipfail(e, "launch vt lookup");
        mxp_kargs AV = A;
        if (A.errlog) {  // class records: a log of their own, counted in errcount[2]
            if (!d_vtlog.p && (e = d_vtlog.alloc((size_t)vtlog_cap * sizeof(mxp_err_rec))) != hipSuccess)
                return hipfail(e, "class errlog");
            AV.errlog = d_vtlog.as<mxp_err_rec>();
            AV.errcount = A.errcount + 2;
            AV.errcap = vtlog_cap;
        }
        uint32_t tiles = 0;
        for (uint32_t a = 0; a < A.n_vt; a++) tiles += db->vt_meta_h[a * 8 + MXP_VTM_CAP] / 64;
        if ((e = mxp_launch_vt_eval(&AV, tiles, (P->vt_max_nw + 3) / 4, s)) != hipSuccess)
            return hipfail(e, "launch vt eval");
    }
    if (A.req_err && !dtp_on && (e = hipMemsetAsync(A.req_err, 0, A.n, s)) != hipSuccess)
        return hipfail(e, "request error flags reset");
    if (dtp_on) {
        A.q0 = lo;
        A.q1 = hi;
        const uint32_t cx = (hi + 63) / 64, grid = (cx + 3) / 4, tiles = (hi + 1023) / 1024;
        // the deferred-pair scratch and counters are engine-wide: a launch on another stream waits
        // for the previous deferred launch to finish with them (its sort kernel resets the counter
        // set this launch uses; its fills read the slots this launch's sort rewrites), and scratch
        // that must grow is released only once that launch is done
        if (!dtp_ev && (e = hipEventCreateWithFlags(&dtp_ev, kOrderEvent)) != hipSuccess) {
            dtp_ev = nullptr;
            return hipfail(e, "deferred-pair event");
        }
        if (dtp_pending) {
            if (dtp_stream != s && (e = hipStreamWaitEvent(s, dtp_ev, 0)) != hipSuccess) return hipfail(e, "deferred-pair wait");
            const size_t need_slots = (size_t)(P->n_fills + P->n_vtfills) * MXP_DTP_ROW(tiles) * 16;
            if ((d_dtp_ent.n < (size_t)cx * dtp_cap * 4 || d_dtp_n.n < (size_t)grid * 16 || d_dtp_slots.n < need_slots ||
                 d_dtp_qn.n < need_slots / 16 || d_dtp_ovf.n < (size_t)dtp_ovf_cap * 8 ||
                 (dtp_count && d_dtp_part.n < (size_t)tiles * ((A.n_rules + 1) / 2) * 4)) &&
                (e = hipEventSynchronize(dtp_ev)) != hipSuccess)
                return hipfail(e, "deferred-pair sync");
        }
        if ((e = d_dtp_ent.reserve((size_t)cx * dtp_cap * 4)) != hipSuccess ||
            (e = d_dtp_n.reserve((size_t)grid * 4 * 4)) != hipSuccess ||
            (e = d_dtp_ovf.reserve((size_t)dtp_ovf_cap * 8)) != hipSuccess ||
            (e = d_dtp_slots.reserve((size_t)(P->n_fills + P->n_vtfills) * MXP_DTP_ROW(tiles) * 16)) != hipSuccess ||
            (e = d_dtp_qn.reserve((size_t)(P->n_fills + P->n_vtfills) * MXP_DTP_ROW(tiles))) != hipSuccess)
            return hipfail(e, "deferred-pair scratch");
        if (!d_dtp_ovf_n.p) {  // two counter sets (count, list full): each launch's sort kernel resets the other
            if ((e = d_dtp_ovf_n.alloc(32)) != hipSuccess) return hipfail(e, "deferred-pair counters");
            if ((e = hipMemsetAsync(d_dtp_ovf_n.p, 0, 32, s)) != hipSuccess) return hipfail(e, "memset dtp");
        }
        uint32_t* const ovf_n = d_dtp_ovf_n.as<uint32_t>() + 4u * dtp_par;
        uint32_t* const ovf_next = d_dtp_ovf_n.as<uint32_t>() + 4u * (dtp_par ^ 1u);
        dtp_par ^= 1u;
        mxp_kargs AI = A;  // the index kernel records
        AI.req_err_init = A.req_err ? 1u : 0u;
        AI.dtp_ent = d_dtp_ent.as<uint32_t>();
        AI.dtp_n = d_dtp_n.as<uint32_t>();
        AI.dtp_ovf_n = ovf_n;
        AI.dtp_ovf_next = ovf_next;
        AI.dtp_ovf = d_dtp_ovf.as<uint32_t>();
        AI.dtp_cap = dtp_cap;
        AI.dtp_ovf_cap = dtp_ovf_cap;
        AI.dtp_chunk = P->d_dtp_chunk.as<uint32_t>();
        AI.dtp_slots = d_dtp_slots.as<uint16_t>();
        AI.dtp_qn = d_dtp_qn.as<uint8_t>();
        AI.dtp_tiles = tiles;
        AI.dtp_nchunks = P->n_fills + P->n_vtfills;
        if (dtp_count) {
            if ((e = d_dtp_part.reserve((size_t)tiles * ((A.n_rules + 1) / 2) * 4)) != hipSuccess)
                return hipfail(e, "deferred-pair histograms");
            AI.dtp_part = d_dtp_part.as<uint32_t>();
        }
        // Request chunks (dtp_chunks > 1, tiles of 1024 requests): chunk c's index and sort kernels
        // run on the side stream while the evaluation stream fills chunk c - 1 -- the latency-bound
        // index waves beside the store-bound fill -- and each fill waits for its chunk's sort only.
        // Chunks own disjoint tiles of every scratch array (wave lists, slots, counts, histograms).
        const uint32_t K = std::max(1u, std::min(dtp_chunks, tiles));
        hipStream_t xs = s;
        if (K > 1) {
            if (!side && (e = hipStreamCreateWithFlags(&side, hipStreamNonBlocking)) != hipSuccess) {
                side = nullptr;
                return hipfail(e, "side stream");
            }
            for (auto& x : dtp_cev)
                if (!x && (e = hipEventCreateWithFlags(&x, kOrderEvent)) != hipSuccess) {
                    x = nullptr;
                    return hipfail(e, "chunk event");
                }
            // the side stream starts after everything before this evaluation on s (the previous
            // evaluation's fills read the slots the sorts rewrite; the value classes)
            if ((e = hipEventRecord(dtp_cev[kDtpChunksMax], s)) != hipSuccess ||
                (e = hipStreamWaitEvent(side, dtp_cev[kDtpChunksMax], 0)) != hipSuccess)
                return hipfail(e, "side stream wait");
            xs = side;
        }
        mxp_kargs AF = A;  // the fills merge
        AF.dtp_slots = AI.dtp_slots;
        AF.dtp_qn = AI.dtp_qn;
        AF.dtp_tiles = tiles;
        // a pair Resolve's evaluation: every word a plain fill chunk's (no lean / VM / deep groups, no
        // value classes), so the filed pairs are the match bitmap -- the fills store it only if some
        // pair overflowed its list or slots (kargs.dtp_lazy)
        if (pair_req && P->n_fills && !P->n_vtfills && !P->n_glean && !P->n_gvm && !P->n_gdeep && !A.n_vt &&
            !A.out_err) {
            AF.dtp_lazy = ovf_n;
            last_pairs.on = true;
            last_pairs.ovf_n = ovf_n;
            last_pairs.slots = AI.dtp_slots;
            last_pairs.qn = AI.dtp_qn;
            last_pairs.fills = P->d_fills.as<uint32_t>();
            last_pairs.row = MXP_DTP_ROW(tiles);
            last_pairs.nch = P->n_fills;
        }
        for (uint32_t c = 0; c < K; c++) {
            const uint32_t t0 = (uint32_t)((uint64_t)tiles * c / K), t1 = (uint32_t)((uint64_t)tiles * (c + 1) / K);
            AI.q0 = t0 * 1024u;
            AI.q1 = std::min(t1 * 1024u, hi);
            AI.dtp_t0 = t0;
            AI.dtp_tn = t1 - t0;
            const uint32_t gc = ((AI.q1 - AI.q0 + 63) / 64 + 3) / 4;
            if ((e = mxp_launch_index(&AI, gc, xs)) != hipSuccess) return hipfail(e, "launch index");
            if ((e = mxp_launch_dtp_sort(&AI, xs)) != hipSuccess) return hipfail(e, "launch dtp sort");
            if (K > 1 && ((e = hipEventRecord(dtp_cev[c], xs)) != hipSuccess || (e = hipStreamWaitEvent(s, dtp_cev[c], 0)) != hipSuccess))
                return hipfail(e, "chunk event");
            if (timing && c == 0 && (e = hipEventRecord(ev[1], s)) != hipSuccess) return hipfail(e, "event");
            AF.q0 = AI.q0;
            AF.q1 = AI.q1;
            AF.fills = A.fills;
            AF.dtp_cbase = 0;
            if (P->n_fills && (e = mxp_launch_fill(&AF, P->n_fills, s)) != hipSuccess) return hipfail(e, "launch fill");
            AF.fills = P->d_vtfills.as<mxp_fill>();
            AF.dtp_cbase = P->n_fills;
            if (P->n_vtfills && (e = mxp_launch_vtfill(&AF, P->n_vtfills, s)) != hipSuccess) return hipfail(e, "launch vtfill");
        }
        AI.q0 = lo;
        AI.q1 = hi;
        if (dtp_count && (e = mxp_launch_dtp_hits(AI.dtp_part, tiles, A.n_rules, A.hits, s)) != hipSuccess)
            return hipfail(e, "launch dtp hits");
        for (const Part& Pt : parts) {
            if (!Pt.n) continue;
            A.glist = Pt.list->as<uint32_t>();
            A.n_glist = Pt.n;
            if ((e = mxp_launch_eval(&A, cx, gy_of(Pt.n), Pt.vm, s)) != hipSuccess) return hipfail(e, "launch eval");
        }
        // the overflow list OR-ed in; if it filled, the index kernel again, OR-ing every pair (no
        // counters, no records: the first pass kept those) -- else it returns after the list
        mxp_kargs AR = A;
        AR.dtp_ovf_n = AI.dtp_ovf_n;
        AR.dtp_ovf = AI.dtp_ovf;
        AR.dtp_ovf_cap = AI.dtp_ovf_cap;
        AR.dtp_gate = AI.dtp_ovf_n + 1;
        AR.hits = nullptr;
        AR.stats = nullptr;
        AR.errlog = nullptr;
        AR.errcount = nullptr;
        AR.wave_t = nullptr;
        AR.gate_out = dtp_count ? gate_next_out : nullptr;
        if ((e = mxp_launch_index(&AR, grid, s)) != hipSuccess) return hipfail(e, "launch index re-run");
        if ((e = hipEventRecord(dtp_ev, s)) != hipSuccess) return hipfail(e, "deferred-pair event");
        dtp_pending = true;
        dtp_stream = s;
        if (timing && (e = hipEventRecord(ev[2], s)) != hipSuccess) return hipfail(e, "event");
        ev_index = true;
        last_mask = mask;
        return MXP_OK;
    }
    for (uint32_t c = 0; c < nchunk; c++) {
        A.q0 = lo + c * step;
        A.q1 = std::min(hi, lo + (c + 1) * step);
        const uint32_t cx = (A.q1 - A.q0 + 63) / 64;
        if (guards_on && P->n_fills && (e = mxp_launch_fill(&A, P->n_fills, s)) != hipSuccess) return hipfail(e, "launch fill");
        if (guards_on && P->n_vtfills) {
            mxp_kargs AF = A;
            AF.fills = P->d_vtfills.as<mxp_fill>();
            if ((e = mxp_launch_vtfill(&AF, P->n_vtfills, s)) != hipSuccess) return hipfail(e, "launch vtfill");
        }
        for (const Part& Pt : parts) {
            if (!Pt.n) continue;
            A.glist = Pt.list->as<uint32_t>();
            A.n_glist = Pt.n;
            if ((e = mxp_launch_eval(&A, cx, gy_of(Pt.n), Pt.vm, s)) != hipSuccess) return hipfail(e, "launch eval");
        }
        if (!use_index) continue;
        if (nchunk == 1) {
            if (timing && (e = hipEventRecord(ev[1], s)) != hipSuccess) return hipfail(e, "event");
            if ((e = mxp_launch_index(&A, (cx + 3) / 4, s)) != hipSuccess) return hipfail(e, "launch index");
            if (A.dense_of && (e = mxp_launch_inject(&A, (cx + 3) / 4, s)) != hipSuccess) return hipfail(e, "launch inject");
            continue;
        }
        if ((e = hipEventRecord(chunk_ev[c], s)) != hipSuccess) return hipfail(e, "chunk event");
        if ((e = hipStreamWaitEvent(side, chunk_ev[c], 0)) != hipSuccess) return hipfail(e, "side wait");
        if ((e = mxp_launch_index(&A, (cx + 3) / 4, side)) != hipSuccess) return hipfail(e, "launch index");
        if (A.dense_of && (e = mxp_launch_inject(&A, (cx + 3) / 4, side)) != hipSuccess) return hipfail(e, "launch inject");
    }
    if (nchunk > 1) {
        // join: ev[1] = the main stream done (fill / guard / VM of every chunk), then the index tail
        if (timing && (e = hipEventRecord(ev[1], s)) != hipSuccess) return hipfail(e, "event");
        if ((e = hipEventRecord(chunk_ev[kChunksMax], side)) != hipSuccess) return hipfail(e, "join event");
        if ((e = hipStreamWaitEvent(s, chunk_ev[kChunksMax], 0)) != hipSuccess) return hipfail(e, "join wait");
    } else if (!use_index && timing && (e = hipEventRecord(ev[1], s)) != hipSuccess) {
        return hipfail(e, "event");
    }
    if (timing && (e = hipEventRecord(ev[2], s)) != hipSuccess) return hipfail(e, "event");
    ev_index = use_index;
    last_mask = mask;
    return MXP_OK;
}

// %v of a packed (interned) column value, for error texts whose host batch is gone (errors
// recomputed on demand, mxp_engine::recompute_errors): strings, byte strings and timestamps through
// the interning tables, string maps through the device CSR
std::string mxp_engine::packed_value_text(const mxp_dbatch* db, uint32_t kind, uint64_t v) const {
    switch (kind) {
    case MXP_STRING: case MXP_OTHER: return string_of(db, v);
    case MXP_INT64: return std::to_string((int64_t)v);
    case MXP_BOOL: return v ? "true" : "false";
    case MXP_DOUBLE: {
        double d;
        memcpy(&d, &v, 8);
        return mxp::go_format_float(d);
    }
    case MXP_DURATION: return mxp::go_format_duration((int64_t)v);
    case MXP_TIMESTAMP: {
        TimeKey t{0, 0};
        if (v < gtimes.size()) t = gtimes[v];
        else if (db) db->overlay_time(v - gtimes.size(), &t);
        return mxp::go_format_time_utc(t.s, t.ns);
    }
    case MXP_BYTES: {
        const uint64_t raw = MXP_BYTES_RAW(v);
        std::string c;
        if (raw < gbytes.size()) c = gbytes[raw];
        else if (db) db->overlay_bytes_at(raw - gbytes.size(), &c);
        return mxp::go_format_bytes((const uint8_t*)c.data(), c.size());
    }
    case MXP_STRING_MAP: {
        if (v < snap_maps.size()) return snap_maps[v];
        uint32_t mo[2] = {0, 0};
        std::string out = "map[";
        if (!db || db->map_off.n < (v + 2) * 4 ||
            hipMemcpy(mo, db->map_off.as<uint32_t>() + v, 8, hipMemcpyDeviceToHost) != hipSuccess)
            return out + "]";
        std::vector<uint32_t> k(mo[1] - mo[0]), w(mo[1] - mo[0]);
        if (!k.empty() &&
            (hipMemcpy(k.data(), db->map_keys.as<uint32_t>() + mo[0], k.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
             hipMemcpy(w.data(), db->map_vals.as<uint32_t>() + mo[0], w.size() * 4, hipMemcpyDeviceToHost) != hipSuccess))
            return out + "]";
        for (size_t e = 0; e < k.size(); e++) out += (e ? " " : "") + string_of(db, k[e]) + ":" + string_of(db, w[e]);
        return out + "]";
    }
    default: return "?";
    }
}

std::string mxp_engine::format_error(const mxp_bag_batch* b, const mxp_dbatch* db, const mxp_err_rec& r,
                                     const ErrWindow* win) const {
    switch (r.code) {
    case ERR_LOOKUP: return "lookup failed: '" + string_of(db, r.aux) + "'";
    case ERR_CONV_S: case ERR_CONV_B: case ERR_CONV_I: case ERR_CONV_D: {
        static const char* what[] = {"string", "bool", "integer or duration", "double"};
        std::string val = "?";
        if (!b && win && r.aux < win->ncol && r.req >= win->q0 && r.req < win->q1) {
            const size_t at = (size_t)r.aux * (win->q1 - win->q0) + (r.req - win->q0);
            val = packed_value_text(db, win->kinds[at], win->vals[at]);
        }
        if (b && r.aux < cols.size()) {
            for (uint32_t c = 0; c < b->n_columns; c++) {
                if (cols[r.aux] != b->column_names[c]) continue;
                uint8_t k = b->kinds[c][r.req];
                uint64_t v = b->values[c][r.req];
                auto bs = [&](uint64_t sid) {
                    return std::string((const char*)b->str_bytes + b->str_offsets[sid],
                                       (size_t)(b->str_offsets[sid + 1] - b->str_offsets[sid]));
                };
                switch (k) {
                case MXP_STRING: case MXP_OTHER: val = bs(v); break;
                case MXP_INT64: val = std::to_string((int64_t)v); break;
                case MXP_BOOL: val = v ? "true" : "false"; break;
                case MXP_DOUBLE: {
                    double d;
                    memcpy(&d, &v, 8);
                    val = mxp::go_format_float(d);
                    break;
                }
                case MXP_DURATION: val = mxp::go_format_duration((int64_t)v); break;
                case MXP_TIMESTAMP: val = mxp::go_format_time_utc(b->time_sec[v], b->time_nsec[v]); break;
                case MXP_BYTES: {
                    std::string raw = bs(v);
                    val = mxp::go_format_bytes((const uint8_t*)raw.data(), raw.size());
                    break;
                }
                case MXP_STRING_MAP: {
                    val = "map[";
                    for (uint64_t e = b->map_offsets[v]; e < b->map_offsets[v + 1]; e++) {
                        if (e != b->map_offsets[v]) val += " ";
                        val += bs(b->map_keys[e]) + ":" + bs(b->map_values[e]);
                    }
                    val += "]";
                    break;
                }
                default: break;
                }
                break;
            }
        }
        return std::string("error converting value to ") + what[r.code - ERR_CONV_S] + ": '" + val + "'";
    }
    case ERR_IP: return "could not convert " + string_of(db, r.aux) + " to IP_ADDRESS";
    case ERR_TS:
        return "could not convert '" + string_of(db, r.aux) +
               "' to TIMESTAMP. expected format: '2006-01-02T15:04:05Z07:00'";
    case ERR_MEMBER: return "member lookup failed: '" + string_of(db, r.aux) + "'";
    case ERR_UNDERFLOW: return "stack underflow";
    case ERR_OVERFLOW: return "stack overflow";
    case ERR_HEAP: return "heap overflow";
    case ERR_REGEX: case ERR_REGEX_UNSUPPORTED: {
        // regexp.MatchString's error: the pattern's compile error (Go's text); or why this engine
        // cannot compile it (a known divergence, reported rather than approximated)
        mxp::Dfa d;
        std::string e;
        mxp::regex_compile({string_of(db, r.aux)}, 1, &d, &e);
        return r.code == ERR_REGEX ? e : "unsupported regexp (engine): " + e;
    }
    case ERR_STATIC: case ERR_UNSUPPORTED: case PANIC_STATIC:
        return r.aux < rules.size() ? rules[r.aux].error : std::string("?");
    case PANIC_MAPTYPE: return "Unknown map type";
    case PANIC_EXTARG: return "reflect: Call using a value of the wrong type";
    case PANIC_NOTBOOL: return "interpreter.Result: result is not bool";
    case PANIC_CONV: return "interface conversion: interface {} is not string";
    case PANIC_INDEX: return "runtime error: index out of range";
    default: return "error code " + std::to_string(r.code);
    }
}

// ===================================================================================== C-ABI
static int put_text(const std::string& s, char* buf, uint32_t cap);
extern "C" {

int mxp_engine_create(int device, mxp_engine** out) {
    if (!out) return MXP_ERR_ARG;
    auto* e = new (std::nothrow) mxp_engine();
    if (!e) return MXP_ERR_NOMEM;
    e->device = device;
    if (const char* f = getenv("MXP_DEBUG_FLAGS")) e->debug_flags = (uint32_t)atoi(f);
    if (const char* f = getenv("MXP_TRACE")) e->trace = atoi(f) != 0;
    if (const char* f = getenv("MXP_D2H_DMA")) e->d2h_dma = atoi(f) != 0;
    if (const char* f = getenv("MXP_RESOLVE_TILE")) e->resolve_tile = atoi(f) != 0;
    if (const char* f = getenv("MXP_RESOLVE_PAIRS")) e->resolve_pairs = atoi(f);
    if (const char* f = getenv("MXP_LAZY_RECORDS")) e->lazy_records = atoi(f) != 0;
    if (const char* f = getenv("MXP_PACK_COLS_BESIDE")) e->pack_cols_beside = atoi(f) != 0;
    if (const char* f = getenv("MXP_DTP")) e->dtp = atoi(f) != 0;
    if (const char* f = getenv("MXP_DTP_CAP")) e->dtp_cap = (uint32_t)std::min(1 << 20, std::max(1, atoi(f)));
    if (const char* f = getenv("MXP_DTP_OVF")) e->dtp_ovf_cap = (uint32_t)std::max(1, atoi(f));
    if (const char* f = getenv("MXP_INDEX_SPARSITY")) e->index_sparsity = (uint32_t)std::min(8, std::max(0, atoi(f)));
    // tuning knobs (results are identical for every setting)
    if (const char* f = getenv("MXP_GPW")) e->groups_per_wave = std::max(1, atoi(f));
    // (at most the kernels' compile-time chunk: their LDS tables are sized for MXP_FILL_CHUNK groups)
    if (const char* f = getenv("MXP_FILL_CHUNK")) e->fill_chunk = (uint32_t)std::min((int)MXP_FILL_CHUNK, std::max(1, atoi(f)));
    if (const char* f = getenv("MXP_FILL_SPAN")) e->fill_span = (uint32_t)std::min(8, std::max(1, atoi(f)));
    if (const char* f = getenv("MXP_ERRCAP")) e->errcap = (uint32_t)std::max(1, atoi(f));
    if (getenv("MXP_WAVE_TIMES")) e->wave_times = true;
    if (const char* h = getenv("MXP_HEADS")) e->heads_on = atoi(h) != 0;
    if (const char* h = getenv("MXP_DTP_CHUNKS")) e->dtp_chunks = std::max(1, std::min(atoi(h), (int)mxp_engine::kDtpChunksMax));
    if (const char* f = getenv("MXP_HOST_PACK")) e->host_pack = atoi(f) != 0;  // A/B: the host packer
    if (device < 0) {  // host-only engine (compiler / lowering inspection without a GPU)
        e->reset_tables();
        *out = e;
        return MXP_OK;
    }
    hipError_t h = hipSetDevice(device);
    // (a blocking stream: ordered with the legacy default stream, so callers that prepare outputs
    // there and pass NULL see them done -- a non-blocking one raced a caller's zeroing of the hit
    // counters with the first evaluation's value-class counts)
    if (h == hipSuccess) h = hipStreamCreateWithFlags(&e->stream, hipStreamDefault);
    if (h != hipSuccess) {
        delete e;
        return MXP_ERR_DEVICE;
    }
    e->reset_tables();
    *out = e;
    return MXP_OK;
}

void mxp_engine_destroy(mxp_engine* eng) {
    if (!eng) return;
    if (eng->device >= 0) (void)hipSetDevice(eng->device);
    for (int k = 0; k < mxp_engine::kCopyStreams; k++)
        if (eng->copy_s[k]) (void)hipStreamDestroy(eng->copy_s[k]);
    for (int k = 0; k < 2; k++) {
        if (eng->bounce_ev[k]) (void)hipEventDestroy(eng->bounce_ev[k]);
        if (eng->bounce[k]) (void)hipHostFree(eng->bounce[k]);
    }
    if (eng->res_small) (void)hipHostFree(eng->res_small);
    eng->bin.release();
    if (eng->stream) (void)hipStreamDestroy(eng->stream);
    for (auto& x : eng->ev)
        if (x) (void)hipEventDestroy(x);
    if (eng->side) (void)hipStreamSynchronize(eng->side);
    for (auto& x : eng->chunk_ev)
        if (x) (void)hipEventDestroy(x);
    for (auto& x : eng->dtp_cev)
        if (x) (void)hipEventDestroy(x);
    if (eng->side) (void)hipStreamDestroy(eng->side);
    if (eng->dtp_ev) (void)hipEventSynchronize(eng->dtp_ev);
    if (eng->dtp_ev) (void)hipEventDestroy(eng->dtp_ev);
    if (eng->stats_ev) (void)hipEventSynchronize(eng->stats_ev);
    if (eng->stats_ev) (void)hipEventDestroy(eng->stats_ev);
    delete eng;
}

const char* mxp_last_error(const mxp_engine* eng) { return eng ? eng->last_error.c_str() : "null engine"; }

int mxp_vocab_set(mxp_engine* eng, const char* const* names, const int32_t* types, uint32_t n) {
    if (!eng || (n && (!names || !types))) return MXP_ERR_ARG;
    eng->vocab.clear();
    eng->vocab_index.clear();
    eng->vocab_names.clear();
    eng->finder = nullptr;
    eng->finder_ctx = nullptr;
    eng->finder_missing.clear();
    for (uint32_t i = 0; i < n; i++) {
        eng->vocab[names[i]] = types[i];
        eng->vocab_index[names[i]] = i;
        eng->vocab_names.push_back(names[i]);
    }
    eng->reset_tables();
    return MXP_OK;
}

int mxp_vocab_set_finder(mxp_engine* eng, mxp_attr_finder find, void* ctx) {
    if (!eng || !find) return MXP_ERR_ARG;
    eng->vocab.clear();
    eng->vocab_index.clear();
    eng->vocab_names.clear();
    eng->finder = find;
    eng->finder_ctx = ctx;
    eng->finder_missing.clear();
    eng->reset_tables();
    return MXP_OK;
}

int mxp_vocab_name(mxp_engine* eng, uint32_t pos, char* buf, uint32_t cap) {
    if (!eng || pos >= eng->vocab_names.size()) return MXP_ERR_ARG;
    return put_text(eng->vocab_names[pos], buf, cap);
}

int mxp_ruleset_compile(mxp_engine* eng, const char* const* exprs, uint32_t n, int32_t* status) {
    if (!eng || (n && !exprs)) return MXP_ERR_ARG;
    return eng->compile(exprs, n, status);
}

static int put_text(const std::string& s, char* buf, uint32_t cap) {
    if (!buf || cap == 0) return MXP_ERR_ARG;
    size_t k = std::min<size_t>(s.size(), cap - 1);
    memcpy(buf, s.data(), k);
    buf[k] = 0;
    return MXP_OK;
}

int mxp_rule_error(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap) {
    if (!eng || rule >= eng->rules.size()) return MXP_ERR_ARG;
    return put_text(eng->rules[rule].error, buf, cap);
}

int mxp_rule_il_text(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap) {
    if (!eng || rule >= eng->rules.size()) return MXP_ERR_ARG;
    return put_text(eng->rules[rule].il_text, buf, cap);
}

int mxp_rule_vm_text(mxp_engine* eng, uint32_t rule, char* buf, uint32_t cap) {
    if (!eng || rule >= eng->rules.size()) return MXP_ERR_ARG;
    return put_text(mxp::vm_disasm(eng->rules[rule].low.code), buf, cap);
}

int mxp_rule_types(mxp_engine* eng, uint32_t rule, int32_t* vt, int32_t* il) {
    if (!eng || rule >= eng->rules.size()) return MXP_ERR_ARG;
    if (vt) *vt = eng->rules[rule].value_type;
    if (il) *il = eng->rules[rule].il_ret;
    return MXP_OK;
}

uint32_t mxp_rule_count(const mxp_engine* eng) { return eng ? (uint32_t)eng->rules.size() : 0; }
uint32_t mxp_dbatch_requests(const mxp_dbatch* db) { return db ? db->n : 0; }

int mxp_set_pipeline(mxp_engine* eng, uint32_t min_requests, uint32_t max_chunks) {
    if (!eng || min_requests == 0 || max_chunks == 0 || max_chunks > mxp_engine::kChunksMax) return MXP_ERR_ARG;
    eng->chunk_min = min_requests;
    eng->chunks_max = max_chunks;
    return MXP_OK;
}

int mxp_set_timing(mxp_engine* eng, int on) {
    if (!eng || eng->device < 0) return MXP_ERR_ARG;
    hipError_t e = hipSetDevice(eng->device);
    if (e != hipSuccess) return eng->hipfail(e, "hipSetDevice");
    for (auto& x : eng->ev)
        if (on && !x && (e = hipEventCreate(&x)) != hipSuccess) return eng->hipfail(e, "hipEventCreate");
    eng->timing = on != 0;
    return MXP_OK;
}

int mxp_kernel_times(mxp_engine* eng, float* ms, uint32_t cap, uint32_t* n_out) {
    if (!eng || !ms || !n_out) return MXP_ERR_ARG;
    *n_out = 0;
    if (!eng->timing) return eng->fail(MXP_ERR_STATE, "timing not enabled");
    hipError_t e;
    float t[2] = {0.f, 0.f};
    if ((e = hipEventSynchronize(eng->ev[2])) != hipSuccess) return eng->hipfail(e, "event sync");
    if ((e = hipEventElapsedTime(&t[0], eng->ev[0], eng->ev[1])) != hipSuccess) return eng->hipfail(e, "elapsed");
    if ((e = hipEventElapsedTime(&t[1], eng->ev[1], eng->ev[2])) != hipSuccess)
        return eng->hipfail(e, "elapsed");
    const float tt[3] = {t[0], t[1], eng->last_dtp ? 1.f : 0.f};
    uint32_t k = 0;
    for (; k < cap && k < 3; k++) ms[k] = tt[k];
    *n_out = k;
    return MXP_OK;
}

int mxp_debug_wave_times(mxp_engine* eng, uint64_t* out, uint64_t cap, uint64_t* n_out) {
    if (!eng || !out || !n_out) return MXP_ERR_ARG;
    *n_out = 0;
    if (!eng->wave_times || !eng->d_wave_t.p) return eng->fail(MXP_ERR_STATE, "MXP_WAVE_TIMES not set");
    hipError_t e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return eng->hipfail(e, "sync");
    const uint64_t k = std::min<uint64_t>(cap, (uint64_t)eng->wave_t_n * 8);
    if (k && (e = hipMemcpy(out, eng->d_wave_t.p, k * 8, hipMemcpyDeviceToHost)) != hipSuccess)
        return eng->hipfail(e, "download wave times");
    *n_out = k;
    return MXP_OK;
}

uint32_t mxp_ruleset_columns(mxp_engine* eng, const char** names, uint32_t cap) {
    if (!eng || !eng->have_rules) return 0;
    eng->attr_names = eng->read_attributes();
    const uint32_t n = (uint32_t)eng->attr_names.size();
    for (uint32_t i = 0; names && i < n && i < cap; i++) names[i] = eng->attr_names[i].c_str();
    return n;
}

uint32_t mxp_ruleset_info(const mxp_engine* eng, uint32_t* out, uint32_t cap) {
    if (!eng || !out) return 0;
    const mxp_engine::Plan* P = eng->plan0();
    if (!P) return 0;
    const uint32_t v[10] = {eng->n_guarded, eng->n_templated, P->n_tmpls, P->n_segs, P->n_indexed,
                            (uint32_t)(eng->cols.size() + eng->vcols.size()), P->n_composite, P->n_alias,
                            P->n_dense, (uint32_t)eng->vt_cand_col.size()};
    uint32_t k = 0;
    for (; k < cap && k < 10; k++) out[k] = v[k];
    return k;
}

int mxp_batch_upload_ex(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t flags, mxp_dbatch** out) {
    if (!eng || (flags & ~(uint32_t)MXP_UPLOAD_NO_WAIT)) return MXP_ERR_ARG;
    eng->upload_no_wait = (flags & MXP_UPLOAD_NO_WAIT) != 0;
    const int rc = mxp_batch_upload(eng, batch, out);
    eng->upload_no_wait = false;
    return rc;
}

int mxp_batch_wait_copied(mxp_dbatch* db) {
    if (!db) return MXP_ERR_ARG;
    if (db->pk_ev[1] && hipEventSynchronize(db->pk_ev[1]) != hipSuccess) return MXP_ERR_DEVICE;
    return MXP_OK;
}

// mxp_batch_upload, and for a narrow batch (mxp_batch_upload2) its host view, handed to the device
// batch (batch points into it)
static int batch_upload(mxp_engine* eng, const mxp_bag_batch* batch, mxp_dbatch** out, std::unique_ptr<WideView>* wide) {
    if (!eng || !batch || !out) return MXP_ERR_ARG;
    if (!eng->have_rules) return eng->fail(MXP_ERR_STATE, "no rule set compiled");
    if (eng->device < 0) return eng->fail(MXP_ERR_STATE, "host-only engine");
    hipError_t h = hipSetDevice(eng->device);
    if (h != hipSuccess) return eng->hipfail(h, "hipSetDevice");
    auto* db = new (std::nothrow) mxp_dbatch();
    if (!db) return MXP_ERR_NOMEM;
    if (wide) db->wide = std::move(*wide);
    // (the batch's own blocks recycled where the bin has them; engine scratch grown meanwhile is not)
    g_bin_take = &eng->bin;
    g_bin_db = db;
    g_bin_db_size = sizeof(mxp_dbatch);
    int rc = eng->pack(batch, db);
    g_bin_take = nullptr;
    g_bin_db = nullptr;
    if (rc) {
        delete db;
        return rc;
    }
    *out = db;
    return MXP_OK;
}

int mxp_batch_upload(mxp_engine* eng, const mxp_bag_batch* batch, mxp_dbatch** out) {
    return batch_upload(eng, batch, out, nullptr);
}

void WideView::materialize() {
    if (full) return;
    full = true;
    const mxp_bag_batch& B = src.base;
    auto widen = [](const uint32_t* in, uint64_t m) {
        std::unique_ptr<uint64_t[]> o(new uint64_t[m ? m : 1]);
        uint64_t* p = o.get();
        mxp::par_for(m, 1u << 16, [&](uint64_t a, uint64_t z, unsigned) {
            for (uint64_t i = a; i < z; i++) p[i] = in[i];
        });
        return o;
    };
    for (uint32_t c = 0; c < B.n_columns; c++)
        if (src.narrow[c] && src.values32 && src.values32[c]) {
            vals[c] = widen(src.values32[c], B.n_requests);
            vptr[c] = vals[c].get();
        }
    if (B.n_strings) {
        soff = widen(src.str_offsets32, (uint64_t)B.n_strings + 1);
        view.str_offsets = soff.get();
    }
    if (B.n_maps) {
        moff = widen(src.map_offsets32, (uint64_t)B.n_maps + 1);
        view.map_offsets = moff.get();
    }
}

int mxp_batch_upload2(mxp_engine* eng, const mxp_bag_batch2* b2, uint32_t flags, mxp_dbatch** out) {
    if (!eng || !b2 || !out || (flags & ~(uint32_t)MXP_UPLOAD_NO_WAIT)) return MXP_ERR_ARG;
    const mxp_bag_batch& B = b2->base;
    const uint64_t n = B.n_requests;
    auto bad = [&](const std::string& what) { return eng->fail(MXP_ERR_ARG, "malformed narrow batch: " + what); };
    if (B.n_columns && (!b2->narrow || !B.kinds)) return bad("narrow / kinds is NULL");
    if (B.n_strings && !b2->str_offsets32) return bad("str_offsets32 is NULL");
    if (B.n_maps && !b2->map_offsets32) return bad("map_offsets32 is NULL");
    for (uint32_t c = 0; c < B.n_columns; c++) {
        const bool nar = b2->narrow[c] != 0;
        if (n && nar && (!b2->values32 || !b2->values32[c])) return bad("values32 of a narrow column is NULL");
        if (n && !nar && (!B.values || !B.values[c])) return bad("values of a wide column is NULL");
    }
    // the host view (WideView): the wide columns as given; the narrow ones and the offsets made on
    // demand (the copies and the batch checks read the narrow arrays)
    std::unique_ptr<WideView> W(new WideView());
    W->view = B;
    W->src = *b2;
    W->vptr.assign(B.n_columns, nullptr);
    W->vals.resize(B.n_columns);
    for (uint32_t c = 0; c < B.n_columns; c++) W->vptr[c] = b2->narrow[c] ? nullptr : B.values ? B.values[c] : nullptr;
    W->view.values = B.n_columns ? W->vptr.data() : B.values;
    W->view.str_offsets = nullptr;
    W->view.map_offsets = nullptr;
    const mxp_bag_batch* view = &W->view;
    eng->upload_no_wait = (flags & MXP_UPLOAD_NO_WAIT) != 0;
    eng->narrow_src = b2;
    const int rc = batch_upload(eng, view, out, &W);
    eng->narrow_src = nullptr;
    eng->upload_no_wait = false;
    return rc;
}

int mxp_batch_pack_host(mxp_engine* eng, const mxp_bag_batch* batch, uint64_t* out, uint32_t cap) {
    if (!eng || !batch) return MXP_ERR_ARG;
    if (!eng->have_rules) return eng->fail(MXP_ERR_STATE, "no rule set compiled");
    if (int rc0 = eng->check_batch(batch)) return rc0;
    mxp_dbatch db;
    mxp_engine::PackedHost H;
    int rc = eng->pack_host(batch, &db, H);
    if (rc) return rc;
    const uint64_t bytes = H.kinds.size() + 8 * (H.vals.size() + H.ipof.size() + H.tsof.size() + db.overlay.size()) +
                           4 * (H.moff.size() + H.mk.size() + H.mv.size() + H.rxof.size()) + db.overlay.blob.size();
    const uint64_t v[3] = {bytes, db.overlay.size(), db.overlay_bytes.size()};
    for (uint32_t i = 0; out && i < cap && i < 3; i++) out[i] = v[i];
    return MXP_OK;
}

// The batch's device blocks go to the engine's bin (no hipFree: it would wait for the whole device),
// with the completion events of the batch's evaluations (recorded by launch on each stream it was
// evaluated on -- the free itself records nothing on a caller stream, which may be gone by now) and
// one on the engine stream (the packer): a later upload reuses a block only after those events.
void mxp_batch_free(mxp_engine* eng, mxp_dbatch* db) {
    if (!db) return;
    if (!eng || eng->device < 0) {
        delete db;
        return;
    }
    (void)hipSetDevice(eng->device);
    eng->recycle(db);
}

int mxp_host_alloc(size_t bytes, void** out) {
    if (!out) return MXP_ERR_ARG;
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
        *out = nullptr;
        return MXP_ERR_NOMEM;
    }
    return MXP_OK;
}

void mxp_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int mxp_debug_bin(mxp_engine* eng, uint64_t* out) {
    if (!eng || !out) return MXP_ERR_ARG;
    if (eng->device >= 0) (void)hipSetDevice(eng->device);
    out[0] = eng->bin.held();
    std::lock_guard<std::mutex> lk(eng->bin.mu);
    out[1] = eng->bin.cap_locked();
    return MXP_OK;
}

int mxp_batch_eval_device(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match, uint32_t* d_err) {
    if (!eng || !db || !d_match || !d_err) return MXP_ERR_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    return eng->launch(db, s, d_match, d_err, nullptr, false);
}

// device evaluation with fused or streamed hit counters; error output as a bitmap (d_err) or as
// per-request flags (d_req_err, compact)
static int eval_device_hits(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match, uint32_t* d_err,
                            uint8_t* d_req_err, unsigned long long* d_hits) {
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    hipError_t e;
    // (the request error flags are reset in launch: by a memset, or by the deferred-pair index kernel)
    if (!d_hits) {
        eng->req_err_out = d_req_err;
        const int rc = eng->launch(db, s, d_match, d_err, nullptr, false);
        eng->req_err_out = nullptr;
        return rc;
    }
    if (!eng->stats_ev) {
        if ((e = eng->d_stats.alloc(8)) != hipSuccess) return eng->hipfail(e, "stats");
        if ((e = eng->d_gate.alloc(8)) != hipSuccess) return eng->hipfail(e, "hits gate");
        if ((e = hipMemsetAsync(eng->d_stats.p, 0, 8, s)) != hipSuccess) return eng->hipfail(e, "stats reset");
        // no evaluation yet: stream the bitmap (a fused first evaluation of a rule set with many true
        // pairs would pay one atomic per pair: C4's first evaluations took 6.5 ms instead of 1.9)
        if ((e = hipMemsetAsync(eng->d_gate.p, 0, 8, s)) != hipSuccess) return eng->hipfail(e, "hits gate");
        if ((e = hipEventCreateWithFlags(&eng->stats_ev, kOrderEvent)) != hipSuccess) {
            eng->stats_ev = nullptr;
            return eng->hipfail(e, "stats event");
        }
    }
    // Fused vs streamed counters are chosen on the device (mxp_hits_gate_kernel after each
    // evaluation sets the next one's gate from its true pairs per request): no host round trip and no
    // stale decision when evaluations are queued back to back.
    const uint32_t R = (uint32_t)eng->rules.size(), W = (R + 31) / 32;
    const uint32_t force = (eng->debug_flags & 524288u) ? 1u : (eng->debug_flags & 1048576u) ? 2u : 0u;
    // (ordered after the previous evaluation's gate update even when the caller switched streams)
    if (eng->stats_pending && eng->stats_stream != s && (e = hipStreamWaitEvent(s, eng->stats_ev, 0)) != hipSuccess)
        return eng->hipfail(e, "stats wait");
    uint32_t* const gate = eng->d_gate.as<uint32_t>() + eng->gate_par;
    uint32_t* const gate_next = eng->d_gate.as<uint32_t>() + (eng->gate_par ^ 1u);
    if (force && (e = mxp_launch_hits_gate(eng->d_stats.as<unsigned long long>(), 0, W, gate, force, s)) != hipSuccess)
        return eng->hipfail(e, "hits gate");
    eng->req_err_out = d_req_err;
    eng->hits_gate_out = gate;
    eng->gate_next_out = gate_next;
    int rc = eng->launch(db, s, d_match, d_err, nullptr, false, d_hits, eng->d_stats.as<uint64_t>());
    eng->req_err_out = nullptr;
    eng->hits_gate_out = nullptr;
    eng->gate_next_out = nullptr;
    if (rc) return rc;
    // the streaming counters (returning at once when the kernels counted); their block (0, 0) also
    // sets the next evaluation's gate from this one's true pairs and resets the pair count.  A
    // deferred-pair evaluation counted everything in its kernels: only the gate update.
    const bool counted = eng->last_dtp_counted;
    if (R && db->n && !counted) {
        if ((e = mxp_launch_hits(d_match, db->n, R, W, d_hits, s, gate, eng->d_stats.as<unsigned long long>(), gate_next,
                                 force)) != hipSuccess)
            return eng->hipfail(e, "launch hits");
    } else if (!counted) {
        if ((e = mxp_launch_hits_gate(eng->d_stats.as<unsigned long long>(), db->n, W, gate_next, force, s)) != hipSuccess)
            return eng->hipfail(e, "hits gate");
        if ((e = hipMemsetAsync(eng->d_stats.p, 0, 8, s)) != hipSuccess) return eng->hipfail(e, "stats reset");
    }
    // (a counted evaluation kept no true-pair count: its post-fill index launch set the next gate to
    // 0 -- stream, should the next evaluation not be counted -- and the count was not touched)
    eng->gate_par ^= 1u;
    // mxp_kernel_times: the evaluation's span ends after the counters too (streamed or gate only)
    if (eng->timing && (e = hipEventRecord(eng->ev[2], s)) != hipSuccess) return eng->hipfail(e, "event");
    if ((e = hipEventRecord(eng->stats_ev, s)) != hipSuccess) return eng->hipfail(e, "stats event");
    eng->stats_pending = true;
    eng->stats_stream = s;
    return MXP_OK;
}

int mxp_batch_eval_device_hits(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match, uint32_t* d_err,
                               unsigned long long* d_hits) {
    if (!eng || !db || !d_match || !d_err || !d_hits) return MXP_ERR_ARG;
    return eval_device_hits(eng, db, stream, d_match, d_err, nullptr, d_hits);
}

int mxp_batch_eval_device_compact(mxp_engine* eng, mxp_dbatch* db, void* stream, uint32_t* d_match,
                                  uint8_t* d_req_err, unsigned long long* d_hits) {
    if (!eng || !db || !d_match || !d_req_err) return MXP_ERR_ARG;
    return eval_device_hits(eng, db, stream, d_match, nullptr, d_req_err, d_hits);
}

int mxp_hits_device(mxp_engine* eng, const uint32_t* d_match, uint32_t n_requests, void* stream,
                    unsigned long long* d_hits) {
    if (!eng || !d_match || !d_hits) return MXP_ERR_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    uint32_t R = (uint32_t)eng->rules.size();
    if (!R || !n_requests) return MXP_OK;
    hipError_t e = mxp_launch_hits(d_match, n_requests, R, (R + 31) / 32, d_hits, s);
    return e == hipSuccess ? MXP_OK : eng->hipfail(e, "launch hits");
}

int mxp_engine::check_batch(const mxp_bag_batch* b, int parts) {
    if (!b) return MXP_ERR_ARG;
    const uint64_t n = b->n_requests, NS = b->n_strings, NT = b->n_times, NM = b->n_maps;
    auto bad = [&](const std::string& what) { return fail(MXP_ERR_ARG, "malformed batch: " + what); };
    if (b->n_columns && !b->column_names) return bad("column_names is NULL");
    // (a narrow upload, mxp_batch_upload2: its u32 columns and offsets where the view has none)
    const mxp_bag_batch2* nb = narrow_src;
    const uint32_t* so32 = nb && !b->str_offsets ? nb->str_offsets32 : nullptr;
    const uint32_t* mo32 = nb && !b->map_offsets ? nb->map_offsets32 : nullptr;
    auto v32_of = [&](uint32_t c) -> const uint32_t* {
        return nb && nb->narrow[c] && nb->values32 ? nb->values32[c] : nullptr;
    };
    if (NS && !b->str_offsets && !so32) return bad("str_offsets is NULL");
    if (NT && (!b->time_sec || !b->time_nsec)) return bad("time_sec / time_nsec is NULL");
    if (NM && !b->map_offsets && !mo32) return bad("map_offsets is NULL");
    // the columns read (by name; the first column of a name is the one read)
    std::vector<std::string> names = read_attributes();
    std::set<std::string> want(names.begin(), names.end());
    std::vector<uint32_t> use;
    std::set<std::string> seen;
    std::atomic<bool> map_col{false};
    for (uint32_t c = 0; c < b->n_columns; c++) {
        if (!b->column_names[c]) return bad("column " + std::to_string(c) + " has no name");
        const std::string nm(b->column_names[c]);
        if (!want.count(nm) || !seen.insert(nm).second) continue;
        if (n && (!b->kinds || !b->kinds[c] || (!v32_of(c) && (!b->values || !b->values[c]))))
            return bad("column '" + nm + "' has no kinds / values");
        use.push_back(c);
    }
    // first failure per worker: (request or item index, message)
    struct Bad {
        uint64_t at = ~0ull;
        std::string what;
    };
    const unsigned T = mxp::pack_threads();
    std::vector<Bad> errs(T);
    auto note = [&](unsigned w, uint64_t at, std::string what) {
        if (at < errs[w].at) errs[w] = Bad{at, std::move(what)};
    };
    auto first = [&]() -> const Bad* {
        const Bad* f = nullptr;
        for (const Bad& x : errs)
            if (!x.what.empty() && (!f || x.at < f->at)) f = &x;
        return f;
    };
    // string offsets: non-decreasing, every string < 16 MiB (the pools' descriptor limit)
    if (NS && (parts & kCheckStrings)) {
        auto offs = [&](const auto* o) {
            mxp::par_for(NS, 1u << 16, [&](uint64_t i0, uint64_t i1, unsigned w) {
                for (uint64_t i = i0; i < i1; i++) {
                    if (o[i + 1] < o[i]) return note(w, i, "str_offsets[" + std::to_string(i + 1) + "] < str_offsets[" +
                                                               std::to_string(i) + "]");
                    if (o[i + 1] - o[i] >= (1u << 24)) return note(w, i, "string " + std::to_string(i) + " is 16 MiB or longer");
                }
            });
        };
        if (so32)
            offs(so32);
        else
            offs(b->str_offsets);
        if (const Bad* f = first()) return bad(f->what);
        if ((so32 ? (uint64_t)so32[NS] : b->str_offsets[NS]) && !b->str_bytes) return bad("str_bytes is NULL");
    }
    // columns: every used column over each slice of requests in one parallel pass, branch-free
    // (a kind's id limit from a table: ~0 for kinds without an id, 0 for kinds past MXP_OTHER); a
    // slice with a failure is rescanned for its message
    uint64_t lim_of[256];
    for (int kd = 0; kd < 256; kd++) lim_of[kd] = 0;
    for (int kd : {MXP_ABSENT, MXP_INT64, MXP_DOUBLE, MXP_BOOL, MXP_DURATION}) lim_of[kd] = ~0ull;
    for (int kd : {MXP_STRING, MXP_BYTES, MXP_OTHER}) lim_of[kd] = NS;
    lim_of[MXP_TIMESTAMP] = NT;
    lim_of[MXP_STRING_MAP] = NM;
    if (!(parts & kCheckColumns)) return MXP_OK;
    // (the u32 scan's limits: id > n - 1 is out of range; n = 0 rejects every id of the kind)
    auto m1 = [](uint64_t lim) { return lim == 0 ? 0u : (uint32_t)std::min<uint64_t>(lim - 1, 0xFFFFFFFFull); };
    const uint32_t ns1 = m1(NS), nt1 = m1(NT), nm1 = m1(NM);
    const uint32_t ns0 = NS == 0, nt0 = NT == 0, nm0 = NM == 0;
    if (!use.empty())
        mxp::par_for(n, 1u << 16, [&](uint64_t q0, uint64_t q1, unsigned w) {
            bool maps = false;
            for (uint32_t c : use) {
                const uint8_t* k = b->kinds[c];
                const uint32_t* v32 = v32_of(c);
                const uint64_t* v64 = v32 ? nullptr : b->values[c];
                bool fail_any = false;
                uint32_t nmap = 0;
                auto scan = [&](const auto* v) {
                    for (uint64_t q = q0; q < q1; q++) {
                        const uint64_t lim = lim_of[k[q]];
                        fail_any |= ((uint64_t)v[q] >= lim) & (lim != ~0ull);
                        nmap += k[q] == MXP_STRING_MAP;
                    }
                };
                if (v32) {
                    // u32 ids: the limits by compares instead of the table (no gather: the loop
                    // vectorises; 1M requests x 5 columns took 0.25 ms of the upload call, r6_s25)
                    uint32_t bad = 0, nm = 0;
                    for (uint64_t q = q0; q < q1; q++) {
                        const uint32_t kd = k[q], x = v32[q];
                        const uint32_t sk = (kd == MXP_STRING) | (kd == MXP_BYTES) | (kd == MXP_OTHER);
                        bad |= (sk & ((x > ns1) | ns0)) | ((kd == MXP_TIMESTAMP) & ((x > nt1) | nt0)) |
                               ((kd == MXP_STRING_MAP) & ((x > nm1) | nm0)) | (kd > MXP_OTHER);
                        nm += kd == MXP_STRING_MAP;
                    }
                    fail_any = bad != 0;
                    nmap = nm;
                } else {
                    scan(v64);
                }
                maps |= nmap != 0;
                if (!fail_any) continue;
                const std::string nm(b->column_names[c]);
                auto v = [&](uint64_t q) -> uint64_t { return v32 ? v32[q] : v64[q]; };
                for (uint64_t q = q0; q < q1; q++) {
                    const uint8_t kd = k[q];
                    if (kd > MXP_OTHER)
                        return note(w, q, "column '" + nm + "' request " + std::to_string(q) + ": kind " +
                                              std::to_string(kd) + " > MXP_OTHER");
                    if (lim_of[kd] != ~0ull && v(q) >= lim_of[kd]) {
                        const char* table = kd == MXP_TIMESTAMP ? "n_times" : kd == MXP_STRING_MAP ? "n_maps" : "n_strings";
                        return note(w, q, "column '" + nm + "' request " + std::to_string(q) + ": id " +
                                              std::to_string(v(q)) + " >= " + table + " (" + std::to_string(lim_of[kd]) + ")");
                    }
                }
            }
            if (maps) map_col.store(true, std::memory_order_relaxed);  // (once per slice)
        });
    if (const Bad* f = first()) return bad(f->what);
    // map CSR: offsets non-decreasing, key / value ids < n_strings (read when a map is)
    if (NM && (map_col.load() || need_maps || !vcols.empty())) {
        auto moffs = [&](const auto* mo) {
            mxp::par_for(NM, 1u << 16, [&](uint64_t m0, uint64_t m1, unsigned w) {
                for (uint64_t m = m0; m < m1; m++)
                    if (mo[m + 1] < mo[m])
                        return note(w, m, "map_offsets[" + std::to_string(m + 1) + "] < map_offsets[" + std::to_string(m) + "]");
            });
        };
        if (mo32)
            moffs(mo32);
        else
            moffs(b->map_offsets);
        if (const Bad* f = first()) return bad(f->what);
        auto mo = [&](uint64_t m) -> uint64_t { return mo32 ? mo32[m] : b->map_offsets[m]; };
        const uint64_t E = mo(NM) - mo(0);
        if (E && (!b->map_keys || !b->map_values)) return bad("map_keys / map_values is NULL");
        const uint64_t e0 = mo(0);
        mxp::par_for(E, 1u << 16, [&](uint64_t x0, uint64_t x1, unsigned w) {
            for (uint64_t x = e0 + x0; x < e0 + x1; x++) {
                if (b->map_keys[x] >= NS)
                    return note(w, x, "map entry " + std::to_string(x) + ": key id " + std::to_string(b->map_keys[x]) +
                                          " >= n_strings (" + std::to_string(NS) + ")");
                if (b->map_values[x] >= NS)
                    return note(w, x, "map entry " + std::to_string(x) + ": value id " +
                                          std::to_string(b->map_values[x]) + " >= n_strings (" + std::to_string(NS) + ")");
            }
        });
        if (const Bad* f = first()) return bad(f->what);
    }
    return MXP_OK;
}

int mxp_engine::evaluate(const mxp_bag_batch* batch, DevBuf& dm, DevBuf& de, DevBuf* dv,
                         std::unique_ptr<mxp_dbatch>& db, uint8_t* d_req_err) {
    if (!batch) return MXP_ERR_ARG;
    if (!have_rules) return fail(MXP_ERR_STATE, "no rule set compiled");
    if (device < 0) return fail(MXP_ERR_STATE, "host-only engine");
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hipfail(e, "hipSetDevice");
    db.reset(new mxp_dbatch());
    trace_mark(nullptr);
    g_bin_take = &bin;  // (the batch's own blocks recycled where the bin has them)
    g_bin_db = db.get();
    g_bin_db_size = sizeof(mxp_dbatch);
    int rc = pack(batch, db.get());
    g_bin_take = nullptr;
    g_bin_db = nullptr;
    if (rc) return rc;
    trace_mark("pack + upload");
    return evaluate_uploaded(db.get(), dm, de, dv, d_req_err);
}

int mxp_engine::evaluate_uploaded(mxp_dbatch* db, DevBuf& dm, DevBuf& de, DevBuf* dv, uint8_t* d_req_err) {
    hipError_t e;
    int rc;
    const uint32_t n = db->n;
    const uint32_t R = (uint32_t)rules.size();
    const uint32_t W = (R + 31) / 32;
    if ((e = dm.reserve((size_t)W * n * 4)) != hipSuccess) return hipfail(e, "alloc match");
    if (!d_req_err && (e = de.reserve((size_t)W * n * 4)) != hipSuccess) return hipfail(e, "alloc err");
    if (dv && (e = dv->reserve((size_t)n * R * 8)) != hipSuccess) return hipfail(e, "alloc values");
    trace_mark("bitmap allocation");
    req_err_out = d_req_err;
    rc = launch(db, stream, dm.as<uint32_t>(), d_req_err ? nullptr : de.as<uint32_t>(),
                dv ? dv->as<uint64_t>() : nullptr, true);
    req_err_out = nullptr;
    trace_mark("evaluation kernels");
    return rc;
}

// Synchronous download of `bytes` from device memory into caller memory, ordered after the work
// already queued on the engine stream.  Into pinned memory: a shader copy (mxp_d2h_copy_kernel,
// ~54 GB/s on the box against ~30 GB/s for the copy engine's DMA; MXP_D2H_DMA=1 keeps the DMA);
// into pageable memory: small copies direct, larger ones through the pinned bounce pair (chunk
// k + 1 copied beside the parallel host copy of chunk k).
bool mxp_engine::is_pinned(const void* p) { return host_dev_ptr(p) != nullptr; }

// the device address of pinned host memory at p (nullptr: pageable)
void* mxp_engine::host_dev_ptr(const void* p) {
    hipPointerAttribute_t pa;
    const bool ok = hipPointerGetAttributes(&pa, p) == hipSuccess && pa.type == hipMemoryTypeHost &&
                    pa.hostPointer != nullptr && pa.devicePointer != nullptr && (const char*)p >= (const char*)pa.hostPointer;
    (void)hipGetLastError();  // (pageable memory: the query fails)
    // (the pair names the same byte, whether the runtime reports it at p or at the allocation's base)
    return ok ? (void*)((char*)pa.devicePointer + ((const char*)p - (const char*)pa.hostPointer)) : nullptr;
}

// one device -> pinned-host copy queued on the engine stream (hd: host_dev_ptr of dst)
hipError_t mxp_engine::queue_d2h(void* dst, void* hd, const void* dsrc, size_t bytes) {
    if (!bytes) return hipSuccess;
    if (d2h_dma || bytes < kShaderCopyMin) return hipMemcpyAsync(dst, dsrc, bytes, hipMemcpyDeviceToHost, stream);
    return mxp_launch_d2h_copy(hd, dsrc, bytes, stream);
}

int mxp_engine::download_all(const std::vector<Piece>& pieces, const char* what) {
    hipError_t e;
    bool queued = false;
    for (const Piece& p : pieces) {
        void* hd = p.bytes ? host_dev_ptr(p.dst) : nullptr;
        if (!hd) continue;
        if ((e = queue_d2h(p.dst, hd, p.src, p.bytes)) != hipSuccess) return hipfail(e, what);
        queued = true;
    }
    if (queued && (e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, what);
    if (trace && queued) fprintf(stderr, "mxp trace     download_all %s: pinned pieces queued together\n", what);
    for (const Piece& p : pieces) {
        if (!p.bytes || is_pinned(p.dst)) continue;
        if (int rc = download(p.dst, p.src, p.bytes, what)) return rc;
    }
    return MXP_OK;
}

int mxp_engine::download(void* dst, const void* dsrc, size_t bytes, const char* what) {
    hipError_t e;
    if (!bytes) return MXP_OK;
    // caller memory that is pinned (mxp_host_alloc arenas): straight into it
    const double t0 = trace ? mxp::now_seconds() : 0.0;
    auto note = [&](const char* path) {
        if (trace)
            fprintf(stderr, "mxp trace     download %-20s %10zu B %s %8.3f ms\n", what, bytes, path,
                    (mxp::now_seconds() - t0) * 1e3);
    };
    if (void* hd = bytes >= kShaderCopyMin ? host_dev_ptr(dst) : nullptr) {
        if ((e = queue_d2h(dst, hd, dsrc, bytes)) != hipSuccess) return hipfail(e, what);
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, what);
        note(d2h_dma ? "pinned dma" : "pinned shader");
        return MXP_OK;
    }
    if (bytes < (64u << 10)) {
        if ((e = hipMemcpyAsync(dst, dsrc, bytes, hipMemcpyDeviceToHost, stream)) != hipSuccess) return hipfail(e, what);
        if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, what);
        return MXP_OK;
    }
    // (from 64 KiB on, pageable memory goes through the bounce buffers: a pageable hipMemcpy of C2's
    // 214 KB of error records took 0.55 ms)
    void* bounce_d[2] = {nullptr, nullptr};
    for (int k = 0; k < 2; k++) {
        if (!bounce[k] && (e = hipHostMalloc(&bounce[k], kBounce, hipHostMallocDefault)) != hipSuccess) {
            bounce[k] = nullptr;
            return hipfail(e, "bounce buffer");
        }
        if (!bounce_ev[k] && (e = hipEventCreateWithFlags(&bounce_ev[k], hipEventDisableTiming)) != hipSuccess) {
            bounce_ev[k] = nullptr;
            return hipfail(e, "bounce event");
        }
        bounce_d[k] = host_dev_ptr(bounce[k]);
        if (!bounce_d[k]) return fail(MXP_ERR_DEVICE, "bounce buffer not mapped");
    }
    const size_t nchunk = (bytes + kBounce - 1) / kBounce;
    auto issue = [&](size_t c) -> hipError_t {
        const size_t off = c * kBounce, len = std::min(kBounce, bytes - off);
        hipError_t r = queue_d2h(bounce[c & 1], bounce_d[c & 1], (const uint8_t*)dsrc + off, len);
        return r == hipSuccess ? hipEventRecord(bounce_ev[c & 1], stream) : r;
    };
    for (size_t c = 0; c < std::min<size_t>(2, nchunk); c++)
        if ((e = issue(c)) != hipSuccess) return hipfail(e, what);
    for (size_t c = 0; c < nchunk; c++) {
        if ((e = hipEventSynchronize(bounce_ev[c & 1])) != hipSuccess) return hipfail(e, what);
        const size_t off = c * kBounce, len = std::min(kBounce, bytes - off);
        const uint8_t* from = (const uint8_t*)bounce[c & 1];
        uint8_t* to = (uint8_t*)dst + off;
        mxp::par_for(len, 1u << 20, [&](uint64_t a, uint64_t b, unsigned) { memcpy(to + a, from + a, b - a); });
        if (c + 2 < nchunk && (e = issue(c + 2)) != hipSuccess) return hipfail(e, what);
    }
    note("bounce");
    return MXP_OK;
}

int mxp_engine::collect_errors(const mxp_bag_batch* batch, std::unique_ptr<mxp_dbatch>& db) {
    hipError_t e;
    // [0] records of the log, [1] error pairs of value-class rules, [2] class records
    uint32_t cnt[4] = {0, 0, 0, 0};
    if ((e = hipMemcpyAsync(cnt, d_errcount.p, 16, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hipfail(e, "download errcount");
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, "eval sync");
    trace_mark("  errors: counts");
    last_error_count = (uint64_t)cnt[0] + cnt[1];
    clear_errors();
    trace_mark("  errors: clear");
    err_windows.clear();
    errors_complete = cnt[0] <= errcap;
    uint32_t kept = std::min(cnt[0], errcap);
    if (kept && lazy_records && !cnt[2] && !cnt[3]) {
        // no conversion error and no class record: the records stay where the kernels wrote them
        // (that buffer set aside from the next evaluation) until a text is asked for
        d_errlog.swap(d_errlog_prev);
        recs_pending = kept;
        kept = 0;
    }
    if (kept) {
        last_recs.resize(kept);
        if (int rc = download(last_recs.data(), d_errlog.p, kept * sizeof(mxp_err_rec), "download errlog")) return rc;
        // conversion errors print the caller's value: formatted now (the others when asked); the
        // records scanned in parallel, the per-record text index kept only when one exists
        std::atomic<bool> conv{false};
        mxp::par_for(kept, 1u << 16, [&](uint64_t i0, uint64_t i1, unsigned) {
            bool any = false;
            for (uint64_t i = i0; i < i1; i++) any |= last_recs[i].code >= ERR_CONV_S && last_recs[i].code <= ERR_CONV_D;
            if (any) conv.store(true, std::memory_order_relaxed);
        });
        if (conv.load()) {
            last_rec_text.assign(kept, -1);
            for (uint32_t i = 0; i < kept; i++)
                if (last_recs[i].code >= ERR_CONV_S && last_recs[i].code <= ERR_CONV_D) {
                    last_rec_text[i] = (int32_t)last_rec_texts.size();
                    last_rec_texts.push_back(format_error(batch, db.get(), last_recs[i]));
                }
        }
    }
    trace_mark("  errors: records");
    if (cnt[2]) {
        int rc = expand_class_errors(batch, db.get(), cnt[2], errcap > kept ? errcap - kept : 0u);
        if (rc) return rc;
    }
    // records past the log are recomputed after the caller's batch is gone: keep its map texts when
    // the device batch has no map contents to print them from
    const uint32_t NM = batch->n_maps;
    if (!errors_complete && NM && db && db->map_off.n < ((size_t)NM + 1) * 4) {
        snap_maps.resize(NM);
        auto bs = [&](uint64_t sid) {
            return std::string((const char*)batch->str_bytes + batch->str_offsets[sid],
                               (size_t)(batch->str_offsets[sid + 1] - batch->str_offsets[sid]));
        };
        mxp::par_for(NM, 4096, [&](uint64_t m0, uint64_t m1, unsigned) {
            for (uint64_t m = m0; m < m1; m++) {
                std::string t = "map[";
                for (uint64_t x = batch->map_offsets[m]; x < batch->map_offsets[m + 1]; x++)
                    t += (x != batch->map_offsets[m] ? " " : "") + bs(batch->map_keys[x]) + ":" + bs(batch->map_values[x]);
                snap_maps[m] = t + "]";
            }
        });
    }
    trace_mark("  errors: map texts");
    recycle(last_db.release());  // (the previous batch's blocks: to the bin, not hipFree)
    last_db = std::move(db);
    trace_mark("  errors: recycle");
    return MXP_OK;
}

// Class records of the last evaluation (mxp_vt_eval_kernel logs each failing (class, rule) once,
// at the class's representative request): every request of the class fails that rule the same
// way, so each record stands for the pairs of all of them.  Expanded here up to `room` records;
// past it the rest are recomputed on demand like any record past the log's capacity.
int mxp_engine::expand_class_errors(const mxp_bag_batch* batch, mxp_dbatch* db, uint32_t n_class, uint32_t room) {
    hipError_t e;
    if (n_class > vtlog_cap || !last_mask) {
        errors_complete = false;
        return MXP_OK;
    }
    std::vector<mxp_err_rec> recs(n_class);
    if ((e = hipMemcpy(recs.data(), d_vtlog.p, n_class * sizeof(mxp_err_rec), hipMemcpyDeviceToHost)) != hipSuccess)
        return hipfail(e, "download class errlog");
    const uint32_t n = db->n, act = (uint32_t)__builtin_popcount(last_mask);
    const size_t pitch = MXP_VT_PITCH(n);
    std::vector<uint16_t> cls((size_t)act * pitch);
    if ((e = hipMemcpy(cls.data(), db->vt_cls.p, cls.size() * 2, hipMemcpyDeviceToHost)) != hipSuccess)
        return hipfail(e, "download classes");
    // requests of every class, per active slot (counting sort by class)
    std::vector<std::vector<uint32_t>> start(act), reqs(act);
    for (uint32_t a = 0; a < act; a++) {
        const uint32_t cap = db->vt_meta_h[a * 8 + MXP_VTM_CAP];
        const uint16_t* c = cls.data() + (size_t)a * pitch;
        start[a].assign(cap + 1, 0);
        for (uint32_t q = 0; q < n; q++) start[a][c[q] + 1]++;
        for (uint32_t k = 0; k < cap; k++) start[a][k + 1] += start[a][k];
        std::vector<uint32_t> at(start[a].begin(), start[a].end() - 1);
        reqs[a].resize(n);
        for (uint32_t q = 0; q < n; q++) reqs[a][at[c[q]]++] = q;
    }
    uint64_t emitted = 0;
    for (const mxp_err_rec& r : recs) {
        const uint32_t s = vt_slot_of_rule[r.rule];
        const uint32_t a = (uint32_t)__builtin_popcount(last_mask & ((1u << s) - 1u));
        const uint32_t k = cls[(size_t)a * pitch + r.req];
        // (every request of the class prints the same value: one text per class record)
        int32_t text = -1;
        if (r.code >= ERR_CONV_S && r.code <= ERR_CONV_D) {
            text = (int32_t)last_rec_texts.size();
            last_rec_texts.push_back(format_error(batch, db, r));
        }
        for (uint32_t i = start[a][k]; i < start[a][k + 1]; i++) {
            if (emitted >= room) {
                errors_complete = false;
                return MXP_OK;
            }
            mxp_err_rec x = r;
            x.req = reqs[a][i];
            last_recs.push_back(x);
            if (text >= 0 || !last_rec_text.empty()) {  // (the index exists once a record has a text)
                last_rec_text.resize(last_recs.size() - 1, -1);
                last_rec_text.push_back(text);
            }
            emitted++;
        }
    }
    return MXP_OK;
}

// Error records past the log's capacity: re-evaluate the window of kErrWindow requests holding
// `request` (same kernels, no bitmap outputs, a fresh log) and add its records to last_errors.
int mxp_engine::recompute_errors(uint32_t request) {
    if (!last_db || request >= last_db->n) return MXP_OK;
    const uint32_t w = request / kErrWindow;
    if (!err_windows.insert(w).second) return MXP_OK;
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return hipfail(e, "hipSetDevice");
    const uint32_t q0 = w * kErrWindow, q1 = std::min(last_db->n, q0 + kErrWindow);
    // (rules fail at most once per request and rule; aliases of an indexed rule are distinct rules)
    win_log_cap = (q1 - q0) * (uint32_t)std::max<size_t>(rules.size(), 1);
    int rc = launch(last_db.get(), stream, nullptr, nullptr, nullptr, true, nullptr, nullptr, q0, q1);
    const uint32_t cap = win_log_cap;
    win_log_cap = 0;
    if (rc) return rc;
    uint32_t cnt = 0;
    if ((e = hipMemcpyAsync(&cnt, d_wincount.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess)
        return hipfail(e, "download errcount");
    if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hipfail(e, "recompute sync");
    const uint32_t kept = std::min(cnt, cap);
    ErrWindow win;
    win.q0 = q0;
    win.q1 = q1;
    win.ncol = (uint32_t)(cols.size() + vcols.size());
    std::vector<mxp_err_rec> recs(kept);
    if (kept && (e = hipMemcpy(recs.data(), d_winlog.p, kept * sizeof(mxp_err_rec), hipMemcpyDeviceToHost)) != hipSuccess)
        return hipfail(e, "download errlog");
    bool conv = false;
    for (auto& r : recs) conv |= r.code >= ERR_CONV_S && r.code <= ERR_CONV_D;
    if (conv) {  // the window's columns, for the values conversion errors print
        const size_t wn = q1 - q0;
        win.kinds.resize(win.ncol * wn);
        win.vals.resize(win.ncol * wn);
        for (uint32_t c = 0; c < win.ncol; c++) {
            if ((e = hipMemcpy(win.kinds.data() + c * wn, last_db->kinds.as<uint8_t>() + (size_t)c * last_db->n + q0, wn,
                               hipMemcpyDeviceToHost)) != hipSuccess ||
                (e = hipMemcpy(win.vals.data() + c * wn, last_db->vals.as<uint64_t>() + (size_t)c * last_db->n + q0,
                               wn * 8, hipMemcpyDeviceToHost)) != hipSuccess)
                return hipfail(e, "download window columns");
        }
    }
    for (auto& r : recs) {
        const uint64_t key = ((uint64_t)r.req << 32) | r.rule;
        if (!last_errors.count(key)) last_errors[key] = {r.code, format_error(nullptr, last_db.get(), r, &win)};
    }
    return MXP_OK;
}

// the record the last batch logged for `key`, or -1 (the index over the records is built on first use)
// the deferred records of the last evaluation into last_recs (collect_errors)
int mxp_engine::ensure_recs() {
    if (!recs_pending) return MXP_OK;
    const uint32_t k = recs_pending;
    recs_pending = 0;
    last_recs.resize(k);
    if (int rc = download(last_recs.data(), d_errlog_prev.p, (size_t)k * sizeof(mxp_err_rec), "download errlog")) {
        last_recs.clear();
        return rc;
    }
    rec_indexed = false;
    return MXP_OK;
}

int64_t mxp_engine::logged_record(uint64_t key) {
    if (ensure_recs()) return -1;
    if (!rec_indexed) {
        rec_index.reserve(last_recs.size());
        for (uint32_t i = 0; i < (uint32_t)last_recs.size(); i++)
            rec_index.emplace(((uint64_t)last_recs[i].req << 32) | last_recs[i].rule, i);
        rec_indexed = true;
    }
    auto it = rec_index.find(key);
    return it == rec_index.end() ? -1 : (int64_t)it->second;
}

// text (when `text` is non-null) and code of a pair's error in the last batch; ERR_NONE when the
// pair did not fail
int mxp_engine::pair_error_text(uint32_t request, uint32_t rule, std::string* text, uint32_t* code) {
    const uint64_t key = ((uint64_t)request << 32) | rule;
    auto it = last_errors.find(key);
    if (it == last_errors.end()) {
        const int64_t i = logged_record(key);
        if (i >= 0) {
            const mxp_err_rec& r = last_recs[(size_t)i];
            *code = r.code;
            if (text) {
                const int32_t t = (size_t)i < last_rec_text.size() ? last_rec_text[(size_t)i] : -1;
                *text = t >= 0 ? last_rec_texts[(size_t)t] : format_error(nullptr, last_db.get(), r);
                last_errors[key] = {r.code, *text};
            }
            return MXP_OK;
        }
    }
    if (it == last_errors.end() && !errors_complete) {
        int rc = recompute_errors(request);
        if (rc) return rc;
        it = last_errors.find(key);
    }
    if (it == last_errors.end()) {
        if (text) text->clear();
        *code = ERR_NONE;
    } else {
        if (text) *text = it->second.second;
        *code = it->second.first;
    }
    return MXP_OK;
}

static int eval_common(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t* match_bits, uint32_t* err_bits,
                       uint64_t* values, uint8_t* codes) {
    if (!eng || !batch) return MXP_ERR_ARG;
    std::unique_ptr<mxp_dbatch> db;
    DevBuf dm, de, dv;
    int rc = eng->evaluate(batch, dm, de, values ? &dv : nullptr, db);
    if (rc) return rc;
    const uint32_t n = batch->n_requests;
    const uint32_t R = (uint32_t)eng->rules.size();
    const uint32_t W = (R + 31) / 32;
    // bitmaps go straight into the caller's arrays; host copies only when per-pair codes are wanted
    std::vector<uint32_t> hm, he;
    if (codes) {
        hm.resize((size_t)W * n);
        he.resize((size_t)W * n);
    }
    uint32_t* to_m = codes ? hm.data() : match_bits;
    uint32_t* to_e = codes ? he.data() : err_bits;
    if (to_m && (rc = eng->download(to_m, dm.p, (size_t)W * n * 4, "download match"))) return rc;
    if (to_e && (rc = eng->download(to_e, de.p, (size_t)W * n * 4, "download err"))) return rc;
    if (values && (rc = eng->download(values, dv.p, (size_t)n * R * 8, "download values"))) return rc;
    if ((rc = eng->collect_errors(batch, db))) return rc;
    if (codes && match_bits) memcpy(match_bits, hm.data(), hm.size() * 4);
    if (codes && err_bits) memcpy(err_bits, he.data(), he.size() * 4);
    if (codes) {
        for (uint32_t q = 0; q < n; q++)
            for (uint32_t r = 0; r < R; r++) {
                size_t w = (size_t)(r / 32) * n + q;
                uint32_t bit = 1u << (r % 32);
                uint8_t c = (hm[w] & bit) ? PC_TRUE : PC_FALSE;
                if (he[w] & bit) {
                    uint32_t code = ERR_NONE;
                    if ((rc = eng->pair_error_text(q, r, nullptr, &code))) return rc;
                    c = code >= 32 ? PC_PANIC : PC_ERROR;
                }
                codes[(size_t)q * R + r] = c;
            }
    }
    return MXP_OK;
}

int mxp_eval_batch(mxp_engine* eng, const mxp_bag_batch* batch, uint32_t* match_bits, uint32_t* err_bits) {
    return eval_common(eng, batch, match_bits, err_bits, nullptr, nullptr);
}

int mxp_eval_values(mxp_engine* eng, const mxp_bag_batch* batch, uint64_t* values, uint8_t* codes) {
    return eval_common(eng, batch, nullptr, nullptr, values, codes);
}

int mxp_pair_error(mxp_engine* eng, uint32_t request, uint32_t rule, char* buf, uint32_t cap) {
    if (!eng) return MXP_ERR_ARG;
    std::string t;
    uint32_t code = ERR_NONE;
    int rc = eng->pair_error_text(request, rule, &t, &code);
    if (rc) return rc;
    rc = put_text(t, buf, cap);
    return rc ? rc : (code >= 32 ? 1 : 0);
}

uint64_t mxp_error_count(mxp_engine* eng) { return eng ? eng->last_error_count : 0; }

int mxp_value_kind(mxp_engine* eng, uint32_t rule, uint64_t v) {
    if (!eng || rule >= eng->rules.size()) return -1;
    switch (eng->rules[rule].il_ret) {
    case mxp::IL_STRING: return MXP_STRING;
    case mxp::IL_BOOL: return MXP_BOOL;
    case mxp::IL_INTEGER: return MXP_INT64;
    case mxp::IL_DURATION: return MXP_DURATION;
    case mxp::IL_DOUBLE: return MXP_DOUBLE;
    default: return (int)MXP_FH_KIND(v);
    }
}

int mxp_value_decode(mxp_engine* eng, uint32_t rule, uint64_t v, mxp_value* out, uint8_t* buf, uint32_t cap) {
    if (!eng || !out || rule >= eng->rules.size()) return MXP_ERR_ARG;
    mxp_value r{};
    const int k = mxp_value_kind(eng, rule, v);
    const uint64_t id = (eng->rules[rule].il_ret == mxp::IL_INTERFACE) ? MXP_FH_ID(v) : v;
    r.kind = (uint32_t)k;
    std::string bytes;
    switch (k) {
    case MXP_STRING: bytes = eng->string_of(nullptr, id); break;
    case MXP_BOOL: r.i = (uint32_t)v != 0; break;
    case MXP_INT64: case MXP_DURATION: r.i = (int64_t)v; break;
    case MXP_DOUBLE: memcpy(&r.d, &v, 8); break;
    case MXP_BYTES: {
        const uint64_t raw = MXP_BYTES_RAW(id);
        if (raw < eng->gbytes.size()) bytes = eng->gbytes[raw];
        else if (eng->last_db) eng->last_db->overlay_bytes_at(raw - eng->gbytes.size(), &bytes);
        break;
    }
    case MXP_TIMESTAMP: {
        TimeKey t{0, 0};
        if (id < eng->gtimes.size()) t = eng->gtimes[id];
        else if (eng->last_db) eng->last_db->overlay_time(id - eng->gtimes.size(), &t);
        r.i = t.s;
        r.nsec = t.ns;
        break;
    }
    case MXP_STRING_MAP: {  // the batch's map CSR (device), keys and values by interned id
        const mxp_dbatch* db = eng->last_db.get();
        uint32_t mo[2] = {0, 0};
        if (!db || hipMemcpy(mo, db->map_off.as<uint32_t>() + id, 8, hipMemcpyDeviceToHost) != hipSuccess)
            return eng->fail(MXP_ERR_STATE, "map value without its batch");
        std::vector<uint32_t> ks(mo[1] - mo[0]), vs(mo[1] - mo[0]);
        if (!ks.empty() &&
            (hipMemcpy(ks.data(), db->map_keys.as<uint32_t>() + mo[0], ks.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
             hipMemcpy(vs.data(), db->map_vals.as<uint32_t>() + mo[0], vs.size() * 4, hipMemcpyDeviceToHost) != hipSuccess))
            return eng->fail(MXP_ERR_DEVICE, "map value download");
        auto put = [&](const std::string& x) {
            const uint32_t len = (uint32_t)x.size();
            bytes.append((const char*)&len, 4);
            bytes += x;
        };
        for (size_t e = 0; e < ks.size(); e++) {
            put(eng->string_of(db, ks[e]));
            put(eng->string_of(db, vs[e]));
        }
        r.i = (int64_t)ks.size();
        break;
    }
    default: return eng->fail(MXP_ERR_ARG, "value of an unknown kind");
    }
    r.n = (uint32_t)bytes.size();
    *out = r;
    if (bytes.size() > cap) return MXP_ERR_NOMEM;
    if (!bytes.empty()) memcpy(buf, bytes.data(), bytes.size());
    return MXP_OK;
}

int mxp_value_text(mxp_engine* eng, uint32_t rule, uint64_t v, char* buf, uint32_t cap) {
    if (!eng || rule >= eng->rules.size()) return MXP_ERR_ARG;
    std::string s;
    int k = mxp_value_kind(eng, rule, v);
    uint64_t id = (eng->rules[rule].il_ret == mxp::IL_INTERFACE) ? MXP_FH_ID(v) : v;
    switch (k) {
    case MXP_STRING: s = eng->string_of(nullptr, id); break;
    case MXP_BOOL: s = v ? "true" : "false"; break;
    case MXP_INT64: s = std::to_string((int64_t)v); break;
    case MXP_DURATION: s = mxp::go_format_duration((int64_t)v); break;
    case MXP_DOUBLE: {
        double d;
        memcpy(&d, &v, 8);
        s = mxp::go_format_float(d);
        break;
    }
    case MXP_BYTES: {
        std::string c;
        uint64_t raw = MXP_BYTES_RAW(id);
        if (raw < eng->gbytes.size()) c = eng->gbytes[raw];
        else if (eng->last_db) eng->last_db->overlay_bytes_at(raw - eng->gbytes.size(), &c);
        s = mxp::go_format_bytes((const uint8_t*)c.data(), c.size());
        break;
    }
    case MXP_TIMESTAMP: {
        TimeKey t{0, 0};
        if (id < eng->gtimes.size()) t = eng->gtimes[id];
        else if (eng->last_db) eng->last_db->overlay_time(id - eng->gtimes.size(), &t);
        s = mxp::go_format_time_utc(t.s, t.ns);
        break;
    }
    default: s = "?"; break;
    }
    return put_text(s, buf, cap);
}

}  // extern "C"
