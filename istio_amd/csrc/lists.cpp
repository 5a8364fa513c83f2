// lists.cpp -- list adapter (mixer/adapter/list) compile + batched checks (include/mxp.h).
//
// Compilation follows the handler's list builders:
//   STRINGS / CASE_INSENSITIVE_STRINGS  parseStringList / parseCaseInsensitiveStringList
//                                       (stringList.go:29-67): a set of the non-empty entries and
//                                       overrides (Go's strings.ToUpper for the case-insensitive
//                                       kind, goupper.h);
//   IP_ADDRESSES                        parseIPList / addEntry (ipList.go:35-75): "/32" appended when
//                                       the entry has no '/', net.ParseCIDR; the IPNets become
//                                       disjoint sorted address intervals (IPNet.Contains per
//                                       family after To4), so a check is a binary search instead of
//                                       the reference's linear scan (ipList.go:77-92).
// Checks run HandleListEntry (list.go:68-101) on the GPU (lists.hip).
#include <algorithm>
#include <cstring>
#include <functional>
#include <limits>

#include "engine_impl.h"
#include "goupper.h"
#include "lists.h"

extern "C" hipError_t mxp_launch_list(const mxp_list_args* a, hipStream_t s);

constexpr uint32_t kListRegexStates = 1u << 22;  // state budget of one part's union DFA (4M states)
constexpr uint64_t kListPartStates = 1u << 20;   // parts are packed to ~1M states of single-pattern DFAs
constexpr uint32_t kPatternStates = 1u << 16;    // one pattern over this: its own bit-parallel NFA

struct mxp_list {
    int type = 0;
    uint64_t n_entries = 0;
    uint32_t hmask = 0;
    DevBuf htab, ent_desc, ent_pool, v4lo, v4hi, v6lo, v6hi, v4dir;
    DevBuf rx_hdr, rx_trans, rx_ascii, rx_hilo, rx_hicls;  // REGEX: the parts' automata
    uint32_t n4 = 0, n6 = 0, rx_n = 0, rx_nfa = 0;
    uint32_t lds_nparts = 0;
    DevBuf lds_plan;  // REGEX: [K per staged part][LDS word base per staged part] (lists.h)
    NfaScratch nfa_scratch;  // REGEX: thread sets of NFA parts wider than the private-memory walk
    DevBuf rxp_tab, rxp_blk, rxp_lead;  // REGEX: literal-prefix dispatch (lists.h MXP_RXP_*)
    uint32_t rxp_mask = 0, rxp_short = 0, rxp_n = 0, rxp_keys = 0;
};

namespace {

const uint32_t kUpperRows[MXP_UPPER_N][3] = {MXP_UPPER_ROWS};

// The tail block (lists.h MXP_RXP_*) of a pattern whose every match starts with the literal bytes
// `pre` (regex_required_prefix): its DFA stepped over the prefix, then the states reachable from
// there with their transitions over the classes the tail tells apart.  False when the tail does not
// fit a block: more than MXP_RXP_STATES states, 16 classes or MXP_RXP_BLOCK_MAX bytes, an NFA, or a state where
// non-ASCII runes lead anywhere but to a decision.  *never: no subject starting with the prefix
// matches (the pattern can be dropped: its prefix is required).
bool rxp_block(const mxp::Dfa& d, std::string pre, std::vector<uint8_t>* out, bool* never) {
    *never = false;
    if (d.is_nfa() || pre.empty()) return false;
    // at most MXP_RXP_MAXPRE bytes, cut at a rune boundary (the DFA steps runes)
    if (pre.size() > MXP_RXP_MAXPRE) {
        size_t L = MXP_RXP_MAXPRE;
        while (L > 0 && ((uint8_t)pre[L] & 0xC0u) == 0x80u) L--;
        pre.resize(L);
        if (pre.empty()) return false;
    }
    auto cls_of_rune = [&](uint32_t r) -> uint32_t {
        if (r < 0x80) return d.ascii[r];
        const size_t at = std::upper_bound(d.hi_lo.begin(), d.hi_lo.end(), r) - d.hi_lo.begin() - 1;
        return d.hi_cls[at];
    };
    uint32_t st = d.start;
    for (size_t b = 0; b < pre.size() && st < mxp::kDfaReject;) {
        const uint8_t c = (uint8_t)pre[b];
        uint32_t r = c, w = 1;
        if (c >= 0x80) {  // a literal rune's UTF-8 bytes (valid: the prefix holds literal runes)
            w = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
            r = c & (0xFFu >> (w + 1));
            for (uint32_t k = 1; k < w; k++) r = (r << 6) | ((uint8_t)pre[b + k] & 0x3Fu);
        }
        st = d.trans[(size_t)st * d.ncls + cls_of_rune(r)];
        b += w;
    }
    if (st == mxp::kDfaReject) {
        *never = true;
        return false;
    }
    std::vector<uint32_t> states;  // tail state -> DFA state (BFS from the state after the prefix)
    std::unordered_map<uint32_t, uint32_t> idx;
    if (st != mxp::kDfaAccept) {
        states.push_back(st);
        idx[st] = 0;
        for (size_t i = 0; i < states.size(); i++)
            for (uint32_t c = 0; c < d.ncls; c++) {
                const uint32_t t = d.trans[(size_t)states[i] * d.ncls + c];
                if (t >= mxp::kDfaReject || idx.count(t)) continue;
                if (states.size() >= MXP_RXP_STATES) return false;
                idx[t] = (uint32_t)states.size();
                states.push_back(t);
            }
    }
    const uint32_t S = (uint32_t)states.size();
    auto code = [&](uint32_t t) -> uint8_t {
        return t == mxp::kDfaAccept ? (uint8_t)MXP_RXP_ACC : t == mxp::kDfaReject ? (uint8_t)MXP_RXP_REJ : (uint8_t)idx[t];
    };
    // non-ASCII runes: per state one decided target for every class a non-ASCII range maps to
    std::vector<uint8_t> hi(S, MXP_RXP_REJ);
    for (uint32_t k = 0; k < S; k++) {
        bool first = true;
        for (uint16_t c : d.hi_cls) {
            const uint32_t t = d.trans[(size_t)states[k] * d.ncls + c];
            if (t < mxp::kDfaReject) return false;
            if (!first && code(t) != hi[k]) return false;
            hi[k] = code(t);
            first = false;
        }
    }
    // ASCII bytes grouped by their tail columns
    std::map<std::vector<uint8_t>, uint32_t> sig_id;
    std::vector<std::vector<uint8_t>> cols;
    uint8_t byte_cls[128];
    for (uint32_t b = 0; b < 128; b++) {
        std::vector<uint8_t> sig(S);
        for (uint32_t k = 0; k < S; k++) sig[k] = code(d.trans[(size_t)states[k] * d.ncls + d.ascii[b]]);
        auto it = sig_id.find(sig);
        if (it == sig_id.end()) {
            it = sig_id.emplace(sig, (uint32_t)cols.size()).first;
            cols.push_back(sig);
        }
        byte_cls[b] = (uint8_t)it->second;
    }
    const uint32_t C = (uint32_t)cols.size() + 2;
    if (C > 16 || MXP_RXP_TRANS + S * C > MXP_RXP_BLOCK_MAX) return false;
    const uint32_t bytes = (MXP_RXP_TRANS + S * C + 15u) & ~15u;
    out->assign(bytes, 0);
    uint8_t* B = out->data();
    B[0] = (uint8_t)S;
    B[1] = (uint8_t)C;
    B[2] = (uint8_t)pre.size();
    B[3] = (uint8_t)(bytes / 16u);
    memcpy(B + 4, pre.data(), pre.size());
    for (uint32_t b = 0; b < 128; b++) B[32 + b / 2] |= (uint8_t)(byte_cls[b] << (4 * (b & 1)));
    for (uint32_t k = 0; k < S; k++) {
        uint8_t* row = B + MXP_RXP_TRANS + k * C;
        for (uint32_t c = 0; c + 2 < C; c++) row[c] = cols[c][k];
        row[C - 2] = hi[k];
        row[C - 1] = code(d.trans[(size_t)states[k] * d.ncls + d.ncls - 1]);
    }
    return true;
}

// hash of a prefix as the kernel computes it from the symbol's first bytes (lists.h)
uint64_t rxp_hash(const std::string& p) {
    uint64_t h = 0;
    for (size_t i = 0; i < p.size(); i += 8) {
        uint64_t w = 0;
        memcpy(&w, p.data() + i, std::min<size_t>(8, p.size() - i));
        h = mxp_hash_step(h, w);
    }
    return mxp_hash_final(h, p.size());
}

// strings.ToUpper (Go 1.9; goupper.h): the key a case-insensitive list stores and looks up
std::string go_to_upper(const std::string& s) {
    std::string o;
    o.reserve(s.size() + 8);
    MxpUpperStream st((const uint8_t*)s.data(), (uint32_t)s.size(), kUpperRows);
    uint64_t w;
    uint32_t k;
    while ((k = st.next8(&w)) != 0) o.append((const char*)&w, k);
    return o;
}

uint64_t host_hash(const std::string& s, bool upper) {
    uint64_t h = 0;
    for (size_t i = 0; i < s.size(); i += 8) {
        uint64_t w = 0;
        memcpy(&w, s.data() + i, std::min<size_t>(8, s.size() - i));
        h = mxp_hash_step(h, upper ? mxp_upper8(w) : w);
    }
    return mxp_hash_final(h, s.size());
}

// net.ParseCIDR (Go 1.9 src/net/ip.go) -> IPNet{IP: ip.Mask(m), Mask: m}; false on ParseError
struct Net {
    uint8_t ip[16];
    int iplen;
    uint8_t mask[16];
    int masklen;
};

bool parse_cidr(const std::string& s, Net* out) {
    const size_t slash = s.find('/');
    if (slash == std::string::npos) return false;
    const uint8_t* a = (const uint8_t*)s.data();
    uint8_t ip[16];
    int iplen = 4;
    if (!mxpnet::parse_v4(a, (uint32_t)slash, ip)) {
        iplen = 16;
        if (!mxpnet::parse_v6(a, (uint32_t)slash, ip)) return false;
    }
    int n;
    uint32_t used;
    const uint8_t* m = a + slash + 1;
    const uint32_t ml = (uint32_t)(s.size() - slash - 1);
    if (!mxpnet::dtoi(m, ml, &n, &used) || used != ml || n < 0 || n > 8 * iplen) return false;
    // CIDRMask(n, 8 * iplen)
    uint8_t mask[16] = {0};
    for (int i = 0; i < iplen; i++) {
        const int bits = std::min(8, std::max(0, n - 8 * i));
        mask[i] = (uint8_t)(0xFF00u >> bits);
    }
    // ip.Mask(m): a 4-byte mask on a v4-in-v6 address masks its last 4 bytes
    Net r{};
    r.masklen = iplen;
    memcpy(r.mask, mask, iplen);
    const uint8_t* src = ip;
    int srclen = 16;
    if (iplen == 4 && mxpnet::is_v4(ip)) {
        src = ip + 12;
        srclen = 4;
    }
    if (srclen != iplen) return false;  // not reachable from ParseCIDR
    r.iplen = iplen;
    for (int i = 0; i < iplen; i++) r.ip[i] = src[i] & mask[i];
    *out = r;
    return true;
}

// networkNumberAndMask (ip.go): the family a net matches after IP.To4, or false (never matches)
bool net_number_and_mask(const Net& n, uint8_t nn[16], int* nnlen, uint8_t m[16]) {
    uint8_t ip16[16];
    const uint8_t* ip = n.ip;
    int iplen = n.iplen;
    if (iplen == 16 && mxpnet::is_v4(n.ip)) {  // To4 of a v4-in-v6 network number
        memcpy(ip16, n.ip + 12, 4);
        ip = ip16;
        iplen = 4;
    }
    const uint8_t* mk = n.mask;
    int mlen = n.masklen;
    if (mlen == 4) {
        if (iplen != 4) return false;
    } else if (mlen == 16) {
        if (iplen == 4) {
            mk = n.mask + 12;
            mlen = 4;
        }
    } else {
        return false;
    }
    memcpy(nn, ip, iplen);
    memcpy(m, mk, mlen);
    *nnlen = iplen;
    return true;
}

template <class T>
void merge(std::vector<std::pair<T, T>>& v) {
    std::sort(v.begin(), v.end());
    std::vector<std::pair<T, T>> o;
    for (auto& p : v) {
        if (!o.empty() && (p.first <= o.back().second || (o.back().second != std::numeric_limits<T>::max() &&
                                                          p.first == o.back().second + 1)))
            o.back().second = std::max(o.back().second, p.second);
        else
            o.push_back(p);
    }
    v.swap(o);
}

// IP lists: address families in waves of their own (mxp_list_ip_kernel); MXP_LIST_IP_SPLIT=0: the
// one-lookup-per-lane kernel (A/B)
// MXP_LIST_OPT (lists.h MXP_LIST_OPT_*): the IPv4 register parse and the string register window are
// on; the /16 directory is off (same-box A/B on C3 CIDR, profiles/r5_s3_ab_c3ip_opt.log: 0.0676 ms
// without it, 0.0678 with it)
uint32_t list_opt() {
    const char* e = getenv("MXP_LIST_OPT");
    return e ? (uint32_t)atoi(e) : (MXP_LIST_OPT_V4REG | MXP_LIST_OPT_STRREG);
}

uint32_t ip_split() {
    const char* e = getenv("MXP_LIST_IP_SPLIT");
    return (uint32_t)(e ? atoi(e) != 0 : 1);
}

void set_lds(mxp_list_args& A, const mxp_list* L) {
    A.lds_nparts = L->lds_nparts;
    A.lds_plan = L->lds_plan.as<uint32_t>();
    A.rxp_tab = L->rxp_tab.as<uint64_t>();
    A.rxp_blk = L->rxp_blk.as<uint8_t>();
    A.rxp_lead = L->rxp_lead.as<uint32_t>();
    A.rxp_mask = L->rxp_mask;
    A.rxp_short = L->rxp_short;
}

}  // namespace

extern "C" {

int mxp_list_create(mxp_engine* eng, int entry_type, const char* const* entries, const uint32_t* entry_lens,
                    uint32_t n_entries, const char* const* overrides, const uint32_t* override_lens,
                    uint32_t n_overrides, mxp_list** out) {
    if (!eng || !out || (n_entries && (!entries || !entry_lens)) || (n_overrides && (!overrides || !override_lens)))
        return MXP_ERR_ARG;
    if (eng->device < 0) return eng->fail(MXP_ERR_STATE, "host-only engine");
    std::unique_ptr<mxp_list> L(new mxp_list());
    L->type = entry_type;
    hipError_t e;
    if ((e = hipSetDevice(eng->device)) != hipSuccess) return eng->hipfail(e, "hipSetDevice");
    auto put = [&](DevBuf& d, const void* src, size_t bytes, const char* what) -> int {
        if ((e = d.alloc(bytes ? bytes : 16)) != hipSuccess) return eng->hipfail(e, what);
        if (bytes && (e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice)) != hipSuccess) return eng->hipfail(e, what);
        return MXP_OK;
    };
    int rc;
    auto str = [](const char* p, uint32_t n) { return std::string(p, n); };
    if (entry_type == MXP_LIST_STRINGS || entry_type == MXP_LIST_CASE_INSENSITIVE_STRINGS) {
        const bool upper = entry_type == MXP_LIST_CASE_INSENSITIVE_STRINGS;
        std::unordered_map<std::string, uint32_t> ids;
        std::vector<std::string> uniq;
        auto add = [&](const std::string& s) {
            if (s.empty()) return;  // empty lines / overrides are skipped
            std::string k = upper ? go_to_upper(s) : s;
            if (ids.emplace(k, (uint32_t)uniq.size()).second) uniq.push_back(k);
        };
        for (uint32_t i = 0; i < n_entries; i++) add(str(entries[i], entry_lens[i]));
        for (uint32_t i = 0; i < n_overrides; i++) add(str(overrides[i], override_lens[i]));
        std::vector<uint64_t> desc;
        std::string pool;
        if (!string_pool(uniq, &desc, &pool)) return eng->fail(MXP_ERR_ARG, "list entry longer than 16 MiB");
        if (pool.size() / 8 >= 0xFFFFFFFFull) return eng->fail(MXP_ERR_ARG, "list entries exceed 32 GiB");
        uint32_t cap = 2;
        while (cap < 2 * uniq.size()) cap <<= 1;
        std::vector<uint64_t> tab(cap, MXP_LIST_EMPTY);
        for (uint32_t i = 0; i < uniq.size(); i++) {
            const uint64_t h = host_hash(uniq[i], false);  // entries are already upper-cased
            uint32_t s = (uint32_t)h & (cap - 1);
            while (tab[s] != MXP_LIST_EMPTY) s = (s + 1) & (cap - 1);
            const size_t len = uniq[i].size();
            tab[s] = len < MXP_LIST_LONG ? MXP_LIST_SLOT(h, len, (desc[i] >> 24) / 8) : MXP_LIST_SLOT(h, MXP_LIST_LONG, i);
        }
        L->n_entries = uniq.size();
        L->hmask = cap - 1;
        if ((rc = put(L->htab, tab.data(), tab.size() * 8, "upload list table"))) return rc;
        if ((rc = put(L->ent_desc, desc.data(), desc.size() * 8, "upload list desc"))) return rc;
        if ((rc = put(L->ent_pool, pool.data(), pool.size(), "upload list pool"))) return rc;
    } else if (entry_type == MXP_LIST_IP_ADDRESSES) {
        std::vector<std::pair<uint32_t, uint32_t>> r4;
        std::vector<std::pair<unsigned __int128, unsigned __int128>> r6;
        auto add = [&](const std::string& orig, bool strict) -> int {
            std::string ip = orig;
            if (ip.find('/') == std::string::npos) ip += "/32";
            Net n;
            if (!parse_cidr(ip, &n)) {
                if (!strict) return MXP_OK;  // overrides: errors ignored (config was validated)
                return eng->fail(MXP_ERR_ARG, "could not parse list entry " + orig + ": invalid CIDR address: " + ip);
            }
            L->n_entries++;
            uint8_t nn[16], m[16];
            int len;
            if (!net_number_and_mask(n, nn, &len, m)) return MXP_OK;  // an IPNet that contains nothing
            if (len == 4) {
                uint32_t lo = 0, mm = 0;
                for (int i = 0; i < 4; i++) {
                    lo = lo << 8 | (uint32_t)(nn[i] & m[i]);
                    mm = mm << 8 | m[i];
                }
                r4.emplace_back(lo, lo | ~mm);
            } else {
                unsigned __int128 lo = 0, mm = 0;
                for (int i = 0; i < 16; i++) {
                    lo = lo << 8 | (unsigned __int128)(nn[i] & m[i]);
                    mm = mm << 8 | m[i];
                }
                r6.emplace_back(lo, lo | ~mm);
            }
            return MXP_OK;
        };
        for (uint32_t i = 0; i < n_entries; i++)
            if ((rc = add(str(entries[i], entry_lens[i]), true))) return rc;
        for (uint32_t i = 0; i < n_overrides; i++) add(str(overrides[i], override_lens[i]), false);
        merge(r4);
        merge(r6);
        std::vector<uint32_t> lo4, hi4;
        std::vector<uint64_t> lo6, hi6;
        for (auto& p : r4) {
            lo4.push_back(p.first);
            hi4.push_back(p.second);
        }
        for (auto& p : r6) {
            lo6.push_back((uint64_t)(p.first >> 64));
            lo6.push_back((uint64_t)p.first);
            hi6.push_back((uint64_t)(p.second >> 64));
            hi6.push_back((uint64_t)p.second);
        }
        L->n4 = (uint32_t)r4.size();
        L->n6 = (uint32_t)r6.size();
        // /16 directory of the IPv4 intervals: dir[k] = intervals whose start is below k << 16
        std::vector<uint32_t> dir(65537, 0);
        for (uint32_t k = 0, i = 0; k <= 65536; k++) {
            const uint64_t at = (uint64_t)k << 16;
            while (i < lo4.size() && lo4[i] < at) i++;
            dir[k] = i;
        }
        if ((rc = put(L->v4dir, dir.data(), dir.size() * 4, "upload v4dir"))) return rc;
        if ((rc = put(L->v4lo, lo4.data(), lo4.size() * 4, "upload v4lo"))) return rc;
        if ((rc = put(L->v4hi, hi4.data(), hi4.size() * 4, "upload v4hi"))) return rc;
        if ((rc = put(L->v6lo, lo6.data(), lo6.size() * 8, "upload v6lo"))) return rc;
        if ((rc = put(L->v6hi, hi6.data(), hi6.size() * 8, "upload v6hi"))) return rc;
    } else if (entry_type == MXP_LIST_REGEX) {
        // parseRegexList (regexList.go:44-65): every non-empty line, then every override, must
        // compile (the first failure fails the list with regexp's error); checkList = any matches.
        // The patterns are packed, in order, into parts whose single-pattern DFAs sum to about
        // kListPartStates; each part is one union DFA (a part over kListRegexStates splits in
        // halves), and a pattern whose own DFA is over kPatternStates becomes its own NFA.  Only a
        // pattern with both a DFA over budget and more than kNfaMaxPos (1023) rune instructions is refused.
        std::vector<std::string> pats;
        for (uint32_t i = 0; i < n_entries; i++)
            if (entry_lens[i]) pats.push_back(str(entries[i], entry_lens[i]));
        for (uint32_t i = 0; i < n_overrides; i++) pats.push_back(str(overrides[i], override_lens[i]));
        std::vector<uint64_t> cost(pats.size());
        std::vector<uint8_t> alone(pats.size(), 0);
        // Literal-prefix dispatch (MXP_LIST_RXP=0: off): a pattern anchored on literal bytes
        // (regex_required_prefix) whose DFA after them fits a tail block is indexed by those bytes
        // and leaves the union parts; a lookup probes the prefixes it starts with and walks the
        // candidates' tails in LDS (lists.hip mxp_list_rxp_kernel) -- a few dependent loads per
        // lookup instead of one per byte through a union DFA far larger than the caches.
        // MXP_LIST_RXP=1: always, 0: never; unset: when the patterns would not fit one union part.  A
        // list that fits one part walks one DFA per lookup, faster than the dispatch's probes and tail
        // walks on C3 (10k patterns: 0.092 against 0.125 ms, profiles/r6_s15_ab_rxp_ilp.log -- the
        // dispatch kernel is bound by its VALU issue and vector-memory instructions, not by one walk's
        // latency); past one part every lookup walks every part, and the dispatch stays flat.
        const char* rxp_env = getenv("MXP_LIST_RXP");
        const bool rxp_on = !rxp_env || atoi(rxp_env) != 0;

        std::map<std::string, std::vector<std::vector<uint8_t>>> rxp_keys;  // prefix -> its patterns' tails
        std::vector<uint8_t> dispatched(pats.size(), 0);
        for (size_t i = 0; i < pats.size(); i++) {  // per-pattern errors, in the reference's order
            mxp::Dfa one;
            std::string e;
            const int prc = mxp::regex_compile({pats[i]}, kPatternStates, &one, &e, nullptr, false);
            if (prc == mxp::RX_SYNTAX) return eng->fail(MXP_ERR_ARG, e);
            if (prc == mxp::RX_UNSUPPORTED) return eng->fail(MXP_ERR_ARG, "unsupported regexp (engine): " + e);
            cost[i] = prc == mxp::RX_OK ? one.nstates : kPatternStates;
            alone[i] = prc != mxp::RX_OK;
            std::string pre;
            if (rxp_on && prc == mxp::RX_OK && mxp::regex_required_prefix(pats[i], &pre)) {
                std::vector<uint8_t> blk;
                bool never = false;
                if (rxp_block(one, pre, &blk, &never)) {
                    auto& v = rxp_keys[std::string((const char*)blk.data() + 4, blk[2])];
                    if (v.size() < 63) {  // (a slot counts at most 63 tails)
                        v.push_back(std::move(blk));
                        dispatched[i] = 1;
                    }
                } else if (never) {
                    dispatched[i] = 1;  // no subject starting with its required prefix matches: never matches
                }
            }
        }
        L->n_entries = pats.size();
        if (!rxp_env && !rxp_keys.empty()) {  // (auto: the union's size, from each pattern's own DFA)
            uint64_t sum = 0;
            bool any_alone = false;
            for (size_t i = 0; i < pats.size(); i++) {
                sum += cost[i];
                any_alone |= alone[i] != 0;
            }
            if (!any_alone && sum <= kListPartStates) {  // one union part: no dispatch
                rxp_keys.clear();
                dispatched.assign(pats.size(), 0);
            }
        }
        if (!rxp_keys.empty()) {
            uint32_t cap = 16;
            while (cap < 2 * rxp_keys.size()) cap <<= 1;
            std::vector<uint64_t> tab(cap, 0);
            std::vector<uint8_t> pool;
            std::vector<uint32_t> lead(MXP_RXP_LEAD, 0);
            for (const auto& kv : rxp_keys) {
                const std::string& key = kv.first;
                const uint64_t first = pool.size() / 16;
                for (const auto& b : kv.second) pool.insert(pool.end(), b.begin(), b.end());
                const uint64_t h = rxp_hash(key);
                uint32_t slot = (uint32_t)h & (cap - 1);
                while (tab[slot]) slot = (slot + 1) & (cap - 1);
                tab[slot] = (h >> 44) << 44 | (uint64_t)key.size() << 38 | (uint64_t)kv.second.size() << 32 | first;
                const uint32_t bit = 1u << (key.size() - 1);
                if (key.size() >= 3)
                    lead[mxp_rxp_lead((uint8_t)key[0], (uint8_t)key[1], (uint8_t)key[2])] |= bit;
                else
                    L->rxp_short |= bit;
                L->rxp_n += (uint32_t)kv.second.size();
            }
            pool.resize(pool.size() + MXP_RXP_BLOCK, 0);  // (slack)
            if ((rc = put(L->rxp_tab, tab.data(), tab.size() * 8, "upload rxp table"))) return rc;
            if ((rc = put(L->rxp_blk, pool.data(), pool.size(), "upload rxp blocks"))) return rc;
            if ((rc = put(L->rxp_lead, lead.data(), lead.size() * 4, "upload rxp lead"))) return rc;
            L->rxp_mask = cap - 1;
            L->rxp_keys = (uint32_t)rxp_keys.size();
            // the union parts keep the other patterns
            std::vector<std::string> p2;
            std::vector<uint64_t> c2;
            std::vector<uint8_t> a2;
            for (size_t i = 0; i < pats.size(); i++)
                if (!dispatched[i]) {
                    p2.push_back(std::move(pats[i]));
                    c2.push_back(cost[i]);
                    a2.push_back(alone[i]);
                }
            pats.swap(p2);
            cost.swap(c2);
            alone.swap(a2);
        }
        // u16 parts (MXP_LIST_RX16=1; off by default): union DFAs of at most 65533 states, u16 rows,
        // the patterns sorted first (any match is a match, so the order is free) so that a part's
        // patterns share their leading literals and a lookup leaves the other parts at their first
        // byte; states numbered BFS for the LDS-staged head, depth-first below it, so one lookup's
        // chain of rows lies in adjacent rows.  A host model of the walks halved the cold lines per
        // lookup (8.8 -> 4.7), but the C3 regex kernel went from 0.094 to 0.267 ms per 1M lookups
        // (profiles/r5_s4_ab_c3rx_16.log): the walks are bound by their dependent loads, not by
        // the lines they touch, and four parts walk more steps than one.
        const char* rx16_env = getenv("MXP_LIST_RX16");
        const bool rx16 = rx16_env && atoi(rx16_env) != 0;
        if (rx16) {
            std::vector<size_t> ord(pats.size());
            for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
            std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return pats[a] < pats[b]; });
            std::vector<std::string> p2(pats.size());
            std::vector<uint64_t> c2(pats.size());
            std::vector<uint8_t> a2(pats.size());
            for (size_t i = 0; i < ord.size(); i++) {
                p2[i] = std::move(pats[ord[i]]);
                c2[i] = cost[ord[i]];
                a2[i] = alone[ord[i]];
            }
            pats.swap(p2);
            cost.swap(c2);
            alone.swap(a2);
        }
        const uint32_t union_budget = rx16 ? 65533u : kListRegexStates;
        const uint64_t pack_budget = rx16 ? 56000u : kListPartStates;
        mxp::DfaSetHost set;
        std::vector<uint32_t> part_states;  // DFA states per part (0: an NFA part)
        std::function<int(size_t, size_t)> part = [&](size_t lo, size_t hi) -> int {
            if (lo >= hi) return MXP_OK;
            const std::vector<std::string> ps(pats.begin() + lo, pats.begin() + hi);
            mxp::Dfa d;
            std::string e;
            const bool one = hi - lo == 1;
            const int prc = mxp::regex_compile(ps, one ? kPatternStates : union_budget, &d, &e, nullptr, one);
            if (prc == mxp::RX_OK) {
                if (rx16 && !d.is_nfa() && d.nstates <= 65533u) {
                    mxp::dfa_renumber_hybrid(&d, std::max(1u, 2u * MXP_LDS_DFA_WORDS / d.ncls));
                    set.add16(d);
                } else {
                    set.add(d);
                }
                part_states.push_back(d.is_nfa() ? 0u : d.nstates);
                return MXP_OK;
            }
            if (one) return eng->fail(MXP_ERR_ARG, "regex list: pattern " + pats[lo] + ": " + e);
            const size_t mid = lo + (hi - lo) / 2;
            int rc2 = part(lo, mid);
            return rc2 ? rc2 : part(mid, hi);
        };
        for (size_t i = 0; i < pats.size();) {
            if (alone[i]) {
                if ((rc = part(i, i + 1))) return rc;
                i++;
                continue;
            }
            size_t j = i;
            uint64_t sum = 0;
            while (j < pats.size() && !alone[j] && (j == i || sum + cost[j] <= pack_budget)) sum += cost[j++];
            if ((rc = part(i, j))) return rc;
            i = j;
        }
        if (set.hdr.empty() && !L->rxp_mask) {  // no patterns: an automaton that never matches
            mxp::Dfa d;
            std::string e;
            mxp::regex_compile({}, 16, &d, &e);
            set.add(d);
            part_states.push_back(d.nstates);
        }
        // LDS staging (mxp_list_rx_kernel): the leading parts' first states (BFS order: the levels
        // every lookup steps through) within MXP_LDS_DFA_WORDS; MXP_LIST_LDS=0 turns it off (A/B)
        const char* lds_env = getenv("MXP_LIST_LDS");
        if (!lds_env || atoi(lds_env) != 0) {
            uint32_t plan[2 * MXP_LDS_DFA_PARTS] = {}, used = 0;
            for (size_t k = 0; k < set.hdr.size() && k < MXP_LDS_DFA_PARTS; k++) {
                const uint32_t ncls = set.hdr[k].ncls;
                const bool w16 = set.hdr[k].kind == MXP_RX_DFA16;  // (two u16 entries per LDS word)
                const uint32_t K = std::min(part_states[k], (MXP_LDS_DFA_WORDS - used) * (w16 ? 2u : 1u) / ncls);
                plan[k] = K;
                plan[MXP_LDS_DFA_PARTS + k] = used;
                used += w16 ? (K * ncls + 1u) / 2u : K * ncls;
                L->lds_nparts = (uint32_t)k + 1;
            }
            if ((rc = put(L->lds_plan, plan, sizeof plan, "upload lds plan"))) return rc;
        }
        if (set.nfa_wmax() > MXP_NFA_WIDE_WORDS && L->nfa_scratch.ensure(set.nfa_wmax()))
            return eng->fail(MXP_ERR_NOMEM, "regex list: NFA thread-set scratch");
        L->rx_n = (uint32_t)set.hdr.size();
        for (const auto& h : set.hdr) L->rx_nfa += h.kind == MXP_RX_NFA ? 1u : 0u;
        if (L->rx_n) {  // (every pattern dispatched by its prefix: no union part)
            if ((rc = put(L->rx_hdr, set.hdr.data(), set.hdr.size() * sizeof(mxp_dfa_hdr), "upload rx hdr"))) return rc;
            if ((rc = put(L->rx_trans, set.trans.data(), set.trans.size() * 4, "upload rx trans"))) return rc;
            if ((rc = put(L->rx_ascii, set.ascii.data(), set.ascii.size() * 2, "upload rx ascii"))) return rc;
            if ((rc = put(L->rx_hilo, set.hilo.data(), set.hilo.size() * 4, "upload rx hilo"))) return rc;
            if ((rc = put(L->rx_hicls, set.hicls.data(), set.hicls.size() * 2, "upload rx hicls"))) return rc;
        }
    } else {
        return eng->fail(MXP_ERR_ARG, "unknown list entry type");
    }
    *out = L.release();
    return MXP_OK;
}

void mxp_list_destroy(mxp_engine* eng, mxp_list* list) {
    if (eng && eng->device >= 0) (void)hipSetDevice(eng->device);
    delete list;
}

uint64_t mxp_list_entries(const mxp_list* list) { return list ? list->n_entries : 0; }

int mxp_go_to_upper(const uint8_t* s, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    if ((n && !s) || (cap && !out) || !out_len || n >= (1ull << 32)) return MXP_ERR_ARG;
    const std::string u = go_to_upper(std::string((const char*)s, (size_t)n));
    if (cap) memcpy(out, u.data(), std::min<uint64_t>(cap, u.size()));
    *out_len = u.size();
    return MXP_OK;
}

void mxp_list_regex_parts(const mxp_list* list, uint32_t out[2]) {
    out[0] = list ? list->rx_n : 0;
    out[1] = list ? list->rx_nfa : 0;
}

void mxp_list_regex_dispatch(const mxp_list* list, uint32_t out[2]) {
    out[0] = list ? list->rxp_n : 0;
    out[1] = list ? list->rxp_keys : 0;
}

int mxp_list_check_device(mxp_engine* eng, const mxp_list* L, int blacklist, const uint8_t* d_sym_bytes,
                          const uint64_t* d_sym_offsets, uint32_t n, void* stream, int32_t* d_codes) {
    if (!eng || !L || (n && (!d_sym_bytes || !d_sym_offsets || !d_codes))) return MXP_ERR_ARG;
    if (!n) return MXP_OK;
    mxp_list_args A;
    memset(&A, 0, sizeof A);
    A.type = (uint32_t)L->type;
    A.blacklist = blacklist ? 1u : 0u;
    A.n = n;
    A.hmask = L->hmask;
    A.sym = d_sym_bytes;
    A.sym_off = d_sym_offsets;
    A.htab = L->htab.as<uint64_t>();
    A.ent_desc = L->ent_desc.as<uint64_t>();
    A.ent_pool = L->ent_pool.as<uint8_t>();
    A.v4lo = L->v4lo.as<uint32_t>();
    A.v4hi = L->v4hi.as<uint32_t>();
    A.v6lo = L->v6lo.as<uint64_t>();
    A.v6hi = L->v6hi.as<uint64_t>();
    A.n4 = L->n4;
    A.n6 = L->n6;
    A.rx_n = L->rx_n;
    A.rx_nfa = L->rx_nfa;
    A.ip_split = ip_split();
    A.v4dir = L->v4dir.as<uint32_t>();
    A.opt = list_opt();
    A.rx = mxp_dfa_set{L->rx_hdr.as<mxp_dfa_hdr>(), L->rx_trans.as<uint32_t>(), L->rx_ascii.as<uint16_t>(),
                       L->rx_hilo.as<uint32_t>(), L->rx_hicls.as<uint16_t>()};
    L->nfa_scratch.set(&A.rx);
    A.codes = d_codes;
    set_lds(A, L);
    hipError_t e = mxp_launch_list(&A, stream ? (hipStream_t)stream : eng->stream);
    return e == hipSuccess ? MXP_OK : eng->hipfail(e, "launch list check");
}

int mxp_listentry_check(mxp_engine* eng, const mxp_list* L, int blacklist, const mxp_bag_batch* batch,
                        uint32_t value_rule, int32_t* codes, uint64_t* values) {
    if (!eng || !L || !batch || (batch->n_requests && !codes)) return MXP_ERR_ARG;
    if (!eng->have_rules || value_rule >= eng->rules.size()) return eng->fail(MXP_ERR_ARG, "listentry: no such rule");
    const auto& R = eng->rules[value_rule];
    const bool iface = R.il_ret == mxp::IL_INTERFACE;
    if (R.status == MXP_RULE_OK && R.il_ret != mxp::IL_STRING && !iface)
        return eng->fail(MXP_ERR_ARG, "listentry: the value expression is not of type STRING");
    const uint32_t n = batch->n_requests;
    const uint32_t NR = (uint32_t)eng->rules.size();
    // Eval of every rule (whole programs, result registers); the batch's string pool is uploaded
    // even when no rule compares strings, since the symbols are read from it
    std::unique_ptr<mxp_dbatch> db;
    DevBuf dm, de, dv;
    const bool saved = eng->need_strings;
    eng->need_strings = true;
    int rc = eng->evaluate(batch, dm, de, &dv, db);
    eng->need_strings = saved;
    if (rc) return rc;
    if (!n) return eng->collect_errors(batch, db);
    hipError_t e;
    DevBuf d_codes;
    if ((e = d_codes.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc codes");
    mxp_list_args A;
    memset(&A, 0, sizeof A);
    A.type = (uint32_t)L->type;
    A.blacklist = blacklist ? 1u : 0u;
    A.n = n;
    A.hmask = L->hmask;
    A.htab = L->htab.as<uint64_t>();
    A.ent_desc = L->ent_desc.as<uint64_t>();
    A.ent_pool = L->ent_pool.as<uint8_t>();
    A.v4lo = L->v4lo.as<uint32_t>();
    A.v4hi = L->v4hi.as<uint32_t>();
    A.v6lo = L->v6lo.as<uint64_t>();
    A.v6hi = L->v6hi.as<uint64_t>();
    A.n4 = L->n4;
    A.n6 = L->n6;
    A.rx_n = L->rx_n;
    A.rx_nfa = L->rx_nfa;
    A.ip_split = ip_split();
    A.v4dir = L->v4dir.as<uint32_t>();
    A.opt = list_opt();
    A.rx = mxp_dfa_set{L->rx_hdr.as<mxp_dfa_hdr>(), L->rx_trans.as<uint32_t>(), L->rx_ascii.as<uint16_t>(),
                       L->rx_hilo.as<uint32_t>(), L->rx_hicls.as<uint16_t>()};
    L->nfa_scratch.set(&A.rx);
    A.codes = d_codes.as<int32_t>();
    set_lds(A, L);
    A.vals = dv.as<uint64_t>() + value_rule;
    A.vstride = NR;
    A.viface = iface ? 1u : 0u;
    A.err_word = de.as<uint32_t>() + (size_t)(value_rule / 32) * n;
    A.err_bit = 1u << (value_rule % 32);
    A.n_gstr = eng->gstrs.size();
    A.gstr_off = eng->d_gstr_off.as<uint64_t>();
    A.gstr = eng->d_gstr.as<uint8_t>();
    A.bstr_off = db->bstr_off.as<uint64_t>();
    A.bstr = db->bstr.as<uint8_t>();
    if ((e = mxp_launch_list(&A, eng->stream)) != hipSuccess) return eng->hipfail(e, "launch listentry");
    if ((e = hipMemcpyAsync(codes, d_codes.p, (size_t)n * 4, hipMemcpyDeviceToHost, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "download codes");
    // the Value registers (rule value_rule's column of the [n][NR] result registers), for the
    // status messages' symbol text (mxp_value_text over the last batch)
    if (values && (e = hipMemcpy2DAsync(values, 8, dv.as<uint64_t>() + value_rule, (size_t)NR * 8, 8, n,
                                        hipMemcpyDeviceToHost, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "download values");
    return eng->collect_errors(batch, db);  // synchronises; error texts for mxp_pair_error
}

int mxp_list_check(mxp_engine* eng, const mxp_list* L, int blacklist, const uint8_t* sym_bytes,
                   const uint64_t* sym_offsets, uint32_t n, int32_t* codes) {
    if (!eng || !L || (n && (!sym_bytes || !sym_offsets || !codes))) return MXP_ERR_ARG;
    if (!n) return MXP_OK;
    hipError_t e;
    if ((e = hipSetDevice(eng->device)) != hipSuccess) return eng->hipfail(e, "hipSetDevice");
    const uint64_t bytes = sym_offsets[n];
    DevBuf d_sym, d_off, d_codes;
    if ((e = d_sym.alloc(bytes + 16)) != hipSuccess) return eng->hipfail(e, "alloc symbols");
    if ((e = d_off.alloc(((size_t)n + 1) * 8)) != hipSuccess) return eng->hipfail(e, "alloc offsets");
    if ((e = d_codes.alloc((size_t)n * 4)) != hipSuccess) return eng->hipfail(e, "alloc codes");
    if ((e = hipMemsetAsync(d_sym.p, 0, bytes + 16, eng->stream)) != hipSuccess) return eng->hipfail(e, "memset");
    if (bytes && (e = hipMemcpyAsync(d_sym.p, sym_bytes, bytes, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "upload symbols");
    if ((e = hipMemcpyAsync(d_off.p, sym_offsets, ((size_t)n + 1) * 8, hipMemcpyHostToDevice, eng->stream)) != hipSuccess)
        return eng->hipfail(e, "upload offsets");
    int rc = mxp_list_check_device(eng, L, blacklist, d_sym.as<uint8_t>(), d_off.as<uint64_t>(), n, eng->stream,
                                   d_codes.as<int32_t>());
    if (rc) return rc;
    return eng->download(codes, d_codes.p, (size_t)n * 4, "download codes");  // (synchronises)
}

}  // extern "C"
