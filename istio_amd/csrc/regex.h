// regex.h -- Go regexp (RE2 syntax) compiled to a DFA the GPU steps one rune at a time.
//
// The reference matches with regexp.MatchString (mixer/pkg/il/runtime/externs.go:118-120) and
// regexList.checkList (mixer/adapter/list/regexList.go:26-33): compile with syntax.Perl flags, then
// an unanchored search whose only output is "some match exists".  That boolean is a regular-language
// membership test, so the engine compiles it ahead of time:
//
//   parse     Go 1.9 regexp/syntax parse.go semantics (same grammar, flags, error codes and texts
//             as the oracle restatement oracle/goregex.py);
//   NFA       Thompson program over rune ranges with empty-width assertions;
//   DFA       subset construction over rune classes (the partition of all runes by every range
//             boundary, '\n' and the ASCII word characters) plus an END symbol; a DFA state is an
//             unclosed NFA thread set plus the context the assertions need (at text begin,
//             previous rune '\n', previous rune a word character), the way RE2's DFA carries flags.
//             The start thread is re-injected at every position (unanchored search), and a step
//             whose closure reaches MATCH goes to the absorbing ACCEPT state.
//
// Unicode classes (\p / \P) and simple case folding come from Go 1.9's Unicode 9.0 tables
// (unicode_tables.h); a DFA beyond the state budget becomes a bit-parallel NFA (dfa_dev.h); only a
// program wider than kNfaMaxPos rune instructions whose DFA is also over budget is refused.
#pragma once

#include <cstdint>
#include <string>
#include <vector>
#include <cstring>
#include <algorithm>

namespace mxp {

constexpr uint32_t kDfaAccept = 0xFFFFFFFFu;
constexpr uint32_t kDfaReject = 0xFFFFFFFEu;

struct Dfa {
    // alphabet: class of each ASCII rune, then non-ASCII class ranges [lo_k, lo_{k+1})
    uint16_t ascii[128] = {};
    std::vector<uint32_t> hi_lo;   // ascending range starts (first is 0x80)
    std::vector<uint16_t> hi_cls;  // class of each range
    uint32_t ncls = 0;             // rune classes + 1 (the last column is END of text)
    uint32_t nstates = 0;
    uint32_t start = 0;
    std::vector<uint32_t> trans;   // [nstates][ncls]: next state, kDfaAccept or kDfaReject
    // A pattern whose DFA exceeds the state budget but whose program has < kNfaMaxPos rune
    // instructions compiles to a bit-parallel NFA instead (trans empty, nfa = the MXP_NFA_* image of
    // dfa_dev.h): the same alphabet, the thread set as a bitset over rune instructions.
    std::vector<uint64_t> nfa;
    bool is_nfa() const { return !nfa.empty(); }
};

constexpr uint32_t kNfaMaxPos = 1023;  // rune instructions walked with private-memory thread sets (MXP_NFA_WIDE_WORDS words)
// wider programs walk with thread sets in global memory (dfa_dev.h mxp_nfa_run_global), up to the
// header's 8-bit word count (255 words: 16319 rune instructions) and 1 GiB of closure tables
constexpr uint32_t kNfaHugePos = 255u * 64u - 1u;
constexpr uint64_t kNfaMaxBytes = 1ull << 30;

enum RegexStatus { RX_OK = 0, RX_SYNTAX = 1, RX_UNSUPPORTED = 2, RX_TOO_BIG = 3 };

// Compile the union of `patterns` (a match of any of them is a match) into `out`.  On RX_SYNTAX,
// *err is Go's error text ("error parsing regexp: <code>: `<expr>`") of the first failing pattern
// and *bad its index; on RX_UNSUPPORTED / RX_TOO_BIG *err says why.  A DFA over `max_states`
// falls back to the bit-parallel NFA when `nfa_fallback` and the program is small enough.
int regex_compile(const std::vector<std::string>& patterns, uint32_t max_states, Dfa* out, std::string* err,
                  uint32_t* bad = nullptr, bool nfa_fallback = true);

// A pattern anchored at text begin (^ without (?m), or \A) followed by literal runes only matches
// subjects that start with those runes' UTF-8 bytes: the engine indexes such rules by that prefix.
bool regex_required_prefix(const std::string& pattern, std::string* prefix);

// The language a DFA accepts from state `st` as a few literal keys, when it is that simple: every
// path from `st` reaches a decision within `max_depth` ASCII bytes (no non-ASCII class leads anywhere
// but REJECT), giving `prefix` keys (a folded ACCEPT transition: any continuation matches) and
// `exact` keys (a state whose END transition accepts: the subject ends there).  A subject read from
// `st` is accepted iff it starts with a prefix key or equals an exact key, and at most one key fits
// any subject.  False when there are more than `max_keys` keys or a path is undecided at max_depth.
struct LiteralKey {
    std::string bytes;
    bool exact;         // the subject must end here
    bool tail = false;  // the subject's remaining bytes must hold no '\n' (a `.*$` tail)
};
bool dfa_literal_keys(const Dfa& d, uint32_t st, uint32_t max_keys, uint32_t max_depth, std::vector<LiteralKey>* out);

// Host stepping of a compiled DFA or NFA (constant folding, tests).
bool dfa_match_host(const Dfa& d, const std::string& s);
// Renumber a DFA's states: the first `bfs_head` in BFS order from the start (the levels every
// subject steps through; what LDS staging copies), the rest in depth-first preorder, so the chain of
// rows one subject walks below the head lies mostly in adjacent rows.
void dfa_renumber_hybrid(Dfa* d, uint32_t bfs_head);
// transitions into decided states -> kDfaReject (ACCEPT unreachable) / kDfaAccept (every continuation
// accepts); run by the DFA builder
void fold_dead_states(Dfa* d);

}  // namespace mxp

#include "dfa_dev.h"

namespace mxp {

// Host image of a set of DFAs in the device layout of dfa_dev.h (upload each vector as is).
struct DfaSetHost {
    std::vector<mxp_dfa_hdr> hdr;
    std::vector<uint32_t> trans;
    std::vector<uint16_t> ascii;
    std::vector<uint32_t> hilo;
    std::vector<uint16_t> hicls;
    uint32_t add(const Dfa& d);  // -> DFA index
    uint32_t add16(const Dfa& d);  // a DFA of <= 65533 states with u16 transitions (MXP_RX_DFA16)
    bool has_nfa() const {
        for (const auto& h : hdr)
            if (h.kind == MXP_RX_NFA) return true;
        return false;
    }
    // the widest NFA's thread-set words (0 without NFAs)
    uint32_t nfa_wmax() const {
        uint32_t w = 0;
        for (const auto& h : hdr)
            if (h.kind == MXP_RX_NFA) {
                uint64_t h0;
                memcpy(&h0, trans.data() + h.trans, 8);
                w = std::max(w, (uint32_t)(h0 >> 16) & 0xFFu);
            }
        return w;
    }
};

}  // namespace mxp
