// regex.cpp -- see regex.h.  Parser follows Go 1.9 src/regexp/syntax/parse.go (Perl flags).
#include "regex.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>

#include "unicode_tables.h"

namespace mxp {
namespace {

constexpr uint32_t kMaxRune = 0x10FFFF;
constexpr int kMaxRepeat = 1000;
constexpr uint32_t kMaxInsts = 200000;

// empty-width assertions (syntax.EmptyOp)
enum : uint8_t { BEGIN_LINE = 1, END_LINE = 2, BEGIN_TEXT = 4, END_TEXT = 8, WORD_B = 16, NO_WORD_B = 32 };

using Ranges = std::vector<std::pair<uint32_t, uint32_t>>;

struct SyntaxError {
    std::string code, expr;
};
struct UnsupportedError {
    std::string why;
};

// utf8.DecodeRune: (rune, width); invalid -> (0xFFFD, 1)
uint32_t decode_rune(const std::string& b, size_t i, size_t* w) {
    const uint8_t c = (uint8_t)b[i];
    const size_t n = b.size() - i;
    auto at = [&](size_t k) { return (uint8_t)b[i + k]; };
    *w = 1;
    if (c < 0x80) return c;
    if (c >= 0xC2 && c <= 0xDF && n >= 2 && at(1) >= 0x80 && at(1) <= 0xBF) {
        *w = 2;
        return ((c & 0x1Fu) << 6) | (at(1) & 0x3Fu);
    }
    if (c >= 0xE0 && c <= 0xEF && n >= 3) {
        uint8_t lo = 0x80, hi = 0xBF;
        if (c == 0xE0) lo = 0xA0;
        if (c == 0xED) hi = 0x9F;
        if (at(1) >= lo && at(1) <= hi && at(2) >= 0x80 && at(2) <= 0xBF) {
            *w = 3;
            return ((c & 0x0Fu) << 12) | ((at(1) & 0x3Fu) << 6) | (at(2) & 0x3Fu);
        }
    }
    if (c >= 0xF0 && c <= 0xF4 && n >= 4) {
        uint8_t lo = 0x80, hi = 0xBF;
        if (c == 0xF0) lo = 0x90;
        if (c == 0xF4) hi = 0x8F;
        if (at(1) >= lo && at(1) <= hi && at(2) >= 0x80 && at(2) <= 0xBF && at(3) >= 0x80 && at(3) <= 0xBF) {
            *w = 4;
            return ((c & 0x07u) << 18) | ((at(1) & 0x3Fu) << 12) | ((at(2) & 0x3Fu) << 6) | (at(3) & 0x3Fu);
        }
    }
    return 0xFFFD;
}

bool is_word(int64_t r) {
    return r >= 0 && ((r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_');
}

bool is_alnum(uint32_t c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

int unhex(uint32_t c) {
    if (c >= '0' && c <= '9') return (int)(c - '0');
    if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
    if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
    return -1;
}

Ranges norm(Ranges rs) {
    std::sort(rs.begin(), rs.end());
    Ranges o;
    for (auto& p : rs) {
        if (p.first > p.second) continue;
        if (!o.empty() && p.first <= o.back().second + 1)
            o.back().second = std::max(o.back().second, p.second);
        else
            o.push_back(p);
    }
    return o;
}

Ranges negate(const Ranges& in) {
    Ranges o;
    uint32_t nxt = 0;
    for (auto& p : norm(in)) {
        if (p.first > nxt) o.emplace_back(nxt, p.first - 1);
        nxt = p.second + 1;
    }
    if (nxt <= kMaxRune) o.emplace_back(nxt, kMaxRune);
    return o;
}

// unicode.SimpleFold over kUniFold: the next rune of r's orbit (r itself when r does not fold)
uint32_t simple_fold(uint32_t r) {
    size_t a = 0, b = sizeof kUniFold / sizeof kUniFold[0];
    while (a < b) {
        const size_t m = (a + b) / 2;
        if (kUniFold[m][0] < r) a = m + 1;
        else b = m;
    }
    return a < sizeof kUniFold / sizeof kUniFold[0] && kUniFold[a][0] == r ? kUniFold[a][1] : r;
}

bool contains(const Ranges& rs, uint32_t r) {  // rs normalised
    auto it = std::upper_bound(rs.begin(), rs.end(), std::make_pair(r, kMaxRune + 1));
    return it != rs.begin() && (it - 1)->second >= r;
}

// appendFoldedRange over every range: the class closed under simple case folding (each member's
// whole orbit joins)
Ranges fold_ranges(const Ranges& in) {
    const Ranges rs = norm(in);
    Ranges o = rs;
    for (const auto& f : kUniFold)
        if (contains(rs, f[0]))
            for (uint32_t x = f[1]; x != f[0]; x = simple_fold(x)) o.emplace_back(x, x);
    return norm(o);
}

// unicodeTable (parse.go): "Any", unicode.Categories, unicode.Scripts; false when unknown
bool unicode_table(const std::string& name, Ranges* out) {
    if (name == "Any") {
        *out = {{0, kMaxRune}};
        return true;
    }
    const uni_class* b = kUniClasses;
    const uni_class* e = kUniClasses + sizeof kUniClasses / sizeof kUniClasses[0];
    const uni_class* it = std::lower_bound(b, e, name, [](const uni_class& c, const std::string& n) { return n.compare(c.name) > 0; });
    if (it == e || name != it->name) return false;
    out->clear();
    for (uint32_t k = 0; k < it->n; k++) out->emplace_back(kUniRanges[it->off + k][0], kUniRanges[it->off + k][1]);
    return true;
}

bool valid_utf8(const std::string& s, size_t a, size_t b) {  // checkUTF8 over s[a, b)
    const std::string t = s.substr(a, b - a);
    for (size_t i = 0; i < t.size();) {
        size_t w;
        const uint32_t r = decode_rune(t, i, &w);
        if (r == 0xFFFD && w == 1 && t.compare(i, 3, "\xEF\xBF\xBD") != 0) return false;
        i += w;
    }
    return true;
}

// ---------------------------------------------------------------------------------- AST
enum NodeKind { N_LIT, N_CLASS, N_ANY, N_ANYNL, N_EMPTY, N_CAT, N_ALT, N_STAR, N_PLUS, N_QUEST, N_REP, N_GROUP };

struct Node {
    NodeKind k;
    uint32_t rune = 0;
    Ranges cls;
    uint8_t empty = 0;
    int lo = 0, hi = 0;
    std::vector<std::unique_ptr<Node>> sub;
};
using NodeP = std::unique_ptr<Node>;

NodeP mk(NodeKind k) {
    NodeP n(new Node());
    n->k = k;
    return n;
}

struct Flags {
    bool i = false, m = false, s = false, U = false;
};

class Parser {
  public:
    explicit Parser(const std::string& src) : s_(src) {}

    NodeP parse() { return alt(true); }

  private:
    const std::string& s_;
    size_t i_ = 0;
    Flags f_;

    [[noreturn]] void err(const char* code, const std::string& expr) { throw SyntaxError{code, expr}; }
    std::string text(size_t a, size_t b = std::string::npos) const {
        return s_.substr(a, b == std::string::npos ? std::string::npos : b - a);
    }
    bool at(size_t k, char c) const { return k < s_.size() && s_[k] == c; }

    // nextRune: invalid UTF-8 -> ErrInvalidUTF8 with the rest of the text
    uint32_t next_rune() {
        size_t w;
        const uint32_t r = decode_rune(s_, i_, &w);
        if (r == 0xFFFD && w == 1 && s_.compare(i_, 3, "\xEF\xBF\xBD") != 0) err("invalid UTF-8", text(i_));
        i_ += w;
        return r;
    }

    NodeP lit(uint32_t r) {
        if (f_.i && simple_fold(r) != r) {
            Ranges orbit{{r, r}};
            for (uint32_t x = simple_fold(r); x != r; x = simple_fold(x)) orbit.emplace_back(x, x);
            NodeP n = mk(N_CLASS);
            n->cls = norm(orbit);
            return n;
        }
        NodeP n = mk(N_LIT);
        n->rune = r;
        return n;
    }

    NodeP cls_node(Ranges rs) {
        NodeP n = mk(N_CLASS);
        n->cls = norm(std::move(rs));
        return n;
    }

    // appendGroup: under (?i) a group is folded BEFORE it is negated
    Ranges group(const Ranges& rs, bool negated) const {
        const Ranges g = f_.i ? fold_ranges(rs) : norm(rs);
        return negated ? negate(g) : g;
    }

    NodeP alt(bool top) {
        std::vector<std::vector<NodeP>> alts(1);
        const Flags saved = f_;
        while (i_ < s_.size()) {
            const char c = s_[i_];
            if (c == '|') {
                i_++;
                alts.emplace_back();
                continue;
            }
            if (c == ')') {
                if (top) err("unexpected )", s_);
                break;
            }
            piece(alts.back());
        }
        if (!top) {
            if (i_ >= s_.size()) err("missing closing )", s_);
            i_++;
            f_ = saved;
        }
        std::vector<NodeP> cats;
        for (auto& a : alts) {
            NodeP c = mk(N_CAT);
            c->sub = std::move(a);
            cats.push_back(std::move(c));
        }
        if (cats.size() == 1) return std::move(cats[0]);
        NodeP n = mk(N_ALT);
        n->sub = std::move(cats);
        return n;
    }

    // parseRepeat at i_ ('{'): {n} {n,} {n,m} -> advance; false = literal '{'
    bool try_repeat(int* lo, int* hi) {
        size_t j = i_ + 1;
        auto num = [&](int* v) -> bool {
            const size_t k0 = j;
            while (j < s_.size() && s_[j] >= '0' && s_[j] <= '9') j++;
            if (j == k0) return false;
            if (j - k0 > 1 && s_[k0] == '0') return false;  // leading zeros
            long x = 0;
            for (size_t k = k0; k < j; k++) {
                x = x * 10 + (s_[k] - '0');
                if (x > kMaxRepeat) x = kMaxRepeat + 1;
            }
            *v = (int)x;
            return true;
        };
        if (!num(lo)) return false;
        if (at(j, ',')) {
            j++;
            if (at(j, '}')) {
                *hi = -1;
            } else if (!num(hi)) {
                return false;
            }
        } else {
            *hi = *lo;
        }
        if (!at(j, '}')) return false;
        j++;
        const size_t start = i_;
        i_ = j;
        if (*lo > kMaxRepeat || *hi > kMaxRepeat || (*hi >= 0 && *lo > *hi)) err("invalid repeat count", text(start, j));
        return true;
    }

    void repeat(std::vector<NodeP>& seq, char op, size_t start, int lo = 0, int hi = 0) {
        if (seq.empty()) err("missing argument to repetition operator", text(start, i_));
        if (at(i_, '?')) i_++;  // lazy form; irrelevant for a boolean match
        if (i_ < s_.size() && (s_[i_] == '*' || s_[i_] == '+' || s_[i_] == '?'))
            err("invalid nested repetition operator", text(start, i_ + 1));
        if (at(i_, '{')) {
            const size_t save = i_;
            int a, b;
            if (try_repeat(&a, &b)) err("invalid nested repetition operator", text(start, i_));
            i_ = save;
        }
        NodeP sub = std::move(seq.back());
        seq.pop_back();
        NodeP n = mk(op == '*' ? N_STAR : op == '+' ? N_PLUS : op == '?' ? N_QUEST : N_REP);
        n->lo = lo;
        n->hi = hi;
        n->sub.push_back(std::move(sub));
        seq.push_back(std::move(n));
    }

    void piece(std::vector<NodeP>& seq) {
        const size_t start = i_;
        const char c = s_[i_];
        switch (c) {
        case '*': case '+': case '?':
            i_++;
            repeat(seq, c, start);
            return;
        case '{': {
            int lo, hi;
            if (try_repeat(&lo, &hi)) {
                repeat(seq, '{', start, lo, hi);
                return;
            }
            i_++;
            seq.push_back(lit('{'));
            return;
        }
        case '(':
            group(seq);
            return;
        case '[':
            seq.push_back(cls_node(parse_class()));
            return;
        case '.':
            i_++;
            seq.push_back(mk(f_.s ? N_ANY : N_ANYNL));
            return;
        case '^': {
            i_++;
            NodeP n = mk(N_EMPTY);
            n->empty = f_.m ? BEGIN_LINE : BEGIN_TEXT;
            seq.push_back(std::move(n));
            return;
        }
        case '$': {
            i_++;
            NodeP n = mk(N_EMPTY);
            n->empty = f_.m ? END_LINE : END_TEXT;
            seq.push_back(std::move(n));
            return;
        }
        case '\\':
            escape_atom(seq);
            return;
        default:
            seq.push_back(lit(next_rune()));
        }
    }

    void group(std::vector<NodeP>& seq) {
        const size_t start = i_;
        if (at(i_ + 1, '?')) {
            if (s_.size() > i_ + 4 && s_[i_ + 2] == 'P' && s_[i_ + 3] == '<') {
                const size_t end = s_.find('>', i_ + 4);
                if (end == std::string::npos) err("invalid named capture", text(start));
                bool ok = end > i_ + 4;
                for (size_t k = i_ + 4; k < end; k++) ok = ok && is_word((uint8_t)s_[k]);
                if (!ok) err("invalid named capture", text(start, end + 1));
                i_ = end + 1;
                NodeP g = mk(N_GROUP);
                g->sub.push_back(alt(false));
                seq.push_back(std::move(g));
                return;
            }
            size_t j = i_ + 2;
            bool sign = true, neg = false, seen = false;
            Flags nf = f_;
            while (true) {
                if (j >= s_.size()) err("invalid or unsupported Perl syntax", text(start));
                const char c = s_[j++];
                if (c == 'i' || c == 'm' || c == 's' || c == 'U') {
                    (c == 'i' ? nf.i : c == 'm' ? nf.m : c == 's' ? nf.s : nf.U) = sign;
                    seen = true;
                } else if (c == '-') {
                    if (neg) err("invalid or unsupported Perl syntax", text(start, j));
                    neg = true;
                    sign = false;
                    seen = false;
                } else if (c == ':' || c == ')') {
                    if (neg && !seen) err("invalid or unsupported Perl syntax", text(start, j));
                    i_ = j;
                    if (c == ')') {
                        f_ = nf;  // rest of the current group
                        return;
                    }
                    const Flags outer = f_;
                    f_ = nf;
                    NodeP g = mk(N_GROUP);
                    g->sub.push_back(alt(false));
                    f_ = outer;
                    seq.push_back(std::move(g));
                    return;
                } else {
                    // the offending rune (possibly multi-byte) is part of the error text
                    size_t w;
                    decode_rune(s_, j - 1, &w);
                    err("invalid or unsupported Perl syntax", text(start, j - 1 + w));
                }
            }
        }
        i_++;
        NodeP g = mk(N_GROUP);
        g->sub.push_back(alt(false));
        seq.push_back(std::move(g));
    }

    // parsePerlClassEscape (\d \s \w and negations) or parseUnicodeClass (\p \P) at i_ -> the group
    bool perl_class(Ranges* out) {
        if (!at(i_, '\\') || i_ + 1 >= s_.size()) return false;
        const char c = s_[i_ + 1];
        if (c == 'p' || c == 'P') {
            *out = unicode_class();
            return true;
        }
        Ranges r;
        switch (c) {
        case 'd': case 'D': r = {{'0', '9'}}; break;
        case 's': case 'S': r = {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}; break;
        case 'w': case 'W': r = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}; break;
        default: return false;
        }
        i_ += 2;
        *out = group(r, c >= 'A' && c <= 'Z');
        return true;
    }

    // parseUnicodeClass: \pN \p{Name} \P.. \p{^Name}; an unknown name is an invalid class range
    Ranges unicode_class() {
        const size_t start = i_;
        bool neg = s_[i_ + 1] == 'P';
        i_ += 2;
        std::string name;
        size_t seq_end;
        if (at(i_, '{')) {
            const size_t end = s_.find('}', i_);
            if (end == std::string::npos) {
                if (!valid_utf8(s_, start, s_.size())) err("invalid UTF-8", text(start));
                err("invalid character class range", text(start));
            }
            if (!valid_utf8(s_, i_ + 1, end)) err("invalid UTF-8", text(i_ + 1, end));
            name = text(i_ + 1, end);
            seq_end = end + 1;
        } else if (i_ < s_.size()) {
            const size_t save = i_;
            next_rune();
            name = text(save, i_);
            seq_end = i_;
        } else {
            seq_end = i_;
        }
        i_ = seq_end;
        if (!name.empty() && name[0] == '^') {
            neg = !neg;
            name.erase(0, 1);
        }
        Ranges tab;
        if (name.empty() || !unicode_table(name, &tab)) err("invalid character class range", text(start, seq_end));
        return group(tab, neg);
    }

    // parseEscape: one escaped rune; errors carry the text consumed so far
    uint32_t escape() {
        const size_t start = i_;
        i_++;
        if (i_ >= s_.size()) err("trailing backslash at end of expression", "");
        const uint32_t c = next_rune();
        auto fail = [&]() { err("invalid escape sequence", text(start, i_)); };
        if (c < 0x80 && !is_alnum(c)) return c;
        if (c >= '1' && c <= '7' && !(i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '7')) fail();
        if (c >= '0' && c <= '7') {
            uint32_t r = c - '0';
            for (int k = 1; k < 3 && i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '7'; k++) r = r * 8 + (s_[i_++] - '0');
            return r;
        }
        if (c == 'x') {
            if (i_ >= s_.size()) fail();
            const uint32_t c2 = next_rune();
            if (c2 == '{') {
                int nhex = 0;
                uint32_t r = 0;
                while (true) {
                    if (i_ >= s_.size()) fail();
                    const uint32_t d = next_rune();
                    if (d == '}') break;
                    const int v = unhex(d);
                    if (v < 0) fail();
                    r = r * 16 + (uint32_t)v;
                    if (r > kMaxRune) fail();
                    nhex++;
                }
                if (!nhex) fail();
                return r;
            }
            const int x = unhex(c2);
            const uint32_t c3 = i_ < s_.size() ? next_rune() : 0xFFFD;
            const int y = unhex(c3);
            if (x < 0 || y < 0) fail();
            return (uint32_t)(x * 16 + y);
        }
        switch (c) {
        case 'a': return 7;
        case 'f': return 12;
        case 'n': return 10;
        case 'r': return 13;
        case 't': return 9;
        case 'v': return 11;
        default: fail();
        }
        return 0;
    }

    void escape_atom(std::vector<NodeP>& seq) {
        if (i_ + 1 < s_.size()) {
            const char c = s_[i_ + 1];
            uint8_t e = c == 'A' ? BEGIN_TEXT : c == 'z' ? END_TEXT : c == 'b' ? WORD_B : c == 'B' ? NO_WORD_B : 0;
            if (e) {
                i_ += 2;
                NodeP n = mk(N_EMPTY);
                n->empty = e;
                seq.push_back(std::move(n));
                return;
            }
            if (c == 'C') err("invalid escape sequence", "\\C");
            if (c == 'Q') {
                i_ += 2;
                const size_t end = s_.find("\\E", i_);
                const size_t stop = end == std::string::npos ? s_.size() : end;
                while (i_ < stop) seq.push_back(lit(next_rune()));
                i_ = end == std::string::npos ? s_.size() : end + 2;
                return;
            }
        }
        Ranges r;
        if (perl_class(&r)) {
            seq.push_back(cls_node(r));
            return;
        }
        seq.push_back(lit(escape()));
    }

    uint32_t class_char(size_t class_start) {
        if (i_ >= s_.size()) err("missing closing ]", text(class_start));
        if (s_[i_] == '\\') return escape();
        return next_rune();
    }

    Ranges parse_class() {
        static const std::map<std::string, Ranges> posix = {
            {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
            {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
            {"ascii", {{0, 0x7F}}},
            {"blank", {{'\t', '\t'}, {' ', ' '}}},
            {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
            {"digit", {{'0', '9'}}},
            {"graph", {{'!', '~'}}},
            {"lower", {{'a', 'z'}}},
            {"print", {{' ', '~'}}},
            {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
            {"space", {{'\t', '\r'}, {' ', ' '}}},
            {"upper", {{'A', 'Z'}}},
            {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
            {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}}};
        const size_t start = i_;
        i_++;
        bool neg = false;
        if (at(i_, '^')) {
            neg = true;
            i_++;
        }
        Ranges rs;
        bool first = true;
        while (true) {
            if (i_ >= s_.size()) err("missing closing ]", text(start));
            if (s_[i_] == ']' && !first) {
                i_++;
                break;
            }
            if (s_[i_] == '[' && at(i_ + 1, ':')) {
                const size_t end = s_.find(":]", i_ + 2);
                if (end != std::string::npos) {
                    std::string name = s_.substr(i_ + 2, end - i_ - 2);
                    const bool pneg = !name.empty() && name[0] == '^';
                    if (pneg) name = name.substr(1);
                    auto it = posix.find(name);
                    if (it == posix.end()) err("invalid character class range", text(i_, end + 2));
                    const Ranges g = group(it->second, pneg);
                    rs.insert(rs.end(), g.begin(), g.end());
                    i_ = end + 2;
                    first = false;
                    continue;
                }
            }
            Ranges pc;
            if (perl_class(&pc)) {
                rs.insert(rs.end(), pc.begin(), pc.end());
                first = false;
                continue;
            }
            const size_t rstart = i_;
            const uint32_t lo = class_char(start);
            if (i_ + 1 < s_.size() && s_[i_] == '-' && s_[i_ + 1] != ']') {
                i_++;
                const uint32_t hi = class_char(start);
                if (hi < lo) err("invalid character class range", text(rstart, i_));
                rs.emplace_back(lo, hi);
            } else {
                rs.emplace_back(lo, lo);
            }
            first = false;
        }
        if (f_.i) rs = fold_ranges(rs);
        rs = norm(rs);
        return neg ? negate(rs) : rs;
    }
};

// ---------------------------------------------------------------------------------- NFA
enum InstOp : uint8_t { I_RUNE, I_SPLIT, I_EMPTY, I_MATCH };
struct Inst {
    InstOp op;
    uint8_t empty = 0;
    int32_t x = -1, y = -1;  // next (RUNE/EMPTY) or the two branches (SPLIT)
    Ranges r;
};

struct Prog {
    std::vector<Inst> ins;
    int emit(Inst i) {
        if (ins.size() >= kMaxInsts) throw UnsupportedError{"regular expression too large for the DFA compiler"};
        ins.push_back(std::move(i));
        return (int)ins.size() - 1;
    }
    int rune(Ranges r, int nxt) {
        Inst i{I_RUNE};
        i.r = std::move(r);
        i.x = nxt;
        return emit(std::move(i));
    }
    int split(int a, int b) {
        Inst i{I_SPLIT};
        i.x = a;
        i.y = b;
        return emit(std::move(i));
    }

    int compile(const Node& n, int nxt) {
        switch (n.k) {
        case N_LIT: return rune({{n.rune, n.rune}}, nxt);
        case N_CLASS: return rune(n.cls, nxt);
        case N_ANY: return rune({{0, kMaxRune}}, nxt);
        case N_ANYNL: return rune({{0, 9}, {11, kMaxRune}}, nxt);
        case N_EMPTY: {
            Inst i{I_EMPTY};
            i.empty = n.empty;
            i.x = nxt;
            return emit(std::move(i));
        }
        case N_GROUP: return compile(*n.sub[0], nxt);
        case N_CAT: {
            int pc = nxt;
            for (size_t k = n.sub.size(); k-- > 0;) pc = compile(*n.sub[k], pc);
            return pc;
        }
        case N_ALT: {
            std::vector<int> e;
            for (auto& s : n.sub) e.push_back(compile(*s, nxt));
            int pc = e.back();
            for (size_t k = e.size() - 1; k-- > 0;) pc = split(e[k], pc);
            return pc;
        }
        case N_QUEST: return split(compile(*n.sub[0], nxt), nxt);
        case N_STAR: {
            const int loop = split(-1, nxt);
            ins[loop].x = compile(*n.sub[0], loop);
            return loop;
        }
        case N_PLUS: {
            const int loop = split(-1, nxt);
            const int body = compile(*n.sub[0], loop);
            ins[loop].x = body;
            return body;
        }
        case N_REP: {
            int pc = nxt;
            if (n.hi < 0) {
                const int loop = split(-1, pc);
                ins[loop].x = compile(*n.sub[0], loop);
                pc = loop;
            } else {
                for (int k = 0; k < n.hi - n.lo; k++) pc = split(compile(*n.sub[0], pc), pc);
            }
            for (int k = 0; k < n.lo; k++) pc = compile(*n.sub[0], pc);
            return pc;
        }
        }
        return nxt;
    }
};

// ---------------------------------------------------------------------------------- DFA
struct StateKey {
    std::vector<int32_t> pcs;  // sorted unclosed thread set
    uint8_t ctx;               // bit0 at text begin, bit1 previous '\n', bit2 previous word rune
    bool operator==(const StateKey& o) const { return ctx == o.ctx && pcs == o.pcs; }
};
struct StateHash {
    size_t operator()(const StateKey& k) const {
        uint64_t h = k.ctx * 0x9E3779B97F4A7C15ull;
        for (int32_t p : k.pcs) h = (h ^ (uint64_t)p) * 0xBF58476D1CE4E5B9ull;
        return (size_t)(h ^ (h >> 31));
    }
};

}  // namespace

namespace {
void append_utf8(std::string* o, uint32_t r) {
    if (r < 0x80) {
        o->push_back((char)r);
    } else if (r < 0x800) {
        o->push_back((char)(0xC0 | (r >> 6)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    } else if (r < 0x10000) {
        o->push_back((char)(0xE0 | (r >> 12)));
        o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    } else {
        o->push_back((char)(0xF0 | (r >> 18)));
        o->push_back((char)(0x80 | ((r >> 12) & 0x3F)));
        o->push_back((char)(0x80 | ((r >> 6) & 0x3F)));
        o->push_back((char)(0x80 | (r & 0x3F)));
    }
}

// the concatenation that starts the pattern (descending through single-alternative groups)
const Node* leading_cat(const Node* n) {
    while (n->k == N_GROUP) n = n->sub[0].get();
    return n->k == N_CAT ? n : nullptr;
}
}  // namespace

bool regex_required_prefix(const std::string& pattern, std::string* prefix) {
    prefix->clear();
    try {
        Parser ps(pattern);
        NodeP ast = ps.parse();
        const Node* cat = leading_cat(ast.get());
        if (!cat || cat->sub.empty()) return false;
        const Node* first = cat->sub[0].get();
        if (first->k != N_EMPTY || first->empty != BEGIN_TEXT) return false;
        // literal runes right after \A / ^ (no (?m)): every match starts with their UTF-8 bytes.
        // (an invalid-UTF-8 subject byte decodes to U+FFFD, so a U+FFFD literal is not a byte prefix)
        for (size_t k = 1; k < cat->sub.size(); k++) {
            const Node* n = cat->sub[k].get();
            while (n->k == N_GROUP && n->sub[0]->k == N_CAT && n->sub[0]->sub.size() == 1) n = n->sub[0]->sub[0].get();
            if (n->k != N_LIT || n->rune == 0xFFFD) break;
            append_utf8(prefix, n->rune);
        }
        return !prefix->empty();
    } catch (...) {
        return false;
    }
}

int regex_compile(const std::vector<std::string>& patterns, uint32_t max_states, Dfa* out, std::string* err,
                  uint32_t* bad, bool nfa_fallback) {
    Prog p;
    std::vector<int> starts;
    const int match = p.emit(Inst{I_MATCH});
    try {
        for (size_t k = 0; k < patterns.size(); k++) {
            if (bad) *bad = (uint32_t)k;
            Parser ps(patterns[k]);
            NodeP ast = ps.parse();
            starts.push_back(p.compile(*ast, match));
        }
    } catch (const SyntaxError& e) {
        *err = "error parsing regexp: " + e.code + ": `" + e.expr + "`";
        return RX_SYNTAX;
    } catch (const UnsupportedError& e) {
        *err = e.why;
        return RX_UNSUPPORTED;
    }
    // union: one start thread per pattern
    // alphabet: boundaries of every rune range, '\n', the ASCII word ranges
    std::vector<uint32_t> cuts = {0, 0x80, '\n', '\n' + 1, '0', '9' + 1, 'A', 'Z' + 1, '_', '_' + 1, 'a', 'z' + 1,
                                  kMaxRune + 1};
    for (auto& i : p.ins)
        if (i.op == I_RUNE)
            for (auto& r : i.r) {
                cuts.push_back(r.first);
                cuts.push_back(r.second + 1);
            }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    while (!cuts.empty() && cuts.back() > kMaxRune + 1) cuts.pop_back();
    // raw class k = [cuts[k], cuts[k+1]).  Raw classes no rune instruction tells apart (same word /
    // '\n' context, same membership everywhere) share one DFA column: partition refinement, one
    // instruction at a time, so \p{L}-sized classes cost a column per distinct behaviour, not per range.
    const uint32_t nrc = (uint32_t)cuts.size() - 1;
    auto span = [&](const std::pair<uint32_t, uint32_t>& r, size_t* a, size_t* b) {
        *a = std::lower_bound(cuts.begin(), cuts.end(), r.first) - cuts.begin();
        *b = std::lower_bound(cuts.begin(), cuts.end(), r.second + 1) - cuts.begin();
    };
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    std::vector<uint32_t> cid(nrc);
    for (uint32_t k = 0; k < nrc; k++) cid[k] = (is_word(cuts[k]) ? 1u : 0u) | (cuts[k] == '\n' ? 2u : 0u);
    uint32_t nid = 4;
    std::vector<uint32_t> remap(nid, kNone), touched;
    for (auto& in : p.ins) {
        if (in.op != I_RUNE) continue;
        for (auto& r : in.r) {
            size_t a, b;
            span(r, &a, &b);
            for (size_t c = a; c < b; c++) {
                const uint32_t old = cid[c];
                if (remap[old] == kNone) {
                    remap[old] = nid++;
                    touched.push_back(old);
                }
                cid[c] = remap[old];
            }
        }
        for (uint32_t o : touched) remap[o] = kNone;
        touched.clear();
        remap.resize(nid, kNone);
    }
    std::vector<uint32_t> comp(nid, kNone), rep_of;
    for (uint32_t k = 0; k < nrc; k++) {
        if (comp[cid[k]] == kNone) {
            comp[cid[k]] = (uint32_t)rep_of.size();
            rep_of.push_back(cuts[k]);
        }
        cid[k] = comp[cid[k]];
    }
    const uint32_t ncc = (uint32_t)rep_of.size();
    if (ncc + 1 > 0xFFFF) {
        *err = "too many rune classes";
        return RX_TOO_BIG;
    }
    Dfa d;
    d.ncls = ncc + 1;  // + END
    for (uint32_t k = 0; k < nrc; k++) {
        if (cuts[k] < 0x80)
            for (uint32_t r = cuts[k]; r < std::min<uint32_t>(cuts[k + 1], 0x80); r++) d.ascii[r] = (uint16_t)cid[k];
        if (cuts[k + 1] > 0x80 && (d.hi_cls.empty() || d.hi_cls.back() != cid[k])) {
            d.hi_lo.push_back(std::max<uint32_t>(cuts[k], 0x80));
            d.hi_cls.push_back((uint16_t)cid[k]);
        }
    }
    // per instruction, per class: does the rune instruction accept the class?
    std::vector<std::vector<uint8_t>> accepts(p.ins.size());
    for (size_t k = 0; k < p.ins.size(); k++) {
        if (p.ins[k].op != I_RUNE) continue;
        accepts[k].assign(ncc, 0);
        for (auto& r : p.ins[k].r) {
            size_t a, b;
            span(r, &a, &b);
            for (size_t c = a; c < b; c++) accepts[k][cid[c]] = 1;
        }
    }
    std::unordered_map<StateKey, uint32_t, StateHash> ids;
    std::vector<StateKey> states;
    auto intern = [&](StateKey k) -> uint32_t {
        auto it = ids.find(k);
        if (it != ids.end()) return it->second;
        const uint32_t id = (uint32_t)states.size();
        ids.emplace(k, id);
        states.push_back(std::move(k));
        return id;
    };
    // epsilon closure under assertion flags; rune instructions go to `out`
    std::vector<uint32_t> mark(p.ins.size(), 0);
    uint32_t stamp = 0;
    std::vector<int32_t> stack;
    auto close = [&](const int32_t* pcs, size_t n, uint8_t flags, std::vector<int32_t>& out) -> bool {
        bool matched = false;
        stack.assign(pcs, pcs + n);
        std::reverse(stack.begin(), stack.end());
        while (!stack.empty()) {
            const int32_t pc = stack.back();
            stack.pop_back();
            if (pc < 0 || mark[pc] == stamp) continue;
            mark[pc] = stamp;
            const Inst& in = p.ins[pc];
            if (in.op == I_SPLIT) {
                stack.push_back(in.y);
                stack.push_back(in.x);
            } else if (in.op == I_EMPTY) {
                if ((in.empty & flags) == in.empty) stack.push_back(in.x);
            } else if (in.op == I_MATCH) {
                matched = true;
            } else {
                out.push_back(pc);
            }
        }
        return matched;
    };
    // the start threads' closure depends only on the assertion flags: computed once per flags value
    std::vector<std::vector<int32_t>> start_cl(64);
    std::vector<int8_t> start_match(64, -1);
    auto start_closure = [&](uint8_t f) -> const std::vector<int32_t>& {
        if (start_match[f] < 0) {
            ++stamp;
            start_match[f] = close(starts.data(), starts.size(), f, start_cl[f]) ? 1 : 0;
        }
        return start_cl[f];
    };
    // over budget: the bit-parallel NFA image (dfa_dev.h) over the same alphabet -- bit j of a thread
    // set is rune instruction j, bit m is MATCH; closures per variant of the flags the program tests
    auto build_nfa = [&]() -> int {
        std::vector<int32_t> pos_of(p.ins.size(), -1), pcs;
        for (size_t k = 0; k < p.ins.size(); k++)
            if (p.ins[k].op == I_RUNE) {
                pos_of[k] = (int32_t)pcs.size();
                pcs.push_back((int32_t)k);
            }
        const uint32_t m = (uint32_t)pcs.size();
        const uint32_t W = (m + 1 + 63) / 64;
        uint32_t tested = 0;
        for (auto& in : p.ins)
            if (in.op == I_EMPTY) tested |= in.empty;
        std::vector<uint32_t> bits;
        for (uint32_t b = 0; b < 6; b++)
            if (tested >> b & 1) bits.push_back(b);
        const uint32_t nvar = 1u << bits.size();
        if (m > kNfaHugePos || ((uint64_t)m + 1 + ncc) * nvar * W * 8 > kNfaMaxBytes) {
            *err = "DFA exceeds the state budget and the program the NFA width";
            return RX_TOO_BIG;
        }
        std::vector<uint64_t> img(MXP_NFA_HDR_WORDS + (size_t)ncc * W + (size_t)(m + 1) * nvar * W, 0);
        img[0] = (uint64_t)m | ((uint64_t)W << 16) | ((uint64_t)nvar << 24);
        uint8_t* var_of = (uint8_t*)&img[1];
        for (uint32_t f = 0; f < 64; f++) {
            uint32_t v = 0;
            for (size_t k = 0; k < bits.size(); k++) v |= (f >> bits[k] & 1u) << k;
            var_of[f] = (uint8_t)v;
        }
        uint64_t* acc = img.data() + MXP_NFA_HDR_WORDS;
        for (uint32_t j = 0; j < m; j++)
            for (uint32_t c = 0; c < ncc; c++)
                if (accepts[pcs[j]][c]) acc[(size_t)c * W + j / 64] |= 1ull << (j % 64);
        uint64_t* cl = acc + (size_t)ncc * W;
        std::vector<int32_t> outv;
        for (uint32_t v = 0; v < nvar; v++) {
            uint8_t f = 0;
            for (size_t k = 0; k < bits.size(); k++)
                if (v >> k & 1) f |= (uint8_t)(1u << bits[k]);
            for (uint32_t j = 0; j <= m; j++) {
                outv.clear();
                ++stamp;
                const bool hit = j < m ? close(&p.ins[pcs[j]].x, 1, f, outv) : close(starts.data(), starts.size(), f, outv);
                uint64_t* row = cl + ((size_t)j * nvar + v) * W;
                for (int32_t pc : outv) row[pos_of[pc] / 64] |= 1ull << (pos_of[pc] % 64);
                if (hit) row[m / 64] |= 1ull << (m % 64);
            }
        }
        Dfa nd;
        nd.ncls = ncc + 1;
        std::copy(d.ascii, d.ascii + 128, nd.ascii);
        nd.hi_lo = d.hi_lo;
        nd.hi_cls = d.hi_cls;
        nd.nfa = std::move(img);
        *out = std::move(nd);
        return RX_OK;
    };
    d.start = intern(StateKey{{}, 1});
    std::vector<int32_t> closure;
    for (uint32_t sidx = 0; sidx < states.size(); sidx++) {
        if (states.size() > max_states) {
            if (nfa_fallback) {
                states.clear();
                ids.clear();
                d.trans.clear();
                d.trans.shrink_to_fit();
                return build_nfa();
            }
            *err = "DFA exceeds the state budget";
            return RX_TOO_BIG;
        }
        const StateKey cur = states[sidx];
        const bool begin = cur.ctx & 1, prev_nl = cur.ctx & 2, prev_word = cur.ctx & 4;
        for (uint32_t c = 0; c <= ncc; c++) {
            const bool end = c == ncc;
            const uint32_t rep = end ? 0 : rep_of[c];
            uint8_t flags = 0;
            if (begin) flags |= BEGIN_TEXT | BEGIN_LINE;
            if (prev_nl) flags |= BEGIN_LINE;
            if (end) flags |= END_TEXT | END_LINE;
            if (!end && rep == '\n') flags |= END_LINE;
            flags |= (prev_word != (!end && is_word(rep))) ? WORD_B : NO_WORD_B;
            // pending threads, then a fresh start thread per pattern (unanchored search)
            const std::vector<int32_t>& sc = start_closure(flags);
            closure.clear();
            ++stamp;
            bool matched = close(cur.pcs.data(), cur.pcs.size(), flags, closure) || start_match[flags] == 1;
            uint32_t next;
            if (matched) {
                next = kDfaAccept;
            } else if (end) {
                next = kDfaReject;
            } else {
                StateKey nk;
                for (int32_t pc : closure)
                    if (accepts[pc][c]) nk.pcs.push_back(p.ins[pc].x);
                for (int32_t pc : sc)
                    if (mark[pc] != stamp && accepts[pc][c]) nk.pcs.push_back(p.ins[pc].x);
                std::sort(nk.pcs.begin(), nk.pcs.end());
                nk.pcs.erase(std::unique(nk.pcs.begin(), nk.pcs.end()), nk.pcs.end());
                nk.ctx = (uint8_t)((rep == '\n' ? 2 : 0) | (is_word(rep) ? 4 : 0));
                next = intern(std::move(nk));
            }
            d.trans.push_back(next);
        }
    }
    d.nstates = (uint32_t)states.size();
    fold_dead_states(&d);
    *out = std::move(d);
    return RX_OK;
}

uint32_t DfaSetHost::add16(const Dfa& d) {
    if (d.is_nfa() || d.nstates > 65533u) return add(d);
    const uint32_t k = add(Dfa());  // (header and alphabet below; no transitions yet)
    mxp_dfa_hdr& h = hdr[k];
    h.ncls = d.ncls;
    h.start = d.start;
    h.kind = MXP_RX_DFA16;
    h.trans = (uint32_t)trans.size();
    const size_t m = d.trans.size();
    trans.resize(trans.size() + (m + 1) / 2, 0u);
    uint16_t* t16 = (uint16_t*)(trans.data() + h.trans);
    for (size_t i = 0; i < m; i++) {
        const uint32_t v = d.trans[i];
        t16[i] = v == kDfaAccept ? 0xFFFFu : v == kDfaReject ? 0xFFFEu : (uint16_t)v;
    }
    ascii.resize(h.ascii);  // (add() appended the empty DFA's alphabet: replace it)
    hilo.resize(h.hi);
    hicls.resize(h.hi);
    h.hi_n = (uint32_t)d.hi_lo.size();
    ascii.insert(ascii.end(), d.ascii, d.ascii + 128);
    hilo.insert(hilo.end(), d.hi_lo.begin(), d.hi_lo.end());
    hicls.insert(hicls.end(), d.hi_cls.begin(), d.hi_cls.end());
    return k;
}

void dfa_renumber_hybrid(Dfa* d, uint32_t bfs_head) {
    const uint32_t N = d->nstates, C = d->ncls;
    if (N < 2 || d->is_nfa()) return;
    std::vector<uint32_t> perm(N, ~0u), order;
    order.reserve(N);
    auto target = [&](uint32_t s, uint32_t c) { return d->trans[(size_t)s * C + c]; };
    // BFS head from the start
    std::vector<uint32_t> queue{d->start};
    perm[d->start] = 0;
    order.push_back(d->start);
    for (size_t i = 0; i < queue.size() && order.size() < bfs_head; i++)
        for (uint32_t c = 0; c < C && order.size() < bfs_head; c++) {
            const uint32_t t = target(queue[i], c);
            if (t < N && perm[t] == ~0u) {
                perm[t] = (uint32_t)order.size();
                order.push_back(t);
                queue.push_back(t);
            }
        }
    // depth-first preorder below the head: the head's children in order, each subtree contiguous
    std::vector<uint32_t> stack;
    for (size_t i = order.size(); i-- > 0;)
        for (uint32_t c = C; c-- > 0;) {
            const uint32_t t = target(order[i], c);
            if (t < N && perm[t] == ~0u) stack.push_back(t);
        }
    while (!stack.empty()) {
        const uint32_t s = stack.back();
        stack.pop_back();
        if (perm[s] != ~0u) continue;
        perm[s] = (uint32_t)order.size();
        order.push_back(s);
        for (uint32_t c = C; c-- > 0;) {
            const uint32_t t = target(s, c);
            if (t < N && perm[t] == ~0u) stack.push_back(t);
        }
    }
    for (uint32_t s = 0; s < N; s++)  // (unreachable states keep a place at the end)
        if (perm[s] == ~0u) {
            perm[s] = (uint32_t)order.size();
            order.push_back(s);
        }
    std::vector<uint32_t> t2((size_t)N * C);
    for (uint32_t k = 0; k < N; k++)
        for (uint32_t c = 0; c < C; c++) {
            const uint32_t t = target(order[k], c);
            t2[(size_t)k * C + c] = t < N ? perm[t] : t;
        }
    d->trans.swap(t2);
    d->start = 0;
}

uint32_t DfaSetHost::add(const Dfa& d) {
    mxp_dfa_hdr h{};
    h.ncls = d.ncls;
    h.start = d.start;
    if (d.is_nfa()) {  // the u64 image, 8-byte aligned in the u32 transition array
        if (trans.size() & 1) trans.push_back(0);
        h.kind = MXP_RX_NFA;
        h.trans = (uint32_t)trans.size();
        const uint32_t* w = (const uint32_t*)d.nfa.data();
        trans.insert(trans.end(), w, w + 2 * d.nfa.size());
    } else {
        h.kind = MXP_RX_DFA;
        h.trans = (uint32_t)trans.size();
        trans.insert(trans.end(), d.trans.begin(), d.trans.end());
    }
    h.ascii = (uint32_t)ascii.size();
    h.hi = (uint32_t)hilo.size();
    h.hi_n = (uint32_t)d.hi_lo.size();
    ascii.insert(ascii.end(), d.ascii, d.ascii + 128);
    hilo.insert(hilo.end(), d.hi_lo.begin(), d.hi_lo.end());
    hicls.insert(hicls.end(), d.hi_cls.begin(), d.hi_cls.end());
    hdr.push_back(h);
    return (uint32_t)hdr.size() - 1;
}

namespace {
uint32_t class_of(const Dfa& d, uint32_t r) {
    if (r < 0x80) return d.ascii[r];
    return d.hi_cls[std::upper_bound(d.hi_lo.begin(), d.hi_lo.end(), r) - d.hi_lo.begin() - 1];
}

// host form of mxp_nfa_run (dfa_dev.h)
bool nfa_match_host(const Dfa& d, const std::string& s) {
    const uint64_t* N = d.nfa.data();
    const uint32_t m = (uint32_t)(N[0] & 0xFFFF), W = (uint32_t)(N[0] >> 16) & 0xFF, nvar = (uint32_t)(N[0] >> 24) & 0xFFFF;
    const uint8_t* var_of = (const uint8_t*)(N + 1);
    const uint64_t* acc = N + MXP_NFA_HDR_WORDS;
    const uint64_t* cl = acc + (size_t)(d.ncls - 1) * W;
    const uint64_t* cls0 = cl + (size_t)m * nvar * W;
    std::vector<uint64_t> U(W, 0), C(W, 0);
    bool begin = true, prev_nl = false, prev_word = false;
    for (size_t i = 0;;) {
        const bool end = i >= s.size();
        size_t w = 1;
        const uint32_t r = end ? 0 : decode_rune(s, i, &w);
        uint8_t f = 0;
        if (begin) f |= BEGIN_TEXT | BEGIN_LINE;
        if (prev_nl) f |= BEGIN_LINE;
        if (end) f |= END_TEXT | END_LINE;
        if (!end && r == '\n') f |= END_LINE;
        f |= (prev_word != (!end && is_word(r))) ? WORD_B : NO_WORD_B;
        const uint32_t v = var_of[f];
        for (uint32_t x = 0; x < W; x++) C[x] = cls0[(size_t)v * W + x];
        for (uint32_t j = 0; j < m; j++)
            if (U[j / 64] >> (j % 64) & 1)
                for (uint32_t x = 0; x < W; x++) C[x] |= cl[((size_t)j * nvar + v) * W + x];
        if (C[m / 64] >> (m % 64) & 1) return true;
        if (end) return false;
        const uint64_t* a = acc + (size_t)class_of(d, r) * W;
        for (uint32_t x = 0; x < W; x++) U[x] = C[x] & a[x];
        begin = false;
        prev_nl = r == '\n';
        prev_word = is_word(r);
        i += w;
    }
}
}  // namespace

// Decided states fold into the two verdicts, so walkers stop at the first byte that settles the
// match instead of reading the rest of the subject:
//   REJECT  states from which ACCEPT is unreachable (an anchored list's near misses): the least
//           fixpoint of "some transition reaches ACCEPT or a live state";
//   ACCEPT  states from which every continuation accepts, the end of text included (a `(/.*)?$`
//           tail after its '/'): the greatest fixpoint of "END accepts and every transition is
//           ACCEPT or stays in the set".
// Transitions into them become kDfaReject / kDfaAccept (the walk's outcome from such a state is
// the verdict whatever follows).  States are in BFS order, so descending sweeps settle in few passes.
void fold_dead_states(Dfa* d) {
    const uint32_t N = d->nstates, C = d->ncls;
    std::vector<uint8_t> live(N, 0), sure(N, 0);
    for (uint32_t s = 0; s < N; s++) sure[s] = d->trans[(size_t)s * C + C - 1] == kDfaAccept;
    for (bool changed = true; changed;) {
        changed = false;
        for (uint32_t s = N; s-- > 0;) {
            const uint32_t* row = d->trans.data() + (size_t)s * C;
            if (!live[s])
                for (uint32_t c = 0; c < C; c++)
                    if (row[c] == kDfaAccept || (row[c] < N && live[row[c]])) {
                        live[s] = 1;
                        changed = true;
                        break;
                    }
            if (sure[s])
                for (uint32_t c = 0; c + 1 < C; c++)
                    if (row[c] != kDfaAccept && !(row[c] < N && sure[row[c]])) {
                        sure[s] = 0;
                        changed = true;
                        break;
                    }
        }
    }
    for (uint32_t& t : d->trans)
        if (t < N) t = sure[t] ? kDfaAccept : !live[t] ? kDfaReject : t;
}

bool dfa_literal_keys(const Dfa& d, uint32_t st, uint32_t max_keys, uint32_t max_depth, std::vector<LiteralKey>* out) {
    out->clear();
    if (d.is_nfa() || st == kDfaReject) return false;
    if (st == kDfaAccept) {
        out->push_back({"", false});
        return true;
    }
    const uint32_t C = d.ncls;
    // `.*$` tail states: from them a match is exactly "no '\n' in the rest of the subject" (end of
    // text accepts, '\n' rejects, every other rune -- non-ASCII and U+FFFD included -- stays in the
    // set): the greatest set closed under those transitions
    std::vector<uint8_t> tail(d.nstates, 0);
    {
        const uint32_t nl = d.ascii['\n'];
        for (uint32_t s = 0; s < d.nstates; s++)
            tail[s] = d.trans[(size_t)s * C + C - 1] == kDfaAccept && d.trans[(size_t)s * C + nl] == kDfaReject;
        for (bool changed = true; changed;) {
            changed = false;
            for (uint32_t s = 0; s < d.nstates; s++) {
                if (!tail[s]) continue;
                auto stays = [&](uint32_t c) {
                    const uint32_t t = d.trans[(size_t)s * C + c];
                    return t < d.nstates && tail[t];
                };
                bool ok = true;
                for (uint32_t b = 0; b < 128 && ok; b++)
                    if (b != '\n') ok = d.ascii[b] != nl && stays(d.ascii[b]);
                for (uint16_t c : d.hi_cls)
                    if (ok) ok = c != nl && stays(c);
                if (!ok) {
                    tail[s] = 0;
                    changed = true;
                }
            }
        }
    }
    // non-ASCII runes (and invalid bytes, U+FFFD) must not lead anywhere but REJECT from the other
    // states the enumeration visits: their keys would be multi-byte runes
    auto hi_dead = [&](uint32_t s) {
        for (uint16_t c : d.hi_cls)
            if (d.trans[(size_t)s * C + c] != kDfaReject) return false;
        return true;
    };
    struct Item {
        uint32_t s;
        std::string w;
    };
    std::vector<Item> level{{st, ""}};
    for (uint32_t depth = 0; !level.empty(); depth++) {
        std::vector<Item> next;
        for (const Item& it : level) {
            if (tail[it.s]) {
                out->push_back({it.w, false, true});
                if (out->size() + next.size() > max_keys) return false;
                continue;
            }
            if (!hi_dead(it.s)) return false;
            if (d.trans[(size_t)it.s * C + C - 1] == kDfaAccept) out->push_back({it.w, true});
            for (uint32_t b = 0; b < 128; b++) {
                const uint32_t t = d.trans[(size_t)it.s * C + d.ascii[b]];
                if (t == kDfaReject) continue;
                std::string w = it.w;
                w.push_back((char)b);
                if (t == kDfaAccept) {
                    out->push_back({w, false});
                } else {
                    if (depth + 1 >= max_depth) return false;
                    next.push_back({t, w});
                }
                if (out->size() + next.size() > max_keys) return false;
            }
        }
        level.swap(next);
    }
    return out->size() <= max_keys;
}

bool dfa_match_host(const Dfa& d, const std::string& s) {
    if (d.is_nfa()) return nfa_match_host(d, s);
    uint32_t st = d.start;
    size_t i = 0;
    while (i < s.size()) {
        size_t w;
        const uint32_t r = decode_rune(s, i, &w);
        i += w;
        uint32_t c;
        if (r < 0x80) {
            c = d.ascii[r];
        } else {
            size_t k = std::upper_bound(d.hi_lo.begin(), d.hi_lo.end(), r) - d.hi_lo.begin() - 1;
            c = d.hi_cls[k];
        }
        st = d.trans[(size_t)st * d.ncls + c];
        if (st == kDfaAccept) return true;
        if (st == kDfaReject) return false;
    }
    return d.trans[(size_t)st * d.ncls + d.ncls - 1] == kDfaAccept;
}

}  // namespace mxp

extern "C" int mxp_regex_match_host(const char* pattern, uint32_t pattern_len, const char* subject,
                                    uint32_t subject_len, char* err, uint32_t err_cap) {
    // (the last pattern's automaton is kept per thread: callers sweep subjects per pattern)
    thread_local std::string last;
    thread_local bool have = false;
    thread_local mxp::Dfa d;
    thread_local std::string e;
    thread_local int rc = 0;
    const std::string pat(pattern ? pattern : "", pattern_len);
    if (!have || pat != last) {
        d = mxp::Dfa();
        e.clear();
        rc = mxp::regex_compile({pat}, 1u << 16, &d, &e);  // the rules' budget
        last = pat;
        have = true;
    }
    if (err && err_cap) {
        const size_t n = std::min<size_t>(e.size(), err_cap - 1);
        memcpy(err, e.data(), n);
        err[n] = 0;
    }
    if (rc == mxp::RX_SYNTAX) return -1;
    if (rc == mxp::RX_UNSUPPORTED) return -2;
    if (rc != mxp::RX_OK) return -3;
    return mxp::dfa_match_host(d, std::string(subject ? subject : "", subject_len)) ? 1 : 0;
}
