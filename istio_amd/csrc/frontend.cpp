// frontend.cpp -- see frontend.h.
//
// The scanner/parser reproduce go/scanner and go/parser (Go 1.9) for single expressions, including
// the error conventions that reach users: "line:col: msg", one parser error per line, scanner
// errors always recorded, "(and N more errors)" suffix, and the inRhs quirk that reports
// `a = 2` as "expected '==', found '='".
#include "frontend.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "goutil.h"

namespace mxp {

const char* value_type_name(int32_t vt) {
    static const char* names[] = {"VALUE_TYPE_UNSPECIFIED", "STRING", "INT64", "DOUBLE", "BOOL", "TIMESTAMP",
                                  "IP_ADDRESS", "EMAIL_ADDRESS", "URI", "DNS_NAME", "DURATION", "STRING_MAP"};
    if (vt >= 0 && vt < 12) return names[vt];
    return "?";
}

std::string Expr::str() const {
    switch (kind) {
    case CONST: return c.src;
    case VAR: return "$" + var;
    case FN: {
        std::string s;
        if (target) s += target->str() + ":";
        s += fn + "(";
        for (size_t i = 0; i < args.size(); i++) {
            if (i) s += ", ";
            s += args[i]->str();
        }
        return s + ")";
    }
    default: return "<nil>";
    }
}

FuncMap default_func_map() {
    FuncMap m;
    auto add = [&](const char* n, bool inst, int32_t tt, int32_t rt, std::vector<int32_t> a) {
        FunctionMetadata f;
        f.name = n;
        f.instance = inst;
        f.target_type = tt;
        f.return_type = rt;
        f.arg_types = std::move(a);
        m[n] = f;
    };
    // intrinsics, func.go:39-72
    add("EQ", false, 0, VT_BOOL, {0, 0});
    add("NEQ", false, 0, VT_BOOL, {0, 0});
    add("OR", false, 0, 0, {0, 0});
    add("LOR", false, 0, VT_BOOL, {VT_BOOL, VT_BOOL});
    add("LAND", false, 0, VT_BOOL, {VT_BOOL, VT_BOOL});
    add("INDEX", false, 0, VT_STRING, {VT_STRING_MAP, VT_STRING});
    // externs, il/runtime/externs.go:42-79
    add("ip", false, 0, VT_IP_ADDRESS, {VT_STRING});
    add("timestamp", false, 0, VT_TIMESTAMP, {VT_STRING});
    add("match", false, 0, VT_BOOL, {VT_STRING, VT_STRING});
    add("matches", true, VT_STRING, VT_BOOL, {VT_STRING});
    add("startsWith", true, VT_STRING, VT_BOOL, {VT_STRING});
    add("endsWith", true, VT_STRING, VT_BOOL, {VT_STRING});
    return m;
}

namespace {

// ------------------------------------------------------------------------------ scanner
enum TokKind { T_EOF, T_ILLEGAL, T_IDENT, T_INT, T_FLOAT, T_IMAG, T_CHAR, T_STRING, T_OP, T_SEMI };

struct Tok {
    TokKind kind = T_EOF;
    std::string lit;
    size_t off = 0;
};

const char* kKeywords[] = {"break", "case", "chan", "const", "continue", "default", "defer", "else",
                           "fallthrough", "for", "func", "go", "goto", "if", "import", "interface", "map",
                           "package", "range", "return", "select", "struct", "switch", "type", "var"};

bool is_keyword(const std::string& s) {
    for (const char* k : kKeywords)
        if (s == k) return true;
    return false;
}

struct ErrorList {
    struct E {
        int line, col;
        std::string msg;
    };
    std::vector<E> v;
};

// decode one UTF-8 rune at s[i]; returns length (1 for invalid bytes) and the rune (0xFFFD if bad)
size_t rune_at(const std::string& s, size_t i, uint32_t* r) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
        *r = c;
        return 1;
    }
    int n = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (n == 0 || i + n > s.size()) {
        *r = 0xFFFD;
        return 1;
    }
    uint32_t v = c & (0x7F >> n);
    for (int k = 1; k < n; k++) {
        unsigned char cc = (unsigned char)s[i + k];
        if ((cc >> 6) != 2) {
            *r = 0xFFFD;
            return 1;
        }
        v = (v << 6) | (cc & 0x3F);
    }
    *r = v;
    return n;
}

bool rune_is_letter(uint32_t r) {
    if (r == '_' || (r >= 'a' && r <= 'z') || (r >= 'A' && r <= 'Z')) return true;
    if (r < 0x80) return false;
    // Non-ASCII letters: approximate unicode.IsLetter with the Latin-1/Greek/Cyrillic/CJK blocks.
    return (r >= 0xC0 && r != 0xD7 && r != 0xF7 && r < 0x2000) || (r >= 0x3040 && r < 0xA000) ||
           (r >= 0xAC00 && r < 0xD7A4);
}

class Scanner {
  public:
    Scanner(const std::string& src, ErrorList* errs) : s_(src), errs_(errs) {}

    void position(size_t off, int* line, int* col) const {
        int l = 1;
        size_t start = 0;
        for (size_t i = 0; i < off && i < s_.size(); i++)
            if (s_[i] == '\n') {
                l++;
                start = i + 1;
            }
        *line = l;
        *col = (int)(off - start) + 1;
    }

    void error(size_t off, const std::string& msg) {
        int l, c;
        position(off, &l, &c);
        errs_->v.push_back({l, c, msg});
    }

    Tok scan() {
        for (;;) {
            while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\r' ||
                                      (s_[p_] == '\n' && !semi_)))
                p_++;
            Tok t;
            t.off = p_;
            if (p_ >= s_.size()) {
                if (semi_) {
                    semi_ = false;
                    t.kind = T_SEMI;
                    t.lit = "\n";
                    return t;
                }
                t.kind = T_EOF;
                return t;
            }
            uint32_t r;
            size_t rl = rune_at(s_, p_, &r);
            if (rune_is_letter(r)) {
                size_t q = p_;
                for (;;) {
                    if (q >= s_.size()) break;
                    uint32_t rr;
                    size_t l = rune_at(s_, q, &rr);
                    if (rune_is_letter(rr) || (rr >= '0' && rr <= '9')) q += l;
                    else break;
                }
                t.kind = T_IDENT;
                t.lit = s_.substr(p_, q - p_);
                p_ = q;
                semi_ = !is_keyword(t.lit) || t.lit == "break" || t.lit == "continue" || t.lit == "fallthrough" ||
                        t.lit == "return";
                return t;
            }
            char c = s_[p_];
            if ((c >= '0' && c <= '9') || (c == '.' && p_ + 1 < s_.size() && s_[p_ + 1] >= '0' && s_[p_ + 1] <= '9')) {
                semi_ = true;
                return number();
            }
            if (c == '\n') {
                p_++;
                semi_ = false;
                t.kind = T_SEMI;
                t.lit = "\n";
                return t;
            }
            if (c == '"') {
                semi_ = true;
                return string_lit();
            }
            if (c == '`') {
                semi_ = true;
                size_t q = p_ + 1;
                while (q < s_.size() && s_[q] != '`') q++;
                if (q >= s_.size()) {
                    error(p_, "raw string literal not terminated");
                    t.kind = T_STRING;
                    t.lit = s_.substr(p_);
                    p_ = s_.size();
                    return t;
                }
                t.kind = T_STRING;
                t.lit = s_.substr(p_, q + 1 - p_);
                p_ = q + 1;
                return t;
            }
            if (c == '\'') {
                semi_ = true;
                return rune_lit();
            }
            if (c == '/' && p_ + 1 < s_.size() && (s_[p_ + 1] == '/' || s_[p_ + 1] == '*')) {
                if (s_[p_ + 1] == '/') {
                    while (p_ < s_.size() && s_[p_] != '\n') p_++;
                } else {
                    size_t e = s_.find("*/", p_ + 2);
                    if (e == std::string::npos) {
                        error(p_, "comment not terminated");
                        p_ = s_.size();
                    } else {
                        p_ = e + 2;
                    }
                }
                continue;
            }
            static const char* ops[] = {"<<=", ">>=", "&^=", "...", "&&", "||", "<-", "++", "--", "==", "!=", "<=",
                                        ">=", ":=", "+=", "-=", "*=", "/=", "%=", "&=", "|=", "^=", "<<", ">>",
                                        "&^", "+", "-", "*", "/", "%", "&", "|", "^", "<", ">", "=", "!", "(",
                                        "[", "{", ",", ".", ")", "]", "}", ";", ":"};
            for (const char* op : ops) {
                size_t l = strlen(op);
                if (s_.compare(p_, l, op) == 0) {
                    t.kind = T_OP;
                    t.lit = op;
                    p_ += l;
                    semi_ = t.lit == ")" || t.lit == "]" || t.lit == "}" || t.lit == "++" || t.lit == "--";
                    return t;
                }
            }
            char buf[64];
            std::string ch = s_.substr(p_, rl);
            snprintf(buf, sizeof buf, "illegal character U+%04X '", r);
            error(p_, std::string(buf) + ch + "'");
            t.kind = T_ILLEGAL;
            t.lit = ch;
            p_ += rl;
            return t;
        }
    }

  private:
    static bool isdig(char c, int base) {
        if (base == 16) return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
        return c >= '0' && c <= '9';
    }
    void digits(int base) {
        while (p_ < s_.size() && isdig(s_[p_], base)) p_++;
    }

    Tok number() {
        Tok t;
        t.off = p_;
        t.kind = T_INT;
        size_t start = p_;
        bool frac_only = s_[p_] == '.';
        if (!frac_only && s_[p_] == '0') {
            p_++;
            if (p_ < s_.size() && (s_[p_] == 'x' || s_[p_] == 'X')) {
                p_++;
                size_t h = p_;
                digits(16);
                if (p_ == h) error(start, "illegal hexadecimal number");
                t.lit = s_.substr(start, p_ - start);
                return t;
            }
            bool bad_octal = false;
            while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') {
                if (s_[p_] > '7') bad_octal = true;
                p_++;
            }
            if (p_ >= s_.size() || (s_[p_] != '.' && s_[p_] != 'e' && s_[p_] != 'E' && s_[p_] != 'i')) {
                if (bad_octal) error(start, "illegal octal number");
                t.lit = s_.substr(start, p_ - start);
                return t;
            }
        } else if (!frac_only) {
            digits(10);
        }
        if (p_ < s_.size() && s_[p_] == '.') {
            t.kind = T_FLOAT;
            p_++;
            digits(10);
        }
        if (p_ < s_.size() && (s_[p_] == 'e' || s_[p_] == 'E')) {
            t.kind = T_FLOAT;
            p_++;
            if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) p_++;
            size_t e = p_;
            digits(10);
            if (e == p_) error(start, "illegal floating-point exponent");
        }
        if (p_ < s_.size() && s_[p_] == 'i') {
            t.kind = T_IMAG;
            p_++;
        }
        t.lit = s_.substr(start, p_ - start);
        return t;
    }

    bool escape(char quote) {
        size_t off = p_;
        if (p_ >= s_.size()) {
            error(off, "escape sequence not terminated");
            return false;
        }
        char c = s_[p_];
        int n, base;
        uint32_t max;
        if (strchr("abfnrtv\\", c) || c == quote) {
            p_++;
            return true;
        }
        if (c >= '0' && c <= '7') {
            n = 3, base = 8, max = 255;
        } else if (c == 'x') {
            p_++;
            n = 2, base = 16, max = 255;
        } else if (c == 'u') {
            p_++;
            n = 4, base = 16, max = 0x10FFFF;
        } else if (c == 'U') {
            p_++;
            n = 8, base = 16, max = 0x10FFFF;
        } else {
            error(off, "unknown escape sequence");
            return false;
        }
        uint32_t x = 0;
        for (int i = 0; i < n; i++) {
            if (p_ >= s_.size()) {
                error(off, "escape sequence not terminated");
                return false;
            }
            char d = s_[p_];
            int v = (d >= '0' && d <= '9') ? d - '0' : (d >= 'a' && d <= 'f') ? d - 'a' + 10
                    : (d >= 'A' && d <= 'F') ? d - 'A' + 10 : 99;
            if (v >= base) {
                char buf[64];
                snprintf(buf, sizeof buf, "illegal character U+%04X in escape sequence", (unsigned)(unsigned char)d);
                error(p_, buf);
                return false;
            }
            x = x * base + v;
            p_++;
        }
        if (x > max || (x >= 0xD800 && x < 0xE000)) {
            error(off, "escape sequence is invalid Unicode code point");
            return false;
        }
        return true;
    }

    Tok string_lit() {
        Tok t;
        t.off = p_;
        t.kind = T_STRING;
        size_t start = p_++;
        for (;;) {
            if (p_ >= s_.size() || s_[p_] == '\n') {
                error(start, "string literal not terminated");
                break;
            }
            char c = s_[p_++];
            if (c == '"') break;
            if (c == '\\') escape('"');
        }
        t.lit = s_.substr(start, p_ - start);
        return t;
    }

    Tok rune_lit() {
        Tok t;
        t.off = p_;
        t.kind = T_CHAR;
        size_t start = p_++;
        bool valid = true;
        int n = 0;
        for (;;) {
            if (p_ >= s_.size() || s_[p_] == '\n') {
                if (valid) {
                    error(start, "rune literal not terminated");
                    valid = false;
                }
                break;
            }
            uint32_t r;
            size_t l = rune_at(s_, p_, &r);
            p_ += l;
            if (r == '\'') break;
            n++;
            if (r == '\\' && !escape('\'')) valid = false;
        }
        if (valid && n != 1) error(start, "illegal rune literal");
        t.lit = s_.substr(start, p_ - start);
        return t;
    }

    const std::string& s_;
    ErrorList* errs_;
    size_t p_ = 0;
    bool semi_ = false;
};

// ------------------------------------------------------------------------------ go/ast subset
struct GoNode {
    enum K { IDENT, LIT, PAREN, SELECTOR, INDEX, CALL, UNARY, BINARY, STAR, OTHER } k;
    std::string name;  // ident name / selector name / operator / literal text / OTHER description
    TokKind lit_kind = T_EOF;
    std::vector<std::unique_ptr<GoNode>> kids;  // x, y, args...
};
using GoP = std::unique_ptr<GoNode>;

GoP mk(GoNode::K k, std::string name = "") {
    GoP n(new GoNode());
    n->k = k;
    n->name = std::move(name);
    return n;
}

struct Bailout {};

int prec_of(const std::string& op) {
    if (op == "||") return 1;
    if (op == "&&") return 2;
    if (op == "==" || op == "!=" || op == "<" || op == "<=" || op == ">" || op == ">=") return 3;
    if (op == "+" || op == "-" || op == "|" || op == "^") return 4;
    if (op == "*" || op == "/" || op == "%" || op == "<<" || op == ">>" || op == "&" || op == "&^") return 5;
    return 0;
}

class Parser {
  public:
    explicit Parser(const std::string& src) : sc_(src, &errs_) { next(); }

    GoP parse(std::string* err) {
        GoP x;
        try {
            x = expr();
            if (tok_.kind == T_SEMI && tok_.lit == "\n") next();
            if (tok_.kind != T_EOF) {
                expected(tok_.off, "'EOF'");
                throw Bailout();
            }
        } catch (Bailout&) {
            x.reset();
            while (tok_.kind != T_EOF) next();
        }
        if (!errs_.v.empty()) {
            std::stable_sort(errs_.v.begin(), errs_.v.end(), [](const ErrorList::E& a, const ErrorList::E& b) {
                return a.line != b.line ? a.line < b.line : a.col < b.col;
            });
            const auto& e = errs_.v[0];
            std::string m = std::to_string(e.line) + ":" + std::to_string(e.col) + ": " + e.msg;
            if (errs_.v.size() > 1) m += " (and " + std::to_string(errs_.v.size() - 1) + " more errors)";
            *err = m;
            return nullptr;
        }
        return x;
    }

  private:
    void next() { tok_ = sc_.scan(); }
    bool is_op(const char* s) const { return tok_.kind == T_OP && tok_.lit == s; }

    std::string tok_string(const Tok& t) const {
        switch (t.kind) {
        case T_OP: return t.lit;
        case T_SEMI: return ";";
        case T_IDENT: return is_keyword(t.lit) ? t.lit : "IDENT";
        case T_INT: return "INT";
        case T_FLOAT: return "FLOAT";
        case T_IMAG: return "IMAG";
        case T_CHAR: return "CHAR";
        case T_STRING: return "STRING";
        case T_EOF: return "EOF";
        default: return "ILLEGAL";
        }
    }

    void error(size_t off, const std::string& msg) {
        int l, c;
        sc_.position(off, &l, &c);
        if (!errs_.v.empty() && errs_.v.back().line == l) return;  // one parser error per line
        errs_.v.push_back({l, c, msg});
    }

    void expected(size_t off, const std::string& what) {
        std::string msg = "expected " + what;
        if (off == tok_.off) {
            if (tok_.kind == T_SEMI && tok_.lit == "\n") {
                msg += ", found newline";
            } else {
                std::string ts = tok_string(tok_);
                msg += ", found '" + ts + "'";
                bool literal = tok_.kind == T_IDENT || tok_.kind == T_INT || tok_.kind == T_FLOAT ||
                               tok_.kind == T_IMAG || tok_.kind == T_CHAR || tok_.kind == T_STRING;
                if (literal && !(tok_.kind == T_IDENT && is_keyword(tok_.lit))) msg += " " + tok_.lit;
            }
        }
        error(off, msg);
    }

    void expect(const std::string& op) {
        if (!(tok_.kind == T_OP && tok_.lit == op)) {
            expected(tok_.off, "'" + op + "'");
            throw Bailout();
        }
        next();
    }

    GoP expr() { return binary(1); }

    GoP binary(int prec1) {
        GoP x = unary();
        for (;;) {
            if (tok_.kind != T_OP) return x;
            std::string op = tok_.lit == "=" ? "==" : tok_.lit;  // go/parser inRhs: ASSIGN ~ EQL
            int p = prec_of(op);
            if (p < prec1) return x;
            expect(op);
            GoP y = binary(p + 1);
            GoP b = mk(GoNode::BINARY, op);
            b->kids.push_back(std::move(x));
            b->kids.push_back(std::move(y));
            x = std::move(b);
        }
    }

    GoP unary() {
        if (tok_.kind == T_OP && (tok_.lit == "+" || tok_.lit == "-" || tok_.lit == "!" || tok_.lit == "^" ||
                                  tok_.lit == "&" || tok_.lit == "<-")) {
            std::string op = tok_.lit;
            next();
            GoP u = mk(GoNode::UNARY, op);
            u->kids.push_back(unary());
            return u;
        }
        if (is_op("*")) {
            next();
            GoP s = mk(GoNode::STAR);
            s->kids.push_back(unary());
            return s;
        }
        return primary();
    }

    void skip_balanced(const char* o, const char* c) {
        int depth = 0;
        for (;;) {
            if (tok_.kind == T_EOF) {
                expected(tok_.off, std::string("'") + c + "'");
                throw Bailout();
            }
            if (is_op(o)) depth++;
            if (is_op(c) && --depth == 0) {
                next();
                return;
            }
            next();
        }
    }

    void type_rest(const std::string& kw) {
        if (kw == "struct" || kw == "interface") {
            if (is_op("{")) skip_balanced("{", "}");
            return;
        }
        if (kw == "func") {
            if (is_op("(")) skip_balanced("(", ")");
            if (is_op("{")) skip_balanced("{", "}");
            return;
        }
        if (kw == "map" && is_op("[")) skip_balanced("[", "]");
        if (tok_.kind == T_IDENT) {
            next();
            while (is_op(".")) {
                next();
                if (tok_.kind == T_IDENT) next();
            }
        } else if (is_op("*")) {
            next();
            type_rest("");
        } else if (is_op("[")) {
            skip_balanced("[", "]");
            type_rest("");
        }
    }

    GoP operand() {
        if (tok_.kind == T_IDENT && !is_keyword(tok_.lit)) {
            GoP n = mk(GoNode::IDENT, tok_.lit);
            next();
            return n;
        }
        if (tok_.kind == T_INT || tok_.kind == T_FLOAT || tok_.kind == T_IMAG || tok_.kind == T_CHAR ||
            tok_.kind == T_STRING) {
            GoP n = mk(GoNode::LIT, tok_.lit);
            n->lit_kind = tok_.kind;
            next();
            return n;
        }
        if (is_op("(")) {
            next();
            lev_++;
            GoP x = expr();
            lev_--;
            expect(")");
            GoP p = mk(GoNode::PAREN);
            p->kids.push_back(std::move(x));
            return p;
        }
        if (is_op("[")) {
            skip_balanced("[", "]");
            type_rest("");
            return mk(GoNode::OTHER, "ArrayType");
        }
        if (tok_.kind == T_IDENT &&
            (tok_.lit == "map" || tok_.lit == "chan" || tok_.lit == "struct" || tok_.lit == "interface" ||
             tok_.lit == "func")) {
            std::string kw = tok_.lit;
            next();
            type_rest(kw);
            return mk(GoNode::OTHER, kw);
        }
        expected(tok_.off, "operand");
        throw Bailout();
    }

    static bool literal_type(const GoNode& x) {
        if (x.k == GoNode::IDENT) return true;
        if (x.k == GoNode::SELECTOR) return x.kids[0]->k == GoNode::IDENT;
        return x.k == GoNode::OTHER && (x.name == "ArrayType" || x.name == "map" || x.name == "struct");
    }

    GoP primary() {
        GoP x = operand();
        for (;;) {
            if (is_op(".")) {
                next();
                if (tok_.kind == T_IDENT) {
                    GoP s = mk(GoNode::SELECTOR, tok_.lit);
                    next();
                    s->kids.push_back(std::move(x));
                    x = std::move(s);
                } else if (is_op("(")) {
                    next();
                    if (tok_.kind == T_IDENT && tok_.lit == "type") next();
                    else expr();
                    expect(")");
                    x = mk(GoNode::OTHER, "TypeAssertExpr");
                } else {
                    expected(tok_.off, "selector or type assertion");
                    throw Bailout();
                }
            } else if (is_op("[")) {
                next();
                lev_++;
                GoP idx;
                int colons = 0;
                if (!is_op(":")) idx = expr();
                while (is_op(":") && colons < 2) {
                    colons++;
                    next();
                    if (!is_op(":") && !is_op("]")) expr();
                }
                lev_--;
                expect("]");
                if (colons) {
                    x = mk(GoNode::OTHER, "SliceExpr");
                } else {
                    GoP ix = mk(GoNode::INDEX);
                    ix->kids.push_back(std::move(x));
                    ix->kids.push_back(std::move(idx));
                    x = std::move(ix);
                }
            } else if (is_op("(")) {
                next();
                lev_++;
                GoP call = mk(GoNode::CALL);
                call->kids.push_back(std::move(x));
                while (!is_op(")") && tok_.kind != T_EOF) {
                    call->kids.push_back(expr());
                    if (is_op("...")) next();
                    if (!is_op(",")) break;
                    next();
                }
                lev_--;
                expect(")");
                x = std::move(call);
            } else if (is_op("{")) {
                if (literal_type(*x) && (lev_ >= 0 || (x->k != GoNode::IDENT && x->k != GoNode::SELECTOR))) {
                    skip_balanced("{", "}");
                    x = mk(GoNode::OTHER, "CompositeLit");
                } else {
                    return x;
                }
            } else {
                return x;
            }
        }
    }

    ErrorList errs_;
    Scanner sc_;
    Tok tok_;
    int lev_ = 0;
};

// ------------------------------------------------------------------------------ process
struct ProcessError {
    std::string msg;
};

std::string op_name(const std::string& op) {
    static const char* tbl[][2] = {{"+", "ADD"}, {"-", "SUB"}, {"*", "MUL"}, {"/", "QUO"},  {"%", "REM"},
                                   {"&", "AND"}, {"|", "OR"},  {"^", "XOR"}, {"&&", "LAND"}, {"||", "LOR"},
                                   {"==", "EQ"}, {"<", "LT"},  {">", "GT"},  {"!", "NOT"},  {"!=", "NEQ"},
                                   {"<=", "LEQ"}, {">=", "GEQ"}};
    for (auto& e : tbl)
        if (op == e[0]) return e[1];
    return "";
}

std::string describe(const GoNode& n) {
    switch (n.k) {
    case GoNode::IDENT: return "&ast.Ident{Name:\"" + n.name + "\"}";
    case GoNode::STAR: return "&ast.StarExpr{...}";
    case GoNode::SELECTOR: return "&ast.SelectorExpr{...}";
    case GoNode::INDEX: return "&ast.IndexExpr{...}";
    case GoNode::CALL: return "&ast.CallExpr{...}";
    default: return "&ast." + (n.name.empty() ? std::string("Expr") : n.name) + "{...}";
    }
}

void process(const GoNode& n, Expr& tgt);

void process_args(Expr& fn, const std::vector<const GoNode*>& args) {
    for (const GoNode* a : args) {
        fn.args.emplace_back(new Expr());
        process(*a, *fn.args.back());
    }
}

// flattenSelectors (expr.go:384-408)
const GoNode* flatten(const GoNode& sel, std::vector<std::string>* parts) {
    const GoNode* ex = &sel;
    for (;;) {
        parts->push_back(ex->name);
        const GoNode& x = *ex->kids[0];
        if (x.k == GoNode::SELECTOR) {
            ex = &x;
        } else if (x.k == GoNode::IDENT) {
            parts->push_back(x.name);
            return nullptr;
        } else if (x.k == GoNode::CALL || x.k == GoNode::LIT || x.k == GoNode::PAREN) {
            return &x;
        } else {
            throw ProcessError{"unexpected expression: " + describe(x)};
        }
    }
}

std::string var_name(const std::vector<std::string>& sel, size_t from) {
    std::string s;
    for (size_t i = sel.size(); i-- > from;) {
        if (!s.empty()) s += ".";
        s += sel[i];
    }
    return s;
}

void new_constant(const std::string& v, int32_t vt, Constant* c) {
    c->src = v;
    c->type = vt;
    std::string err;
    if (vt == VT_INT64) {
        if (!go_parse_int10(v, &c->i, &err)) throw ProcessError{err};
        return;
    }
    if (vt == VT_DOUBLE) {
        if (!go_parse_float(v, &c->d, &err)) throw ProcessError{err};
        return;
    }
    std::string u;
    if (!go_unquote(v, &u)) throw ProcessError{"invalid syntax"};
    int64_t dur;
    if (go_parse_duration(u, &dur, nullptr)) {
        c->type = VT_DURATION;
        c->i = dur;
        return;
    }
    c->s = u;
}

void process(const GoNode& n, Expr& tgt) {
    switch (n.k) {
    case GoNode::UNARY:
        tgt.kind = Expr::FN;
        tgt.fn = op_name(n.name);
        process_args(tgt, {n.kids[0].get()});
        return;
    case GoNode::BINARY:
        tgt.kind = Expr::FN;
        tgt.fn = op_name(n.name);
        process_args(tgt, {n.kids[0].get(), n.kids[1].get()});
        return;
    case GoNode::CALL: {
        const GoNode& fun = *n.kids[0];
        std::vector<const GoNode*> args;
        for (size_t i = 1; i < n.kids.size(); i++) args.push_back(n.kids[i].get());
        if (fun.k == GoNode::SELECTOR) {
            std::vector<std::string> w;
            const GoNode* anchor = flatten(fun, &w);
            tgt.kind = Expr::FN;
            tgt.fn = w[0];
            tgt.target.reset(new Expr());
            if (!anchor) {
                tgt.target->kind = Expr::VAR;
                tgt.target->var = var_name(w, 1);
            } else {
                process(*anchor, *tgt.target);
                if (w.size() != 1) throw ProcessError{"unexpected expression: " + describe(fun)};
            }
            process_args(tgt, args);
        } else if (fun.k == GoNode::IDENT) {
            tgt.kind = Expr::FN;
            tgt.fn = fun.name;
            process_args(tgt, args);
        }
        // any other callee leaves tgt empty, exactly like the reference (nil Fn at EvalType)
        return;
    }
    case GoNode::PAREN:
        process(*n.kids[0], tgt);
        return;
    case GoNode::LIT: {
        int32_t vt = n.lit_kind == T_INT ? VT_INT64 : n.lit_kind == T_FLOAT ? VT_DOUBLE
                     : (n.lit_kind == T_CHAR || n.lit_kind == T_STRING) ? VT_STRING : VT_UNSPECIFIED;
        tgt.kind = Expr::CONST;
        new_constant(n.name, vt, &tgt.c);
        return;
    }
    case GoNode::IDENT: {
        std::string lv = n.name;
        for (auto& ch : lv) ch = (char)tolower((unsigned char)ch);
        if (lv == "true" || lv == "false") {
            tgt.kind = Expr::CONST;
            tgt.c.src = lv;
            tgt.c.type = VT_BOOL;
            tgt.c.b = lv == "true";
        } else {
            tgt.kind = Expr::VAR;
            tgt.var = n.name;
        }
        return;
    }
    case GoNode::SELECTOR: {
        std::vector<std::string> w;
        if (flatten(n, &w)) throw ProcessError{"unexpected expression: " + describe(n)};
        tgt.kind = Expr::VAR;
        tgt.var = var_name(w, 0);
        return;
    }
    case GoNode::INDEX:
        tgt.kind = Expr::FN;
        tgt.fn = "INDEX";
        process_args(tgt, {n.kids[0].get(), n.kids[1].get()});
        return;
    default:
        throw ProcessError{"unexpected expression: " + describe(n)};
    }
}

struct TypeError {
    std::string msg;
    bool panic;
};

int32_t etype(const Expr& e, const Vocabulary& v, const FuncMap& f);

int32_t ftype(const Expr& e, const Vocabulary& v, const FuncMap& fm) {
    auto it = fm.find(e.fn);
    if (it == fm.end()) throw TypeError{"unknown function: " + e.fn, false};
    const FunctionMetadata& fn = it->second;
    int32_t tmpl = VT_UNSPECIFIED;
    if (e.target) {
        if (!fn.instance) throw TypeError{"invoking regular function on instance method: " + e.fn, false};
        int32_t tt = etype(*e.target, v, fm);
        if (fn.target_type == VT_UNSPECIFIED) tmpl = tt;
        else if (tt != fn.target_type)
            throw TypeError{e.str() + " target typeError got " + value_type_name(tt) + ", expected " +
                                value_type_name(fn.target_type),
                            false};
    } else if (fn.instance) {
        throw TypeError{"invoking instance method without an instance: " + e.fn, false};
    }
    if (e.args.size() < fn.arg_types.size())
        throw TypeError{e.str() + " arity mismatch. Got " + std::to_string(e.args.size()) + " arg(s), expected " +
                            std::to_string(fn.arg_types.size()) + " arg(s)",
                        false};
    for (size_t i = 0; i < e.args.size() && i < fn.arg_types.size(); i++) {
        int32_t at = etype(*e.args[i], v, fm);
        int32_t want = fn.arg_types[i];
        if (want == VT_UNSPECIFIED) {
            if (tmpl == VT_UNSPECIFIED) {
                tmpl = at;
                continue;
            }
            want = tmpl;
        }
        if (at != want)
            throw TypeError{e.str() + " arg " + std::to_string(i + 1) + " (" + e.args[i]->str() + ") typeError got " +
                                value_type_name(at) + ", expected " + value_type_name(want),
                            false};
    }
    return fn.return_type == VT_UNSPECIFIED ? tmpl : fn.return_type;
}

int32_t etype(const Expr& e, const Vocabulary& v, const FuncMap& f) {
    switch (e.kind) {
    case Expr::CONST: return e.c.type;
    case Expr::VAR: {
        auto it = v.find(e.var);
        if (it == v.end()) throw TypeError{"unknown attribute " + e.var, false};
        return it->second;
    }
    case Expr::FN: return ftype(e, v, f);
    default: throw TypeError{"runtime error: invalid memory address or nil pointer dereference", true};
    }
}

}  // namespace

ExprP parse_expression(const std::string& src, std::string* err) {
    Parser p(src);
    std::string perr;
    GoP ast = p.parse(&perr);
    if (!ast) {
        *err = "unable to parse expression '" + src + "': " + perr;
        return nullptr;
    }
    ExprP e(new Expr());
    try {
        process(*ast, *e);
    } catch (ProcessError& pe) {
        *err = pe.msg;
        return nullptr;
    }
    return e;
}

bool eval_type(const Expr& e, const Vocabulary& v, const FuncMap& f, int32_t* out, std::string* err, bool* panicked) {
    try {
        *out = etype(e, v, f);
        if (panicked) *panicked = false;
        return true;
    } catch (TypeError& te) {
        *err = te.msg;
        if (panicked) *panicked = te.panic;
        return false;
    }
}

}  // namespace mxp
