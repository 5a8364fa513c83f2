// ilgen.cpp -- see ilgen.h.
#include "ilgen.h"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace mxp {

const char* il_type_name(uint8_t t) {
    static const char* n[] = {"unknown", "void", "string", "integer", "double", "bool", "duration", "interface"};
    return t < 8 ? n[t] : "unknown";
}

static const std::map<uint32_t, OpInfo>& op_table() {
    static const std::map<uint32_t, OpInfo> t = {
        {Halt, {"halt", {}}}, {Nop, {"nop", {}}}, {Err, {"err", {ARG_STR}}}, {Errz, {"errz", {ARG_STR}}},
        {Errnz, {"errnz", {ARG_STR}}}, {PopS, {"pop_s", {}}}, {PopB, {"pop_b", {}}}, {PopI, {"pop_i", {}}},
        {PopD, {"pop_d", {}}}, {DupS, {"dup_s", {}}}, {DupB, {"dup_b", {}}}, {DupI, {"dup_i", {}}},
        {DupD, {"dup_d", {}}}, {RLoadS, {"rload_s", {ARG_REG}}}, {RLoadB, {"rload_b", {ARG_REG}}},
        {RLoadI, {"rload_i", {ARG_REG}}}, {RLoadD, {"rload_d", {ARG_REG}}},
        {ALoadS, {"aload_s", {ARG_REG, ARG_STR}}}, {ALoadB, {"aload_b", {ARG_REG, ARG_BOOL}}},
        {ALoadI, {"aload_i", {ARG_REG, ARG_INT}}}, {ALoadD, {"aload_d", {ARG_REG, ARG_DBL}}},
        {APushS, {"apush_s", {ARG_STR}}}, {APushB, {"apush_b", {ARG_BOOL}}}, {APushI, {"apush_i", {ARG_INT}}},
        {APushD, {"apush_d", {ARG_DBL}}}, {RPushS, {"rpush_s", {ARG_REG}}}, {RPushB, {"rpush_b", {ARG_REG}}},
        {RPushI, {"rpush_i", {ARG_REG}}}, {RPushD, {"rpush_d", {ARG_REG}}}, {EqS, {"eq_s", {}}},
        {EqB, {"eq_b", {}}}, {EqI, {"eq_i", {}}}, {EqD, {"eq_d", {}}}, {AEqS, {"aeq_s", {ARG_STR}}},
        {AEqB, {"aeq_b", {ARG_BOOL}}}, {AEqI, {"aeq_i", {ARG_INT}}}, {AEqD, {"aeq_d", {ARG_DBL}}},
        {Xor, {"xor", {}}}, {And, {"and", {}}}, {Or, {"or", {}}}, {AXor, {"axor", {ARG_BOOL}}},
        {AAnd, {"aand", {ARG_BOOL}}}, {AOr, {"aor", {ARG_BOOL}}}, {Not, {"not", {}}},
        {ResolveS, {"resolve_s", {ARG_STR}}}, {ResolveB, {"resolve_b", {ARG_STR}}},
        {ResolveI, {"resolve_i", {ARG_STR}}}, {ResolveD, {"resolve_d", {ARG_STR}}},
        {ResolveF, {"resolve_f", {ARG_STR}}}, {TResolveS, {"tresolve_s", {ARG_STR}}},
        {TResolveB, {"tresolve_b", {ARG_STR}}}, {TResolveI, {"tresolve_i", {ARG_STR}}},
        {TResolveD, {"tresolve_d", {ARG_STR}}}, {TResolveF, {"tresolve_f", {ARG_STR}}}, {AddI, {"add_i", {}}},
        {AddD, {"add_d", {}}}, {SubI, {"sub_i", {}}}, {SubD, {"sub_d", {}}}, {AAddI, {"aadd_i", {ARG_INT}}},
        {AAddD, {"aadd_d", {ARG_DBL}}}, {ASubI, {"asub_i", {ARG_INT}}}, {ASubD, {"asub_d", {ARG_DBL}}},
        {Jmp, {"jmp", {ARG_ADDR}}}, {Jz, {"jz", {ARG_ADDR}}}, {Jnz, {"jnz", {ARG_ADDR}}},
        {Call, {"call", {ARG_FN}}}, {Ret, {"ret", {}}}, {Lookup, {"lookup", {}}}, {TLookup, {"tlookup", {}}},
        {ALookup, {"alookup", {ARG_STR}}}, {NLookup, {"nlookup", {}}}, {ANLookup, {"anlookup", {ARG_STR}}},
    };
    return t;
}

const OpInfo* op_info(uint32_t op) {
    auto& t = op_table();
    auto it = t.find(op);
    return it == t.end() ? nullptr : &it->second;
}

static uint32_t arg_words(ArgKind a) { return (a == ARG_INT || a == ARG_DBL) ? 2 : 1; }

uint32_t op_words(uint32_t op) {
    const OpInfo* i = op_info(op);
    if (!i) return 1;
    uint32_t n = 1;
    for (ArgKind a : i->args) n += arg_words(a);
    return n;
}

uint32_t StringTable::add(const std::string& s) {
    auto it = ids_.find(s);
    if (it != ids_.end()) return it->second;
    uint32_t id = (uint32_t)strs_.size();
    ids_.emplace(s, id);
    strs_.push_back(s);
    return id;
}

uint32_t StringTable::try_id(const std::string& s) const {
    auto it = ids_.find(s);
    return it == ids_.end() ? 0 : it->second;
}

bool IlProgram::add_function(const std::string& name, const std::vector<uint8_t>& params, uint8_t ret,
                             const std::vector<uint32_t>& body, std::string* err) {
    code.push_back(Halt);  // program.go:107: one Halt between bodies
    uint32_t start = (uint32_t)code.size();
    size_t n = body.size();
    for (size_t i = 0; i < n;) {
        uint32_t op = body[i];
        const OpInfo* inf = op_info(op);
        if (!inf || i + op_words(op) > n) {
            *err = "opcode requires more arguments than are present in the body";
            return false;
        }
        code.push_back(op);
        i++;
        for (ArgKind a : inf->args)
            for (uint32_t j = 0; j < arg_words(a); j++, i++) code.push_back(a == ARG_ADDR ? body[i] + start : body[i]);
    }
    IlFunction f;
    f.id = strings.add(name);
    f.address = start;
    f.length = (uint32_t)n;
    f.params = params;
    f.ret = ret;
    functions[f.id] = f;
    return true;
}

const IlFunction* IlProgram::get(const std::string& name) const {
    uint32_t id = strings.try_id(name);
    if (!id) return nullptr;
    auto it = functions.find(id);
    return it == functions.end() ? nullptr : &it->second;
}

namespace {

// il.Builder (mixer/pkg/il/builder.go)
class Builder {
  public:
    explicit Builder(StringTable* s) : s_(s) {}
    void op0(uint32_t op) { body.push_back(op); }
    void op1(uint32_t op, uint32_t a) {
        body.push_back(op);
        body.push_back(a);
    }
    void op2(uint32_t op, uint32_t a, uint32_t b) {
        body.push_back(op);
        body.push_back(a);
        body.push_back(b);
    }
    uint32_t id(const std::string& s) { return s_->add(s); }
    int label() {
        // Label names only matter for text output, which renumbers them; ids suffice here.
        int l = (int)pos_.size();
        pos_.push_back(-1);
        return l;
    }
    void set(int l) {
        pos_[l] = (int)body.size();
        for (auto& f : fix_)
            if (f.first == l) body[f.second] = (uint32_t)pos_[l];
    }
    void jump(uint32_t op, int l) {
        op1(op, pos_[l] > 0 ? (uint32_t)pos_[l] : 0);
        if (pos_[l] <= 0) fix_.push_back({l, body.size() - 1});
    }
    std::vector<uint32_t> body;

  private:
    StringTable* s_;
    std::vector<int> pos_;
    std::vector<std::pair<int, size_t>> fix_;
};

uint8_t to_il(int32_t t, bool* ok) {
    *ok = true;
    switch (t) {
    case VT_STRING: return IL_STRING;
    case VT_BOOL: return IL_BOOL;
    case VT_INT64: return IL_INTEGER;
    case VT_DURATION: return IL_DURATION;
    case VT_DOUBLE: return IL_DOUBLE;
    case VT_STRING_MAP: case VT_IP_ADDRESS: case VT_EMAIL_ADDRESS: case VT_DNS_NAME: case VT_URI:
    case VT_TIMESTAMP: return IL_INTERFACE;
    default: *ok = false; return IL_UNKNOWN;
    }
}

struct Panic {
    std::string msg;
};

// compiler.go generator
class Generator {
  public:
    Generator(IlProgram* p, const Vocabulary& v, const FuncMap& f) : b_(&p->strings), v_(v), f_(f) {}

    std::string err;
    Builder b_;

    uint8_t il_of(int32_t vt) {
        bool ok;
        uint8_t t = to_il(vt, &ok);
        if (!ok) fail(std::string("unhandled expression type: '") + value_type_name(vt) + "'");
        return t;
    }

    void fail(const std::string& m) {
        if (err.empty()) err = "internal compiler error -- " + m;
    }

    int32_t vtype(const Expr& e) {
        int32_t t = VT_UNSPECIFIED;
        std::string ignored;
        bool pan;
        eval_type(e, v_, f_, &t, &ignored, &pan);
        return t;
    }

    void gen(const Expr& e, int depth, bool jmp_mode, int label) {
        switch (e.kind) {
        case Expr::CONST: gen_const(e.c, jmp_mode, label); break;
        case Expr::VAR: gen_var(e.var, jmp_mode, label); break;
        case Expr::FN: gen_fn(e, depth, jmp_mode, label); break;
        default: fail("unexpected expression type encountered."); break;
        }
    }

    void gen_var(const std::string& name, bool jmp, int label) {
        int32_t vt = v_.at(name);
        uint8_t t = il_of(vt);
        uint32_t plain, tried;
        switch (t) {
        case IL_INTEGER: case IL_DURATION: plain = ResolveI; tried = TResolveI; break;
        case IL_STRING: plain = ResolveS; tried = TResolveS; break;
        case IL_BOOL: plain = ResolveB; tried = TResolveB; break;
        case IL_DOUBLE: plain = ResolveD; tried = TResolveD; break;
        case IL_INTERFACE: plain = ResolveF; tried = TResolveF; break;
        default: fail(std::string("unrecognized variable type: '") + value_type_name(vt) + "'"); return;
        }
        if (!jmp) {
            b_.op1(plain, b_.id(name));
        } else {
            b_.op1(tried, b_.id(name));
            b_.jump(Jnz, label);
        }
    }

    void gen_fn(const Expr& f, int depth, bool jmp, int label) {
        if (f.fn == "EQ") gen_eq(f, depth);
        else if (f.fn == "NEQ") {
            gen_eq(f, depth + 1);
            b_.op0(Not);
        } else if (f.fn == "LOR") gen_lor(f, depth);
        else if (f.fn == "LAND") gen_land(f, depth);
        else if (f.fn == "INDEX") gen_index(f, depth, jmp, label);
        else if (f.fn == "OR") gen_or(f, depth, jmp, label);
        else {
            if (f.target) gen(*f.target, depth, false, -1);
            for (auto& a : f.args) gen(*a, depth, false, -1);
            b_.op1(Call, b_.id(f.fn));
        }
    }

    void gen_eq(const Expr& f, int depth) {
        int32_t vt0 = vtype(*f.args[0]);
        uint8_t t = il_of(vt0);
        gen(*f.args[0], depth + 1, false, -1);
        const Constant* k = f.args[1]->kind == Expr::CONST ? &f.args[1]->c : nullptr;
        if (!k) gen(*f.args[1], depth + 1, false, -1);
        switch (t) {
        case IL_BOOL:
            if (k) {
                if (k->type != VT_BOOL) throw Panic{"interface conversion: interface {} is not bool"};
                b_.op1(AEqB, k->b ? 1 : 0);
            } else b_.op0(EqB);
            break;
        case IL_STRING:
            if (k) {
                if (k->type != VT_STRING) throw Panic{"interface conversion: interface {} is not string"};
                b_.op1(AEqS, b_.id(k->s));
            } else b_.op0(EqS);
            break;
        case IL_INTEGER:
            if (k) {
                if (k->type != VT_INT64) throw Panic{"interface conversion: interface {} is not int64"};
                b_.op2(AEqI, (uint32_t)((uint64_t)k->i & 0xFFFFFFFFu), (uint32_t)((uint64_t)k->i >> 32));
            } else b_.op0(EqI);
            break;
        case IL_DOUBLE:
            if (k) {
                if (k->type != VT_DOUBLE) throw Panic{"interface conversion: interface {} is not float64"};
                uint64_t u;
                memcpy(&u, &k->d, 8);
                b_.op2(AEqD, (uint32_t)(u & 0xFFFFFFFFu), (uint32_t)(u >> 32));
            } else b_.op0(EqD);
            break;
        case IL_INTERFACE:
            if (vt0 == VT_IP_ADDRESS) b_.op1(Call, b_.id("ip_equal"));
            else if (vt0 == VT_TIMESTAMP) b_.op1(Call, b_.id("timestamp_equal"));
            else fail(std::string("equality for type not yet implemented: ") + il_type_name(t));
            break;
        default:
            fail(std::string("equality for type not yet implemented: ") + il_type_name(t));
        }
    }

    void gen_lor(const Expr& f, int depth) {
        gen(*f.args[0], depth + 1, false, -1);
        int lr = b_.label(), le = b_.label();
        b_.jump(Jz, lr);
        b_.op1(APushB, 1);
        if (depth == 0) b_.op0(Ret);
        else b_.jump(Jmp, le);
        b_.set(lr);
        gen(*f.args[1], depth + 1, false, -1);
        if (depth != 0) b_.set(le);
    }

    void gen_land(const Expr& f, int depth) {
        int lf = b_.label(), le = b_.label();
        for (size_t i = 0; i < f.args.size(); i++) {
            gen(*f.args[i], depth + 1, false, -1);
            if (i + 1 < f.args.size()) b_.jump(Jz, lf);
            else b_.jump(Jmp, le);
        }
        b_.set(lf);
        b_.op1(APushB, 0);
        b_.set(le);
    }

    const std::string& const_string(const Expr& e) {
        if (e.c.type != VT_STRING) throw Panic{"interface conversion: interface {} is not string"};
        return e.c.s;
    }

    void gen_index(const Expr& f, int depth, bool jmp, int label) {
        if (!jmp) {
            gen(*f.args[0], depth + 1, false, -1);
            if (f.args[1]->kind == Expr::CONST) {
                b_.op1(ANLookup, b_.id(const_string(*f.args[1])));
            } else {
                gen(*f.args[1], depth + 1, false, -1);
                b_.op0(NLookup);
            }
            return;
        }
        int lend = b_.label(), ltr = b_.label();
        gen(*f.args[0], depth + 1, true, ltr);
        b_.jump(Jmp, lend);
        b_.set(ltr);
        if (f.args[1]->kind == Expr::CONST) {
            b_.op1(APushS, b_.id(const_string(*f.args[1])));
        } else {
            int lar = b_.label();
            gen(*f.args[1], depth + 1, true, lar);
            b_.jump(Jmp, lend);
            b_.set(lar);
        }
        b_.op0(TLookup);
        b_.jump(Jnz, label);
        b_.set(lend);
    }

    void gen_or(const Expr& f, int depth, bool jmp, int label) {
        if (!jmp) {
            int lend = b_.label();
            gen(*f.args[0], depth + 1, true, lend);
            if (f.args[1]->kind == Expr::FN && f.args[1]->fn == "OR") gen(*f.args[1], depth + 1, true, lend);
            else gen(*f.args[1], depth + 1, false, -1);
            b_.set(lend);
        } else {
            gen(*f.args[0], depth + 1, true, label);
            gen(*f.args[1], depth + 1, true, label);
        }
    }

    void gen_const(const Constant& c, bool jmp, int label) {
        switch (c.type) {
        case VT_STRING: b_.op1(APushS, b_.id(c.s)); break;
        case VT_BOOL: b_.op1(APushB, c.b ? 1 : 0); break;
        case VT_INT64: case VT_DURATION:
            b_.op2(APushI, (uint32_t)((uint64_t)c.i & 0xFFFFFFFFu), (uint32_t)((uint64_t)c.i >> 32));
            break;
        case VT_DOUBLE: {
            uint64_t u;
            memcpy(&u, &c.d, 8);
            b_.op2(APushD, (uint32_t)(u & 0xFFFFFFFFu), (uint32_t)(u >> 32));
            break;
        }
        default: fail(std::string("unhandled constant type: ") + value_type_name(c.type));
        }
        if (jmp) b_.jump(Jmp, label);
    }

  private:
    const Vocabulary& v_;
    const FuncMap& f_;
};

}  // namespace

void compile_rule(const std::string& text, const Vocabulary& vocab, const FuncMap& fmap, CompiledRule* out) {
    std::string err;
    ExprP e = parse_expression(text, &err);
    if (!e) {
        out->status = CompiledRule::PARSE_ERROR;
        out->error = err;
        return;
    }
    int32_t vt;
    bool panicked = false;
    if (!eval_type(*e, vocab, fmap, &vt, &err, &panicked)) {
        out->status = panicked ? CompiledRule::COMPILE_PANIC : CompiledRule::TYPE_ERROR;
        out->error = err;
        return;
    }
    out->value_type = vt;
    Generator g(&out->program, vocab, fmap);
    try {
        uint8_t ret = g.il_of(vt);
        g.gen(*e, 0, false, -1);
        if (!g.err.empty()) {
            out->status = CompiledRule::COMPILE_ERROR;
            out->error = g.err;
            return;
        }
        g.b_.op0(Ret);
        if (!out->program.add_function("eval", {}, ret, g.b_.body, &err)) {
            out->status = CompiledRule::COMPILE_ERROR;
            out->error = err;
            return;
        }
    } catch (Panic& p) {
        out->status = CompiledRule::COMPILE_PANIC;
        out->error = p.msg;
        return;
    }
    out->status = CompiledRule::OK;
}

static std::string fmt_f(double d) {
    if (std::isnan(d)) return "NaN";
    if (std::isinf(d)) return d > 0 ? "+Inf" : "-Inf";
    char b[512];
    snprintf(b, sizeof b, "%f", d);
    return b;
}

std::string write_il_text(const IlProgram& p) {
    std::vector<std::string> names;
    for (auto& kv : p.functions) names.push_back(p.strings.get(kv.first));
    std::sort(names.begin(), names.end());
    std::string out;
    for (auto& name : names) {
        const IlFunction* f = p.get(name);
        std::map<uint32_t, int> labels;
        int next = 0;
        // write.go:49-60: one word per argument (the second word of int/double args is re-read)
        for (uint32_t i = f->address; i < f->address + f->length; i++) {
            const OpInfo* inf = op_info(p.code[i]);
            if (!inf) continue;
            for (ArgKind a : inf->args) {
                i++;
                if (a == ARG_ADDR && !labels.count(p.code[i])) labels[p.code[i]] = next++;
            }
        }
        out += "fn " + name + "(";
        for (size_t k = 0; k < f->params.size(); k++) out += (k ? " " : "") + std::string(il_type_name(f->params[k]));
        out += ") " + std::string(il_type_name(f->ret)) + "\n";
        for (uint32_t i = f->address; i < f->address + f->length; i++) {
            auto lit = labels.find(i);
            if (lit != labels.end()) out += "L" + std::to_string(lit->second) + ":\n";
            const OpInfo* inf = op_info(p.code[i]);
            out += "  " + std::string(inf ? inf->keyword : "");
            if (inf) {
                for (ArgKind a : inf->args) {
                    out += " ";
                    uint32_t v = p.code[++i];
                    switch (a) {
                    case ARG_STR: {
                        std::string s = p.strings.get(v), e;
                        for (char c : s) {
                            if (c == '"') e += "\\\"";
                            else e += c;
                        }
                        out += "\"" + e + "\"";
                        break;
                    }
                    case ARG_ADDR: out += "L" + std::to_string(labels[v]); break;
                    case ARG_FN: out += p.strings.get(v); break;
                    case ARG_REG: out += "r" + std::to_string(v); break;
                    case ARG_INT: {
                        uint32_t hi = p.code[++i];
                        out += std::to_string((int64_t)((uint64_t)v | ((uint64_t)hi << 32)));
                        break;
                    }
                    case ARG_DBL: {
                        uint32_t hi = p.code[++i];
                        uint64_t u = (uint64_t)v | ((uint64_t)hi << 32);
                        double d;
                        memcpy(&d, &u, 8);
                        out += fmt_f(d);
                        break;
                    }
                    case ARG_BOOL: out += v ? "true" : "false"; break;
                    }
                }
            }
            out += "\n";
        }
        out += "end\n\n";
    }
    return out;
}

}  // namespace mxp
