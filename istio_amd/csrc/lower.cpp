// lower.cpp -- see lower.h.
//
// Shape-specialised lowering.  The reference VM addresses its operand stack top-relatively, and the
// reference compiler sometimes reaches a label with different stack contents on different paths
// (e.g. `ar[as] | "foo"` leaves the map `ar` behind when `as` is missing; an OR whose left operand
// ignores nmJmpOnValue leaves an extra value).  To give every stack slot a static register we lower
// each (IL address, incoming stack shape) pair -- a *context* -- separately: a label reached with two
// shapes gets two copies of the code that follows it, each with its own exact layout, so garbage
// below the top is modelled exactly as the reference sees it.  Contexts are emitted in IL-address
// order, which keeps every VM jump forward.
#include "lower.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>

#include "goutil.h"
#include "vmopt.h"
#include "../../include/mxp_batch.h"

namespace mxp {
namespace {

enum Cls : uint8_t { C_S = W_S, C_B = W_B, C_I = W_I, C_D = W_D, C_F = W_F };

constexpr size_t kMaxVmCode = 4096;
constexpr size_t kMaxContexts = 512;

struct Slot {
    Cls cls;
    bool konst = false;
    uint64_t kval = 0;   // register value of the constant
    std::string ktext;   // text of a constant string
    std::string attr;    // attribute the slot was resolved from (resolve_f), for fusion
};

struct State {
    std::vector<Slot> st;
    int words = 0;
    int heap = 0;
};

std::string signature(const State& s) {
    std::string sig;
    for (const Slot& x : s.st) sig.push_back((char)('0' + x.cls));
    return sig;
}

int words_of(Cls c) { return (c == C_I || c == C_D) ? 2 : 1; }

struct Irregular {
    std::string why;
};

// merge two states of the same signature
void merge_into(State& dst, const State& src) {
    for (size_t i = 0; i < dst.st.size(); i++) {
        Slot& a = dst.st[i];
        const Slot& b = src.st[i];
        if (!(a.konst && b.konst && a.kval == b.kval && a.ktext == b.ktext)) {
            a.konst = false;
            a.ktext.clear();
        }
        if (a.attr != b.attr) a.attr.clear();
    }
    dst.heap = std::max(dst.heap, src.heap);
}

struct Ctx {
    State state;
    std::vector<size_t> sources;  // VM instructions whose jump target (z) is this context's block
    bool has_fallthrough = false;
};

class Lowerer {
  public:
    Lowerer(const IlProgram& p, LowerTables* t) : p_(p), t_(t) {}

    LoweredRule run() {
        LoweredRule out;
        const IlFunction* f = p_.get("eval");
        if (!f) {
            out.why = "no eval function";
            return out;
        }
        fn_ret_ = f->ret;
        try {
            body(*f);
            finish();
        } catch (Irregular& ir) {
            out.why = ir.why;
            return out;
        }
        out.ok = true;
        out.code = code_;
        out.nregs = maxregs_;
        out.uses_ipof = ipof_;
        out.uses_rxof = rxof_;
        out.uses_tsof = tsof_;
        out.uses_strings = strings_;
        out.uses_maps = maps_;
        return out;
    }

  private:
    // ------------------------------------------------------------------ emission helpers
    size_t emit(uint8_t op, int d, int a, int b, uint32_t x, uint32_t y, uint32_t z) {
        if (code_.size() >= kMaxVmCode) throw Irregular{"lowered program too large"};
        mxp_vm_ins i;
        i.op = op;
        i.d = (uint8_t)d;
        i.a = (uint8_t)a;
        i.b = (uint8_t)b;
        i.x = x;
        i.y = y;
        i.z = z;
        code_.push_back(i);
        return code_.size() - 1;
    }

    int top() const { return (int)cur_.st.size() - 1; }

    Slot& push(Cls c) {
        Slot s;
        s.cls = c;
        cur_.st.push_back(s);
        cur_.words += words_of(c);
        if ((int)cur_.st.size() > MXP_VM_MAXREG) throw Irregular{"more than MXP_VM_MAXREG live stack slots"};
        // the reference checks sp against 64 words before each push; keep 3 words of slack
        if (cur_.words + 3 > 64) throw Irregular{"reference stack could overflow"};
        maxregs_ = std::max<uint32_t>(maxregs_, (uint32_t)cur_.st.size());
        return cur_.st.back();
    }

    Slot pop_raw() {
        if (cur_.st.empty()) throw Irregular{"stack underflow"};
        Slot s = cur_.st.back();
        cur_.st.pop_back();
        cur_.words -= words_of(s.cls);
        return s;
    }

    // Pop an operand the reference reads as `want`.  A string read from a slot that holds an
    // interface value is Go's `heap[i].(string)` (emulated by VM_FTOS); interface reads of a string
    // slot just see the string.  Other mismatches would reinterpret raw words: not lowered.
    Slot pop(Cls want) {
        if (cur_.st.empty()) throw Irregular{"stack underflow"};
        Slot s = cur_.st.back();
        int reg = top();
        if (s.cls != want) {
            if (want == C_S && s.cls == C_F) {
                emit(VM_FTOS, reg, reg, 0, 0, 0, 0);
                s.cls = C_S;
                s.konst = false;
            } else if (want == C_F && s.cls == C_S) {
                emit(VM_STOF, reg, reg, 0, 0, 0, 0);
                s.cls = C_F;
                s.konst = false;
            } else {
                throw Irregular{"operand type mismatch"};
            }
        }
        pop_raw();
        return s;
    }

    // The reference checks operand availability before touching anything (interpreterRun.go, e.g.
    // :247 `if sp < 2 goto STACK_UNDERFLOW`).  Paths of an OR chain can reach a consumer with too few
    // values; those paths raise "stack underflow" there.
    bool need(size_t k) {
        if (cur_.st.size() >= k) return true;
        emit(VM_ERR, 0, 0, 0, 0, ERR_UNDERFLOW, 0);
        live_ = false;
        return false;
    }

    void alloc() {
        cur_.heap++;
        if (cur_.heap > 63) throw Irregular{"reference heap could overflow"};
    }

    void add_edge(uint32_t target, const State& s, size_t vm_src, bool fallthrough) {
        if (target <= at_ && !fallthrough) throw Irregular{"backward jump"};
        std::string sig = signature(s);
        auto& bucket = pending_[target];
        auto it = bucket.find(sig);
        if (it == bucket.end()) {
            if (++ncontexts_ > kMaxContexts) throw Irregular{"too many stack-shape contexts"};
            Ctx c;
            c.state = s;
            it = bucket.emplace(sig, c).first;
            order_[target].push_back(sig);
        } else {
            merge_into(it->second.state, s);
        }
        if (fallthrough) it->second.has_fallthrough = true;
        else it->second.sources.push_back(vm_src);
    }

    std::string str(uint32_t id) const { return p_.strings.get(id); }

    static Cls want_of_resolve(uint32_t op) {
        switch (op) {
        case ResolveS: case TResolveS: return C_S;
        case ResolveB: case TResolveB: return C_B;
        case ResolveI: case TResolveI: return C_I;
        case ResolveD: case TResolveD: return C_D;
        default: return C_F;
        }
    }

    bool is_target(uint32_t addr) const { return jump_targets_.count(addr) != 0; }

    // ------------------------------------------------------------------ driver
    void body(const IlFunction& f) {
        const auto& c = p_.code;
        start_ = f.address;
        end_ = f.address + f.length;
        // every address some jump names (fused pairs must not be split by a jump)
        for (uint32_t a = start_; a < end_;) {
            const OpInfo* inf = op_info(c[a]);
            if (!inf) throw Irregular{"unknown opcode"};
            if (c[a] == Jmp || c[a] == Jz || c[a] == Jnz) jump_targets_.insert(c[a + 1]);
            a += op_words(c[a]);
        }
        Ctx entry;
        entry.has_fallthrough = true;
        pending_[start_].emplace("", entry);
        order_[start_].push_back("");
        ncontexts_ = 1;
        // A fall-through edge into a context is honoured only if that context's block is emitted
        // immediately after its predecessor; otherwise an explicit VM_JMP is appended (prev_ctx_).
        for (uint32_t a = start_; a < end_;) {
            uint32_t sz = op_words(c[a]);
            auto pit = pending_.find(a);
            if (pit != pending_.end()) {
                for (const std::string& sig : order_[a]) {
                    Ctx& cx = pit->second.at(sig);
                    block(a, cx);
                }
                pending_.erase(pit);
            }
            a += sz;
        }
        if (!pending_.empty()) throw Irregular{"jump outside function"};
    }

    // Lower the instruction(s) at `a` for one incoming context.
    void block(uint32_t a, Ctx& cx) {
        at_ = a;
        cur_ = cx.state;
        size_t start_index = code_.size();
        // patch jumps into this block
        for (size_t s : cx.sources) code_[s].z = (uint32_t)start_index;
        for (size_t s : pending_ft_jumps_[{a, signature(cur_)}]) code_[s].z = (uint32_t)start_index;
        wake_.insert(start_index);
        uint32_t next = lower_one(a);
        // fall-through successor
        if (live_) {
            State s = cur_;
            add_edge(next, s, 0, true);
            // emit an explicit jump; removed later when it lands on the next instruction
            size_t j = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
            pending_ft_jumps_[{next, signature(s)}].push_back(j);
        }
        if (code_.size() == start_index) emit(VM_NOP, 0, 0, 0, 0, 0, 0);
    }

    // Lowers the instruction at `a` (plus a fused successor) from cur_; returns the next address.
    // Sets live_ = false when control does not fall through.
    uint32_t lower_one(uint32_t a) {
        const auto& c = p_.code;
        uint32_t op = c[a];
        const OpInfo* inf = op_info(op);
        uint32_t next = a + op_words(op);
        live_ = true;
        switch (op) {
        case ResolveS: case ResolveB: case ResolveI: case ResolveD: case ResolveF: {
            Cls w = want_of_resolve(op);
            std::string attr = str(c[a + 1]);
            // fuse `resolve_f <map>; anlookup "k"` into a virtual column
            if (op == ResolveF && next < end_ && c[next] == ANLookup && !is_target(next) &&
                t_->attr_type(attr) == VT_STRING_MAP) {
                std::string key = str(c[next + 1]);
                push(C_S);
                alloc();
                alloc();
                emit(VM_VCOL, top(), 0, 0, t_->vcolumn(attr, key), 0, t_->intern_string(attr));
                return next + op_words(ANLookup);
            }
            Slot& s = push(w);
            s.attr = attr;
            if (w == C_S || w == C_F) alloc();
            emit(VM_RES, top(), 0, 0, t_->column(attr), w, t_->intern_string(attr));
            return next;
        }
        case TResolveS: case TResolveB: case TResolveI: case TResolveD: case TResolveF: {
            if (next >= end_ || c[next] != Jnz || is_target(next)) throw Irregular{"tresolve not followed by a private jnz"};
            Cls w = want_of_resolve(op);
            std::string attr = str(c[a + 1]);
            State saved = cur_;
            push(w).attr = attr;
            if (w == C_S || w == C_F) alloc();
            State found = cur_;
            int reg = top();
            cur_ = saved;
            size_t j = emit(VM_TRES, reg, 0, 0, t_->column(attr), w, 0);
            add_edge(c[next + 1], found, j, false);
            return next + op_words(Jnz);
        }
        case APushS: {
            Slot& s = push(C_S);
            alloc();
            std::string txt = str(c[a + 1]);
            uint32_t id = t_->intern_string(txt);
            s.konst = true;
            s.kval = id;
            s.ktext = txt;
            emit(VM_CONST, top(), 0, 0, 0, id, 0);
            return next;
        }
        case APushB: {
            Slot& s = push(C_B);
            s.konst = true;
            s.kval = c[a + 1];
            emit(VM_CONST, top(), 0, 0, 0, c[a + 1], 0);
            return next;
        }
        case APushI: case APushD: {
            uint64_t v = (uint64_t)c[a + 1] | ((uint64_t)c[a + 2] << 32);
            Slot& s = push(op == APushI ? C_I : C_D);
            s.konst = true;
            s.kval = v;
            emit(VM_CONST, top(), 0, 0, 0, (uint32_t)v, (uint32_t)(v >> 32));
            return next;
        }
        case EqS: case EqB: case EqI: case EqD: {
            if (!need(2)) return next;
            Cls k = op == EqS ? C_S : op == EqB ? C_B : op == EqI ? C_I : C_D;
            pop(k);
            pop(k);
            push(C_B);
            emit(VM_EQ, top(), top(), top() + 1, 0, 0, 0);
            return next;
        }
        case AEqS: {
            if (!need(1)) return next;
            pop(C_S);
            push(C_B);
            emit(VM_EQK, top(), top(), 0, 0, t_->intern_string(str(c[a + 1])), 0);
            return next;
        }
        case AEqB: case AEqI: case AEqD: {
            if (!need(1)) return next;
            Cls k = op == AEqB ? C_B : op == AEqI ? C_I : C_D;
            pop(k);
            push(C_B);
            emit(VM_EQK, top(), top(), 0, 0, c[a + 1], op == AEqB ? 0 : c[a + 2]);
            return next;
        }
        case Not:
            if (!need(1)) return next;
            pop(C_B);
            push(C_B);
            emit(VM_NOT, top(), top(), 0, 0, 0, 0);
            return next;
        case And: case Or: case Xor:
            if (!need(2)) return next;
            pop(C_B);
            pop(C_B);
            push(C_B);
            emit(VM_LOGIC, top(), top(), top() + 1, 0, op == And ? 0 : op == Or ? 1 : 2, 0);
            return next;
        case AAnd: case AOr: case AXor:
            if (!need(1)) return next;
            pop(C_B);
            push(C_B);
            emit(VM_LOGICK, top(), top(), 0, c[a + 1], op == AAnd ? 0 : op == AOr ? 1 : 2, 0);
            return next;
        case Jz: case Jnz: {
            if (!need(1)) return next;
            pop(C_B);
            size_t j = emit(op == Jz ? VM_JZ : VM_JNZ, 0, top() + 1, 0, 0, 0, 0);
            add_edge(c[a + 1], cur_, j, false);
            return next;
        }
        case Jmp: {
            size_t j = emit(VM_JMP, 0, 0, 0, 0, 0, 0);
            add_edge(c[a + 1], cur_, j, false);
            live_ = false;
            return next;
        }
        case Ret: {
            Cls want = fn_ret_ == IL_BOOL ? C_B : fn_ret_ == IL_STRING ? C_S
                       : (fn_ret_ == IL_INTEGER || fn_ret_ == IL_DURATION) ? C_I
                       : fn_ret_ == IL_DOUBLE ? C_D : C_F;
            if (!need(1)) return next;
            Slot s = pop(want);
            (void)s;
            emit(VM_RET, 0, top() + 1, 0, 0, fn_ret_ == IL_BOOL ? 1 : 0, fn_ret_);
            live_ = false;
            return next;
        }
        case ANLookup: case ALookup: {
            if (!need(1)) return next;
            pop(C_F);
            push(C_S);
            alloc();
            maps_ = true;
            emit(VM_LOOKUPK, top(), top(), 0, t_->intern_string(str(c[a + 1])), op == ANLookup ? LK_N : LK_ERR, 0);
            return next;
        }
        case NLookup: case Lookup: {
            if (!need(2)) return next;
            pop(C_S);
            pop(C_F);
            push(C_S);
            alloc();
            maps_ = true;
            emit(VM_LOOKUP, top(), top(), top() + 1, 0, op == NLookup ? LK_N : LK_ERR, 0);
            return next;
        }
        case TLookup: {
            if (next >= end_ || c[next] != Jnz || is_target(next)) throw Irregular{"tlookup not followed by a private jnz"};
            if (!need(2)) return next + op_words(Jnz);
            pop(C_S);
            pop(C_F);
            State saved = cur_;
            push(C_S);
            alloc();
            State found = cur_;
            int reg = top();
            cur_ = saved;
            maps_ = true;
            size_t j = emit(VM_LOOKUP, reg, reg, reg + 1, 0, LK_TRY, 0);
            add_edge(c[next + 1], found, j, false);
            return next + op_words(Jnz);
        }
        case Call:
            call(str(c[a + 1]));
            return next;
        default:
            throw Irregular{std::string("opcode not lowered: ") + (inf ? inf->keyword : "?")};
        }
    }

    void call(const std::string& name) {
        if (name == "ip" || name == "timestamp") {
            if (!need(1)) return;
            Slot s = pop(C_S);
            push(C_F);
            alloc();
            bool ip = name == "ip";
            if (s.konst) {
                const std::string& txt = s.ktext;
                if (ip) {
                    uint8_t b[16];
                    if (go_parse_ip((const uint8_t*)txt.data(), txt.size(), b)) {
                        uint64_t h = MXP_FH(MXP_BYTES, t_->intern_bytes(std::string((const char*)b, 16)));
                        emit(VM_CONST, top(), 0, 0, 0, (uint32_t)h, (uint32_t)(h >> 32));
                    } else {
                        emit(VM_ERR, top(), 0, 0, 0, ERR_IP, (uint32_t)s.kval);
                    }
                } else {
                    int64_t sec;
                    int32_t ns;
                    if (go_parse_rfc3339((const uint8_t*)txt.data(), txt.size(), &sec, &ns)) {
                        uint64_t h = MXP_FH(MXP_TIMESTAMP, t_->intern_time(sec, ns));
                        emit(VM_CONST, top(), 0, 0, 0, (uint32_t)h, (uint32_t)(h >> 32));
                    } else {
                        emit(VM_ERR, top(), 0, 0, 0, ERR_TS, (uint32_t)s.kval);
                    }
                }
            } else {
                if (ip) ipof_ = true;
                else tsof_ = true;
                emit(ip ? VM_IPOF : VM_TSOF, top(), top(), 0, 0, 0, 0);
            }
            return;
        }
        if (name == "ip_equal" || name == "timestamp_equal") {
            if (!need(2)) return;
            pop(C_F);
            pop(C_F);
            push(C_B);
            emit(name == "ip_equal" ? VM_IPEQ : VM_TSEQ, top(), top(), top() + 1, 0, 0, 0);
            return;
        }
        int fn = name == "match" ? SF_MATCH : name == "startsWith" ? SF_STARTS : name == "endsWith" ? SF_ENDS
                 : name == "matches" ? SF_REGEX : -1;
        if (fn < 0) throw Irregular{"call of unknown function " + name};
        if (!need(2)) return;
        Slot b = pop(C_S);
        Slot a = pop(C_S);
        push(C_B);
        if (fn == SF_REGEX) {  // externMatches(pattern = receiver, subject): regexp.MatchString
            if (a.konst) {
                std::string e;
                const int32_t id = t_->regex_const(a.ktext, &e);
                if (id == -2) throw Irregular{"regexp: " + e};
                if (id < 0) {
                    emit(VM_ERR, top(), 0, 0, 0, ERR_REGEX, (uint32_t)a.kval);
                    return;
                }
                if (b.konst) {
                    emit(VM_CONST, top(), 0, 0, 0, t_->regex_const_match(id, b.ktext) ? 1 : 0, 0);
                    return;
                }
                strings_ = true;
                emit(VM_REGEX, top(), top() + 1, 0, (uint32_t)id, 0, 0);
                return;
            }
            // run-time pattern: only straight from a string attribute, whose values the packer compiles
            if (a.attr.empty() || a.cls != C_S) throw Irregular{"regexp pattern computed at run time"};
            t_->regex_column(t_->column(a.attr));
            strings_ = true;
            rxof_ = true;
            emit(VM_REGEXD, top(), top(), top() + 1, 0, 0, 0);
            return;
        }
        if (a.konst && b.konst) {
            const std::string& s = a.ktext;
            const std::string& q = b.ktext;
            bool r;
            if (fn == SF_STARTS) r = s.size() >= q.size() && s.compare(0, q.size(), q) == 0;
            else if (fn == SF_ENDS) r = s.size() >= q.size() && s.compare(s.size() - q.size(), q.size(), q) == 0;
            else if (!q.empty() && q.back() == '*')
                r = s.size() >= q.size() - 1 && s.compare(0, q.size() - 1, q, 0, q.size() - 1) == 0;
            else if (!q.empty() && q[0] == '*')
                r = s.size() >= q.size() - 1 && s.compare(s.size() - (q.size() - 1), q.size() - 1, q, 1, q.size() - 1) == 0;
            else r = s == q;
            emit(VM_CONST, top(), 0, 0, 0, r ? 1 : 0, 0);
            return;
        }
        strings_ = true;
        if (b.konst) emit(VM_STRFNK, top(), top(), 0, (uint32_t)b.kval, (uint32_t)fn, 0);
        else emit(VM_STRFN, top(), top(), top() + 1, 0, (uint32_t)fn, 0);
    }

    // Drop explicit fall-through jumps that land on the next instruction, renumber, set WAKE flags.
    void finish() {
        std::vector<uint32_t> newidx(code_.size() + 1, 0);
        std::vector<bool> keep(code_.size(), true);
        for (size_t i = 0; i < code_.size(); i++)
            if ((code_[i].op & 0x7F) == VM_JMP && code_[i].z == i + 1) keep[i] = false;
        uint32_t k = 0;
        for (size_t i = 0; i < code_.size(); i++) {
            newidx[i] = k;
            if (keep[i]) k++;
        }
        newidx[code_.size()] = k;
        std::vector<mxp_vm_ins> out;
        out.reserve(k);
        std::set<uint32_t> targets;
        for (size_t i = 0; i < code_.size(); i++) {
            if (!keep[i]) continue;
            mxp_vm_ins ins = code_[i];
            uint32_t op = ins.op & 0x7F;
            bool jumps = op == VM_JMP || op == VM_JZ || op == VM_JNZ || op == VM_TRES ||
                         (op == VM_LOOKUP && ins.y == LK_TRY) || (op == VM_LOOKUPK && ins.y == LK_TRY);
            if (jumps) {
                if (ins.z >= code_.size()) throw Irregular{"dangling jump"};
                ins.z = newidx[ins.z];
                targets.insert(ins.z);
            }
            out.push_back(ins);
        }
        for (uint32_t t : targets) {
            if (t >= out.size()) throw Irregular{"jump past end"};
            out[t].op |= MXP_VM_WAKE;
        }
        for (size_t i = 0; i < out.size(); i++) {
            uint32_t op = out[i].op & 0x7F;
            bool jumps = op == VM_JMP || op == VM_JZ || op == VM_JNZ || op == VM_TRES ||
                         (op == VM_LOOKUP && out[i].y == LK_TRY) || (op == VM_LOOKUPK && out[i].y == LK_TRY);
            if (jumps && out[i].z <= i) throw Irregular{"non-forward jump after layout"};
        }
        code_ = out;
        try {
            optimize_vm(code_);
        } catch (std::exception& e) {
            throw Irregular{e.what()};
        }
    }

    const IlProgram& p_;
    LowerTables* t_;
    uint8_t fn_ret_ = IL_BOOL;
    uint32_t start_ = 0, end_ = 0, at_ = 0;
    State cur_;
    bool live_ = true;
    std::map<uint32_t, std::map<std::string, Ctx>> pending_;
    std::map<uint32_t, std::vector<std::string>> order_;
    std::map<std::pair<uint32_t, std::string>, std::vector<size_t>> pending_ft_jumps_;
    std::set<uint32_t> jump_targets_;
    std::set<size_t> wake_;
    size_t ncontexts_ = 0;
    std::vector<mxp_vm_ins> code_;
    uint32_t maxregs_ = 0;
    bool ipof_ = false, tsof_ = false, strings_ = false, maps_ = false, rxof_ = false;
};

}  // namespace

LoweredRule lower_rule(const IlProgram& prog, LowerTables* tables) { return Lowerer(prog, tables).run(); }

std::string vm_disasm(const std::vector<mxp_vm_ins>& code) {
    static const char* names[] = {"nop", "res", "tres", "vcol", "const", "eq", "eqk", "not", "jz", "jnz", "jmp",
                                  "ret", "lookup", "lookupk", "strfn", "strfnk", "ipof", "tsof", "ipeq", "tseq",
                                  "err", "logic", "logick", "ftos", "stof", "jzret", "jnzret", "retk", "mov", "regex", "regexd", "regexr"};
    std::string o;
    char buf[160];
    for (size_t i = 0; i < code.size(); i++) {
        const mxp_vm_ins& c = code[i];
        unsigned op = c.op & 0x7F;
        snprintf(buf, sizeof buf, "%3zu%s %-7s d=%u a=%u b=%u x=%u y=%u z=%u\n", i, (c.op & MXP_VM_WAKE) ? "*" : " ",
                 op < sizeof(names) / sizeof(names[0]) ? names[op] : "?", c.d, c.a, c.b, c.x, c.y, c.z);
        o += buf;
    }
    return o;
}

}  // namespace mxp
